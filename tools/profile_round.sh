#!/bin/bash
# Round profile refresh on the GPU box (each GPU step under its own timeout,
# stop at the first fault/timeout via tools/gpu_run.sh):
#   bench.py JSON per config (the driver's exact command for config 2),
#   rocprofv3 --kernel-trace --stats per config, separate FETCH_SIZE /
#   WRITE_SIZE PMC passes for configs 2 and 3.
#   tools/profile_round.sh <outdir under gpurun_out>
set -e
out="$1"; mkdir -p "gpurun_out/$out"
export TMPDIR=/tmp
tools/gpu_run.sh $out/bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5
for c in 2 3 4 5; do
  tools/gpu_run.sh $out/bench_config$c 300 python bench.py --config $c --steps 100 --no-cpu-baseline
done
tools/gpu_run.sh $out/bench_config2_umem 300 python bench.py --config 2 --layout umem --no-cpu-baseline
tools/gpu_run.sh $out/bench_config3_umem 300 python bench.py --config 3 --layout umem --no-cpu-baseline
for c in 2 3 4 5; do
  tools/gpu_run.sh $out/stats$c 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/$out/stats$c -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline
done
for c in 2 3; do
  tools/gpu_run.sh $out/fetch$c 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
      -d gpurun_out/$out/fetch$c -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-graph --ramp-ms 0 --reps 1 --no-ceiling
  tools/gpu_run.sh $out/write$c 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
      -d gpurun_out/$out/write$c -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-graph --ramp-ms 0 --reps 1 --no-ceiling
done
# receive kernels: every mode on configs 2, 4, 3, 5, and rocprofv3 stats of config 2
tools/gpu_run.sh $out/bench_rx 300 python tools/bench_rx.py --configs 2,4,3,5
tools/gpu_run.sh $out/rx_stats2 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/$out/rx_stats2 -o run -- python3 tools/bench_rx.py --configs 2 --reps 5
