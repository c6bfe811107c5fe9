#!/bin/bash
# Round profile refresh on the GPU box (each GPU step under its own time limit
# via tools/gpu_run.sh, which stops the chain at a fault or time-out):
#   the bench line under the driver's exact command; bench lines per config,
#   xudp's slot layout and the in-place mode; rocprofv3 --kernel-trace --stats
#   per workload; separate FETCH_SIZE / WRITE_SIZE PMC passes per workload,
#   summarised into profiles-ready JSON (tools/pmc_summary.py, tied to the
#   library's SHA-256 prefix).
#   tools/profile_round.sh <outdir under gpurun_out>
set -eu
out="$1"; mkdir -p "gpurun_out/$out"
export TMPDIR=/tmp
SHA=$(python3 -c "import bench; print(bench.lib_sha16())")
B="python3 bench.py --no-cpu-baseline"
tools/gpu_run.sh $out/bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5
for c in 2 3 4 5; do
  tools/gpu_run.sh $out/bench_config$c 300 $B --config $c --steps 100
done
tools/gpu_run.sh $out/bench_config2_umem 300 $B --config 2 --layout umem --steps 100
tools/gpu_run.sh $out/bench_config2_inplace 300 $B --config 2 --steps 100 --flags inplace,iphdr
tools/gpu_run.sh $out/bench_config4_inplace 300 $B --config 4 --steps 100 --flags inplace
# name:bench args
WL="c2:--config 2|c3:--config 3|c4:--config 4|c5:--config 5|c2_inplace:--config 2 --flags inplace,iphdr|c4_inplace:--config 4 --flags inplace"
IFS='|' read -ra wls <<< "$WL"
for w in "${wls[@]}"; do
  n=${w%%:*}; a=${w#*:}
  tools/gpu_run.sh $out/stats_$n 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/$out/stats_$n -o run -- $B $a --steps 20 --warmup 5 --no-order-ab
done
for w in "${wls[@]}"; do
  n=${w%%:*}; a=${w#*:}
  P="$B $a --steps 10 --warmup 2 --no-graph --ramp-ms 0 --reps 1 --no-ceiling"
  tools/gpu_run.sh $out/fetch_$n 120 rocprofv3 --pmc FETCH_SIZE --output-format csv \
      -d gpurun_out/$out/fetch_$n -o run -- $P
  tools/gpu_run.sh $out/write_$n 120 rocprofv3 --pmc WRITE_SIZE --output-format csv \
      -d gpurun_out/$out/write_$n -o run -- $P
  cid=$(echo "$a" | sed -n 's/.*--config \([0-9]\).*/\1/p')
  fl=$(echo "$a" | grep -q "inplace,iphdr" && echo 0x3 || (echo "$a" | grep -q inplace && echo 0x1 || echo 0))
  alg=$(python3 -c "
import bench, libxudp_amd as X
cfg = dict(bench.CONFIGS[$cid], id=$cid)
desc, _ = X.gen_layout(cfg['n'], cfg['family'], cfg['pmin'], cfg['pmax'], seed=bench.SEED_BASE ^ $cid)
f = $fl
print(bench.alg_bytes_flags(desc, cfg['family'], f, not (f & X.F_INPLACE)))")
  python3 tools/pmc_summary.py --config $cid --flags $fl --lib-sha $SHA --alg-bytes $alg \
      --fetch "$(find gpurun_out/$out/fetch_$n -name "*counter_collection.csv" -print -quit)" \
      --write "$(find gpurun_out/$out/write_$n -name "*counter_collection.csv" -print -quit)" \
      --out gpurun_out/$out/pmc_$n.json > gpurun_out/$out/pmc_$n.log 2>&1 || true
done
