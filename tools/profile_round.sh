#!/bin/bash
# Round profile refresh on the GPU box (each GPU step under its own time limit
# via tools/gpu_run.sh, which stops the chain at a fault or time-out):
#   the bench line under the driver's exact command; bench lines per
#   workload; rocprofv3 --kernel-trace --stats per workload; separate
#   FETCH_SIZE / WRITE_SIZE PMC passes per workload, summarised into
#   profiles-ready JSON (tools/pmc_summary.py, keyed by the counted kernel's
#   code hash).
#   tools/profile_round.sh <outdir under gpurun_out>
# The --stats runs pass --no-calibrate --no-order-ab: every launch of the
# measured kernel in them is a timed-path launch (warm-up, clock ramp, timed
# repetitions, the parity pass), so the rocprofv3 mean is the timed kernel's
# own duration (the order A/B and calibration launches
# run the same kernel with other visiting orders).
set -eu
out="$1"; mkdir -p "gpurun_out/$out"
export TMPDIR=/tmp
SHA=$(python3 -c "import bench; print(bench.lib_sha16())")
B="python3 bench.py --no-cpu-baseline"
tools/gpu_run.sh $out/bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5
# name:bench args
WL="c2:--config 2|c3:--config 3|c4:--config 4|c5:--config 5|c2u:--config 2 --layout umem\
|c2_inplace:--config 2 --flags inplace,iphdr|c4_inplace:--config 4 --flags inplace\
|c2_iphdr_only:--config 2 --flags inplace,iphdr_only\
|c2u_iphdr_only:--config 2 --flags inplace,iphdr_only --layout umem"
IFS='|' read -ra wls <<< "${PROFILE_WL:-$WL}"
for w in "${wls[@]}"; do
  n=${w%%:*}; a=${w#*:}
  tools/gpu_run.sh $out/bench_$n 300 $B $a --steps 100
done
for w in "${wls[@]}"; do
  n=${w%%:*}; a=${w#*:}
  tools/gpu_run.sh $out/stats_$n 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/$out/stats_$n -o run -- $B $a --steps 20 --warmup 5 --no-order-ab \
      --no-calibrate
done
for w in "${wls[@]}"; do
  n=${w%%:*}; a=${w#*:}
  P="$B $a --steps 10 --warmup 2 --no-graph --ramp-ms 0 --reps 1 --no-ceiling --no-calibrate"
  tools/gpu_run.sh $out/fetch_$n 120 rocprofv3 --pmc FETCH_SIZE --output-format csv \
      -d gpurun_out/$out/fetch_$n -o run -- $P
  tools/gpu_run.sh $out/write_$n 120 rocprofv3 --pmc WRITE_SIZE --output-format csv \
      -d gpurun_out/$out/write_$n -o run -- $P
  # config, flags, layout and algorithmic bytes of the workload, as bench.py
  # computes them
  read -r cid fl lay alg <<< "$(python3 - $a <<'PY'
import argparse, sys
import bench, libxudp_amd as X
ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=2)
ap.add_argument("--flags", default="")
ap.add_argument("--layout", default="packed")
a, _ = ap.parse_known_args(sys.argv[1:])
f = bench.parse_flags(a.flags)
cfg = dict(bench.CONFIGS[a.config], id=a.config)
kw = dict(stride=4096, offset=322 if cfg["family"] == 6 else 342) if a.layout == "umem" else {}
desc, _ = X.gen_layout(cfg["n"], cfg["family"], cfg["pmin"], cfg["pmax"],
                       seed=bench.SEED_BASE ^ a.config, **kw)
with_out = not (f & X.F_INPLACE) or bool(f & X.F_VERIFY)
print(a.config, hex(f), a.layout, bench.alg_bytes_flags(desc, cfg["family"], f, with_out))
PY
)"
  python3 tools/pmc_summary.py --config $cid --flags $fl --layout $lay --lib-sha $SHA \
      --alg-bytes $alg \
      --fetch "$(find gpurun_out/$out/fetch_$n -name "*counter_collection.csv" -print -quit)" \
      --write "$(find gpurun_out/$out/write_$n -name "*counter_collection.csv" -print -quit)" \
      --out gpurun_out/$out/pmc_$n.json > gpurun_out/$out/pmc_$n.log 2>&1 || true
done
