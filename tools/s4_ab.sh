#!/bin/bash
# round-2 session-2 A/B call: config 5 first-row temporal loads / all temporal,
# receive kernel capped at 3 waves/SIMD, config 3 in xudp's slot layout sweep
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/s4
for r in 1 2; do
  for v in cur edget nt0; do
    L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
    XCSUM_LIB=$L tools/gpu_run.sh s4/c5_${v}_$r 200 python bench.py --config 5 --steps 10 --warmup 2 --reps 3 --no-cpu-baseline --no-ceiling
  done
done
for v in edget nt0; do
  XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so tools/gpu_run.sh s4/fetch5_$v 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/s4/fetch5_$v -o run -- python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline --no-graph --ramp-ms 0 --reps 1 --no-ceiling
done
ROUNDS=2 tools/ab_rx_libs.sh gpurun_out/s4/rx 2,4 auto rxw3
tools/gpu_run.sh s4/sweep3_umem 300 python tools/sweep.py --config 3 --layout umem --geoms "4,1,2;8,1,2;4,2,2;2,1,4" --bpc 0,2,4,8 --orders="-1,0;0,0;3,4;7,4" --rounds 3 --launches 20
