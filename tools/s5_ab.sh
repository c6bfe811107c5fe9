#!/bin/bash
# A/B: sparse fallback of the stream kernel at G = 8 (config 3 in xudp's
# slots), nontemporal receive-record stores
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/s5
for r in 1 2; do
  for v in cur sg8; do
    L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
    XCSUM_LIB=$L tools/gpu_run.sh s5/c3u_${v}_$r 200 python bench.py --config 3 --layout umem --steps 100 --warmup 5 --reps 3 --no-cpu-baseline --no-ceiling
    XCSUM_LIB=$L tools/gpu_run.sh s5/c3p_${v}_$r 200 python bench.py --config 3 --steps 100 --warmup 5 --reps 3 --no-cpu-baseline --no-ceiling
  done
done
ROUNDS=2 tools/ab_rx_libs.sh gpurun_out/s5/rx 2,4,5 auto ntrec
