#!/bin/bash
# full GPU suite on nontemporal receive records; A/B nontemporal result /
# in-place stores in the checksum kernels (flags none / INPLACE / INPLACE+IPHDR)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/s6
tools/gpu_run.sh s6/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh s6/bench_rx 300 python tools/bench_rx.py --configs 2,4,3,5
for r in 1 2; do
  for v in cur ntst; do
    L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
    for fl in none inplace inplace,iphdr verify; do
      XCSUM_LIB=$L tools/gpu_run.sh s6/c2_${v}_${fl/,/_}_$r 200 python tools/sweep.py --config 2 --geoms 16,2,6 --bpc 0 --orders=-1,0 --flags $fl --rounds 3 --launches 20
    done
    XCSUM_LIB=$L tools/gpu_run.sh s6/c2u_${v}_inplace_iphdr_$r 200 python tools/sweep.py --config 2 --layout umem --geoms 16,2,6 --bpc 0 --orders=-1,0 --flags inplace,iphdr --rounds 3 --launches 20
    XCSUM_LIB=$L tools/gpu_run.sh s6/c3_${v}_$r 200 python tools/sweep.py --config 3 --geoms 64,0,8 --bpc 0 --orders=-1,0 --rounds 3 --launches 40
    XCSUM_LIB=$L tools/gpu_run.sh s6/c5_${v}_$r 200 python tools/sweep.py --config 5 --geoms 64,1,9 --bpc 0 --orders=-1,0 --rounds 2 --launches 10
  done
done
