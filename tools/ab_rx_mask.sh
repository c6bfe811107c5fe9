#!/bin/bash
# receive kernel edge masks: per-chunk branch (shipped) vs masking every chunk
# (variant maskall: make -C libxudp_amd variant NAME=maskall DEFS=-DXCSUM_RX_MASK_ALL=1)
set -e
for i in 1 2; do
for v in cur maskall; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh rxmask/${v}_$i 200 python tools/bench_rx.py --configs 2,3 --reps 30 --geoms "auto;16,6,1,1"
done
done
for v in cur maskall; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh rxmask/${v}_c5 300 python tools/bench_rx.py --configs 5 --reps 10
done
