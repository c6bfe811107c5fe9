#!/bin/bash
# receive kernel header path: cross-lane broadcast (shipped) vs the LDS stage
# (variant hdrlds: make -C libxudp_amd variant NAME=hdrlds DEFS=-DXCSUM_RX_HDR_LDS=1)
set -e
for i in 1 2; do
for v in cur hdrlds; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh rxhdr/${v}_$i 200 python tools/bench_rx.py --configs 2,3 --reps 30 --geoms "auto;16,6,1,1"
done
done
for v in cur hdrlds; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh rxhdr/${v}_c5 300 python tools/bench_rx.py --configs 5 --reps 10
done
