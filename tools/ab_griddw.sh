#!/bin/bash
# csum kernel at MTU: 16-byte aligned chunk grid (shipped) vs the dword grid
# (variant griddw: make -C libxudp_amd variant NAME=griddw DEFS=-DXCSUM_GRID_DW=1)
set -e
for i in 1 2; do
for v in cur griddw; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh abl/grid_${v}_$i 200 python tools/sweep.py --config 2 --rounds 4 --geoms "16,2,6;16,1,6" --bpc 1,2 --flags verify
done
done
