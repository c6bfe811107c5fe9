#!/bin/bash
# A/B of the checksum kernel's loop shape (tuning only): the current build
# vs libxudp_amd/variants/latch (make -C libxudp_amd variant NAME=latch
# DEFS=-DXCSUM_PINGPONG=0), same sweeps, each library in its own process.
set -e
for v in cur latch; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh s1/pp_${v}_3 200 python tools/sweep.py --config 3 --rounds 3 --geoms "4,1,2;8,1,2;2,1,4;4,2,2" --bpc 0,4,6
  tools/gpu_run.sh s1/pp_${v}_2 200 python tools/sweep.py --config 2 --rounds 3 --geoms "16,1,6;32,1,6;16,1,3" --bpc 0,2,3,4
  tools/gpu_run.sh s1/pp_${v}_4 200 python tools/sweep.py --config 4 --rounds 3 --geoms "16,1,6" --bpc 0,2,3
  tools/gpu_run.sh s1/pp_${v}_5 200 python tools/sweep.py --config 5 --rounds 2 --geoms "64,1,9;64,1,2;32,1,6" --bpc 0,2,3
done
