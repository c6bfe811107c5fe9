#!/bin/bash
# A/B of the in-place store width (timing only; the variants write wrong data)
set -e
for v in cur inplace_16 inplace_32 inplace_64 inplace_128; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh s1/abj_$v 120 python tools/sweep.py --config 2 --rounds 3 --geoms "16,2,6" --bpc 1 --flags inplace,rfc
done
