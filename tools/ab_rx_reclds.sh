#!/bin/bash
# wide receive kernel: records stored through LDS (1 KB per store instruction,
# variant reclds: make -C libxudp_amd variant NAME=reclds DEFS=-DXCSUM_RX_WIDE_REC_LDS=1)
# against per-lane 64-byte records.  Adopted: the macro is gone, the LDS
# path is the shipped one.  $1 = log dir
set -e
d=${1:-reclds}
XCSUM_LIB=libxudp_amd/variants/reclds/libxcsum.so tools/gpu_run.sh $d/pytest_var 400 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread
for i in 1 2; do
for v in cur reclds; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh $d/${v}_$i 300 python tools/bench_rx.py --configs 2,4 --reps 30
done
done
unset XCSUM_LIB
