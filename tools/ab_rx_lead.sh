#!/bin/bash
# lane-per-frame receive kernel: when the next batch's header chunks are loaded
# (lead 0 = at batch start; lead N = N steps before the batch end; 4 shipped),
# variants: make -C libxudp_amd variant NAME=leadN DEFS=-DXCSUM_RX_WIDE_HDR_LEAD=N.
# $1 = log dir
set -e
d=${1:-rxlead}
for v in lead4 lead8; do
  XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so tools/gpu_run.sh $d/pytest_$v 400 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread
done
for v in cur lead4 lead8; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh $d/$v 300 python tools/bench_rx.py --configs 2,4,5 --reps 20
done
unset XCSUM_LIB
tools/gpu_run.sh $d/bytes_lead8 300 env XCSUM_LIB=libxudp_amd/variants/lead8/libxcsum.so bash tools/pmc_rx_bytes.sh 2 gpurun_out/$d/bytes_lead8
