#!/bin/bash
# box-to-box spread of the receive kernel: clocks/power caps of this box next
# to the config 5 receive bench (RX VERIFY vs the checksum kernel).  $1 = log dir
set -e
d=${1:-box}
mkdir -p gpurun_out/$d
(rocm-smi --showclocks --showmaxpower --showpower --showproductname || true) > gpurun_out/$d/smi.log 2>&1
tools/gpu_run.sh $d/bench_c5 300 python tools/bench_rx.py --configs 5,2 --reps 10
(rocm-smi --showclocks --showpower || true) >> gpurun_out/$d/smi.log 2>&1
