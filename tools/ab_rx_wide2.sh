#!/bin/bash
# receive kernel at MTU: wide-kernel group sizes (16,6,0) (32,3,0) (64,2,0)
# against the shipped (16,6,1) at 2 blocks/CU.  $1 = log directory
set -e
d=${1:-rxwide5}
tools/gpu_run.sh $d/pytest 400 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh $d/bench_mtu 300 python tools/bench_rx.py --configs 2,4 --reps 30 --geoms "16,6,1,2;16,6,0;32,3,0;32,3,0,2;64,2,0;64,2,0,2;64,2,0,3"
tools/gpu_run.sh $d/bench_c5 300 python tools/bench_rx.py --configs 5 --reps 10 --geoms "64,9,1;64,9,0"
