#!/bin/bash
# small frames (config 3): lane-per-frame kernel (4,2,0) (8,2,0) vs the group
# kernel defaults.  $1 = log dir
set -e
d=${1:-rxsmall}
tools/gpu_run.sh $d/pytest 400 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh $d/bench_c3 300 python tools/bench_rx.py --configs 3 --reps 30 --geoms "auto;4,2,1;4,2,0;4,2,0,2;8,2,0;8,2,0,2"
