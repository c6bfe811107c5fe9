#!/bin/bash
# wide receive kernel with temporal header loads: timing + FETCH_SIZE.  $1 = log dir
set -e
d=${1:-rxwide6}
tools/gpu_run.sh $d/pytest 400 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh $d/bench_mtu 300 python tools/bench_rx.py --configs 2,4 --reps 30 --geoms "16,6,1,2;16,6,0;32,3,0;32,3,0,2;64,2,0"
tools/gpu_run.sh $d/bench_c3 300 python tools/bench_rx.py --configs 3 --reps 30 --geoms "auto;8,2,0"
tools/gpu_run.sh $d/bench_c5 300 python tools/bench_rx.py --configs 5 --reps 10 --geoms "64,9,1;64,9,0"
tools/gpu_run.sh $d/bytes2 300 bash tools/pmc_rx_bytes.sh 2 gpurun_out/$d/bytes2 --geoms "16,6,1,2;32,3,0"
