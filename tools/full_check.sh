# whole GPU suite, smoke, default bench; then the receive bench for config 5
# under rocprofv3 --kernel-trace --stats (the lane-per-frame kernel).  $1 = log dir
set -e
d=${1:-fc}
export TMPDIR=/tmp
tools/gpu_run.sh $d/pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh $d/smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tools/gpu_run.sh $d/bench 300 python bench.py
tools/gpu_run.sh $d/rx_stats5 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/$d/rx_stats5 -o run -- python3 tools/bench_rx.py --configs 5 --reps 10
