set -e
d=${1:-s2}
tools/gpu_run.sh $d/pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh $d/bench_rx 300 python tools/bench_rx.py --configs 2,4,3,5
tools/gpu_run.sh $d/smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
