set -e
tools/gpu_run.sh fc/pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh fc/smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tools/gpu_run.sh fc/bench 300 python bench.py
