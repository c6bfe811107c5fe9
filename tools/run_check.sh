set -e
tools/gpu_run.sh s2/pytest_rx 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_host_path.py -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh s2/bench_rx 300 python tools/bench_rx.py --configs 2,4,3,5
