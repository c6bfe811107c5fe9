set -e
tools/gpu_run.sh s1/pytest_gpu4 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tools/gpu_run.sh s1/bench12_2 200 python bench.py --no-cpu-baseline
tools/gpu_run.sh s1/bench12_3 200 python bench.py --config 3 --no-cpu-baseline
tools/gpu_run.sh s1/bench_rx12 300 python tools/bench_rx.py --configs 2,4,3
