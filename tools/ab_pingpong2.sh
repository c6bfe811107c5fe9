set -e
tools/gpu_run.sh s1/pytest_gpu3 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tools/gpu_run.sh s1/pp2_3 200 python tools/sweep.py --config 3 --rounds 3 --geoms "4,1,2;4,2,2;2,2,4" --bpc 0,3,4,5
tools/gpu_run.sh s1/pp2_2 200 python tools/sweep.py --config 2 --rounds 3 --geoms "16,1,6;16,2,6;16,1,12;8,1,12" --bpc 1,2,3
tools/gpu_run.sh s1/pp2_5 200 python tools/sweep.py --config 5 --rounds 2 --geoms "64,1,9;16,1,12" --bpc 1,2,3
tools/gpu_run.sh s1/pp2_2u 200 python tools/sweep.py --config 2 --layout umem --rounds 3 --geoms "16,1,6" --bpc 2,3
tools/gpu_run.sh s1/bench2 200 python bench.py
