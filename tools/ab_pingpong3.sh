set -e
tools/gpu_run.sh s1/pp3_2 200 python tools/sweep.py --config 2 --rounds 6 --geoms "16,1,6;16,2,6" --bpc 1,2
tools/gpu_run.sh s1/pp3_4 200 python tools/sweep.py --config 4 --rounds 6 --geoms "16,1,6;16,2,6" --bpc 1,2
tools/gpu_run.sh s1/pp3_2u 200 python tools/sweep.py --config 2 --layout umem --rounds 6 --geoms "16,1,6;16,2,6" --bpc 1,2
tools/gpu_run.sh s1/pp3_5 200 python tools/sweep.py --config 5 --rounds 3 --geoms "64,1,9;64,2,9" --bpc 1,2
