#!/bin/bash
# Round 3 sweeps on xudp's own TX layout (one frame per 4096-byte slot):
# small frames (config 3) over frame-group geometries and visiting orders,
# and the in-place mode on MTU frames over blocks per CU and orders.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R03_TAG:-r03s}
tools/gpu_run.sh $t/sweep_c3_umem_geoms 300 python tools/sweep.py --config 3 --layout umem \
    --geoms "auto;4,1,2;4,2,2;4,4,2;8,1,2;8,2,1;2,2,4;16,1,2" --rounds 4 &&
tools/gpu_run.sh $t/sweep_c3_umem_orders 300 python tools/sweep.py --config 3 --layout umem \
    --geoms "auto;4,4,2" --orders "-1,0;5,4;6,4;4,4;5,6;3,4;7,3;0,0" --rounds 4 &&
tools/gpu_run.sh $t/sweep_c2_umem_inplace 300 python tools/sweep.py --config 2 --layout umem \
    --flags inplace,iphdr --geoms "auto;16,2,6;16,1,6" --bpc "0,1,2,3" --rounds 4 &&
tools/gpu_run.sh $t/sweep_c2_umem_inplace_orders 300 python tools/sweep.py --config 2 --layout umem \
    --flags inplace,iphdr --geoms "auto" --orders "-1,0;5,4;4,3;4,4;6,4;5,3;0,0" --rounds 4
