#!/bin/bash
# Round 4: the in-place schedules on config 2 and 4 (same box, alternating),
# then the driver's bench command, then the product suite with the
# registration trace (XCSUM_REG_TRACE).  Each step under its own limit; the
# chain stops at a fault (tools/gpu_run.sh).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04b}
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
tools/gpu_run.sh $t/c2_inplace_fused 300 $B --flags inplace,iphdr --inplace-schedule fused &&
tools/gpu_run.sh $t/c2_inplace_two_pass 300 $B --flags inplace,iphdr --inplace-schedule two_pass &&
tools/gpu_run.sh $t/c4_inplace_fused 300 $B --config 4 --flags inplace --inplace-schedule fused &&
tools/gpu_run.sh $t/c4_inplace_two_pass 300 $B --config 4 --flags inplace --inplace-schedule two_pass &&
tools/gpu_run.sh $t/c2_inplace_fused_2 300 $B --flags inplace,iphdr --inplace-schedule fused &&
tools/gpu_run.sh $t/c2_inplace_two_pass_2 300 $B --flags inplace,iphdr --inplace-schedule two_pass &&
tools/gpu_run.sh $t/bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5 &&
XCSUM_REG_TRACE=$PWD/gpurun_out/$t/regtrace.log \
  tools/gpu_run.sh $t/pytest_gpu 700 python -u -m pytest tests -m gpu -x -q -s --timeout 300 \
  --timeout-method thread
