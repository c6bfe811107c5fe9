#!/bin/bash
# Round 4 GPU check on the current tree: box facts, the product suite, the
# suite under the bounds-checked debug build (R04_DEBUG=1), smoke, and the
# bench under the driver's own command.  Each step under its own time limit;
# the chain stops at a fault (tools/gpu_run.sh).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04a}
mkdir -p gpurun_out/$t
bash tools/r04_env.sh > gpurun_out/$t/env.log 2>&1
P="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_run.sh $t/pytest_gpu 600 $P &&
if [ "${R04_DEBUG:-0}" = 1 ]; then
  XCSUM_LIB=$PWD/libxudp_amd/debug/libxcsum.so tools/gpu_run.sh $t/pytest_gpu_debug 900 $P
fi &&
tools/gpu_run.sh $t/smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
tools/gpu_run.sh $t/bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5
