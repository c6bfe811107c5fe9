#!/bin/bash
# Round 3 GPU check on the current tree: the product suite, the suite under
# the bounds-checked debug build, smoke, and the bench under the driver's own
# command.  Each step under its own time limit; the chain stops at a fault.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R03_TAG:-r03e}
P="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_run.sh $t/pytest_gpu 600 $P &&
XCSUM_LIB=$PWD/libxudp_amd/debug/libxcsum.so tools/gpu_run.sh $t/pytest_gpu_debug 900 $P &&
tools/gpu_run.sh $t/smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
tools/gpu_run.sh $t/bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5
