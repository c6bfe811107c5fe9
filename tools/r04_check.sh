#!/bin/bash
# Round 4 tree check: box facts, the host-core crossover timing, the product
# suite (registration trace on), the bounds-checked suite, smoke, and the
# driver's bench command.  Each step under its own limit; the chain stops at
# a fault (tools/gpu_run.sh).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04f}
mkdir -p gpurun_out/$t
bash tools/r04_env.sh > gpurun_out/$t/env.log 2>&1
python tools/crossover.py > gpurun_out/$t/crossover.log 2>&1
P="python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread"
XCSUM_REG_TRACE=$PWD/gpurun_out/$t/regtrace.log tools/gpu_run.sh $t/pytest_gpu 700 $P &&
XCSUM_LIB=$PWD/libxudp_amd/debug/libxcsum.so tools/gpu_run.sh $t/pytest_gpu_debug 900 $P &&
tools/gpu_run.sh $t/smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
tools/gpu_run.sh $t/bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5
