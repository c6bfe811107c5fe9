#!/bin/bash
# Round 3 GPU check: the product suite, the suite under the bounds-checked
# debug build, and the end-to-end host path (pageable copies now staged by
# the library).  Each step under its own time limit; the chain stops at a
# fault.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R03_TAG:-r03d}
P="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_run.sh $t/pytest_gpu 600 $P &&
XCSUM_LIB=$PWD/libxudp_amd/debug/libxcsum.so tools/gpu_run.sh $t/pytest_gpu_debug 900 $P &&
tools/gpu_run.sh $t/e2e_config2 300 python tools/bench_e2e.py
