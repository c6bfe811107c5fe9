#!/bin/bash
# Round 3 GPU check: the product suite, then the same suite under the
# bounds-checked debug build (every kernel load/store checked, conftest fails
# a test that made an out-of-bounds access), then a same-box A/B of this
# library against round 2's on configs 2 and 3, and the in-place bench.
# Each step under its own time limit; the chain stops at a fault.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
P="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_run.sh r03b/pytest_gpu 600 $P &&
XCSUM_LIB=$PWD/libxudp_amd/debug/libxcsum.so tools/gpu_run.sh r03b/pytest_gpu_debug 900 $P &&
tools/ab_bench.sh r03b/ab 2 "--config 2;--config 3" new=libxudp_amd/libxcsum.so \
    r02=libxudp_amd/variants/r02/libxcsum.so &&
tools/gpu_run.sh r03b/bench_inplace_c2 240 python bench.py --steps 100 --warmup 5 \
    --no-cpu-baseline --flags inplace,iphdr
