#!/bin/bash
# full GPU suite + TX ring harness + end-to-end bench on the final host path
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/s10
tools/gpu_run.sh s10/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh s10/ring_check 200 tests/c/umem_ring
tools/gpu_run.sh s10/ring_bench 300 tests/c/umem_ring --bench 1,16,100,1024,4096
tools/gpu_run.sh s10/e2e 300 python tools/bench_e2e.py
