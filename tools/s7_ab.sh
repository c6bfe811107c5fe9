#!/bin/bash
# copy-free small-batch host path (XCSUM_DIRECT_MAX) vs current: correctness
# (TX ring harness, host-path GPU tests) and per-call cost by batch size
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/s7
V=libxudp_amd/variants/direct
LD_LIBRARY_PATH=$V tools/gpu_run.sh s7/ring_direct_check 200 tests/c/umem_ring
XCSUM_LIB=$V/libxcsum.so tools/gpu_run.sh s7/pytest_host_direct 300 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_config1.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  tools/gpu_run.sh s7/ring_cur_$r 300 tests/c/umem_ring --bench 1,16,100,1024,4096
  LD_LIBRARY_PATH=$V tools/gpu_run.sh s7/ring_direct_$r 300 tests/c/umem_ring --bench 1,16,100,1024,4096
done
