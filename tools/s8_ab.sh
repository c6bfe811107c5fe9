#!/bin/bash
# host path per-call cost: copy-free small batches, and spin-wait on the slot event
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/s8
for r in 1 2 3; do
  for v in cur direct dspin; do
    L=; [ $v = cur ] || L=libxudp_amd/variants/$v
    LD_LIBRARY_PATH=$L tools/gpu_run.sh s8/ring_${v}_$r 300 tests/c/umem_ring --bench 1,16,100,1024
  done
done
