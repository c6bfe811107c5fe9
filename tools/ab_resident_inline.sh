#!/bin/bash
# The XCSUM_* tuning variables are read only by the A/B build (`make -C
# libxudp_amd variant NAME=ab`, -DXCSUM_ENV_TUNING): run with
# XCSUM_LIB=libxudp_amd/variants/ab/libxcsum.so; libxcsum.so takes them
# through xcsum_ctx_set_tuning only.
# same-box A/B of the resident inline descriptors: ring bench, 1/2/4 frames
set -u
for r in 1 2; do
  for v in 1 0; do
    XCSUM_RESIDENT_INLINE=$v RING_RESIDENT_WG=16 tools/gpu_run.sh r03t/ab_inline${v}_$r 200 tests/c/umem_ring --bench 1,2,4 || exit $?
  done
done
