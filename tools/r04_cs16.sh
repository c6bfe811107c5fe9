#!/bin/bash
# In-place A/B: whole-chunk field stores from the lane holding the chunk
# (variant cs16, XCSUM_INPLACE_CHUNK16) vs the shipped 2-byte stores.  Parity
# of the variant first (in-place tests), then alternating bench runs.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04i}
V=$PWD/libxudp_amd/variants/cs16/libxcsum.so
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-order-ab"
XCSUM_LIB=$V tools/gpu_run.sh $t/pytest_cs16 400 python -u -m pytest tests/test_gpu_inplace.py \
  tests/test_gpu_parity.py -x -q -k "inplace or schedules or widths" --timeout 300 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/$t/pytest_cs16.log && ! grep -q "failed" gpurun_out/$t/pytest_cs16.log || exit 1
for r in 1 2; do
  tools/gpu_run.sh $t/c2_ship_$r 300 $B --flags inplace,iphdr &&
  XCSUM_LIB=$V tools/gpu_run.sh $t/c2_cs16_$r 300 $B --flags inplace,iphdr &&
  tools/gpu_run.sh $t/c4_ship_$r 300 $B --config 4 --flags inplace &&
  XCSUM_LIB=$V tools/gpu_run.sh $t/c4_cs16_$r 300 $B --config 4 --flags inplace &&
  tools/gpu_run.sh $t/c2u_ship_$r 300 $B --flags inplace,iphdr --layout umem &&
  XCSUM_LIB=$V tools/gpu_run.sh $t/c2u_cs16_$r 300 $B --flags inplace,iphdr --layout umem || exit $?
done
