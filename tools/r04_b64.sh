#!/bin/bash
# Whole 64-B block in-place stores (XCSUM_INPLACE_B64): parity, then the
# interleaved in-place probe on configs 2 and 4 (packed) and xudp's slots.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04m}
mkdir -p gpurun_out/$t
timeout -k 10 400 python -u -m pytest tests/test_gpu_inplace.py -x -q -k "block or golden or fuzz" \
  --timeout 300 --timeout-method thread > gpurun_out/$t/pytest_b64.log 2>&1 || { tail -30 gpurun_out/$t/pytest_b64.log; exit 1; }
tail -3 gpurun_out/$t/pytest_b64.log
L=read,lib_plain,lib_fused,lib_b64_1,lib_b64_2,lib_b64_2_tl0,read+blind64
for fam in 4 6; do
  for lay in packed umem; do
    timeout -k 10 240 python -u tools/inplace_probe.py --family $fam --layout $lay --legs $L --rounds 3 \
      >> gpurun_out/$t/probe.log 2>&1 || exit $?
  done
done
grep ms_per gpurun_out/$t/probe.log
