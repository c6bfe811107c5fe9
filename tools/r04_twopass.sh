#!/bin/bash
# TWO_PASS store widths vs fused vs the probe's plain + 2-byte second pass.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04x}
mkdir -p gpurun_out/$t
L=lib_plain,lib_fused,lib_plain+w2,lib_two_pass_w0,lib_two_pass_w32,lib_two_pass_w64,lib_two_pass_w0_out
for fam in 4 6; do
  for lay in packed umem; do
    timeout -k 10 240 python -u tools/inplace_probe.py --family $fam --layout $lay --legs $L --rounds 3 \
      >> gpurun_out/$t/probe.log 2>&1 || exit $?
  done
done
grep ms_per gpurun_out/$t/probe.log
