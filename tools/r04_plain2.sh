#!/bin/bash
# Library plain pass + a second pass (saved-block copy / blind 64-B / 2-byte)
# vs the fused in-place pass: does any two-pass schedule with complete
# blocks beat fused when the first pass is the real kernel?
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04w}
mkdir -p gpurun_out/$t
L=lib_plain,lib_fused,lib_plain+copy64,lib_plain+blind64,lib_plain+w2,copy64,blind64
for fam in 4 6; do
  timeout -k 10 240 python -u tools/inplace_probe.py --family $fam --legs $L --rounds 3 \
    >> gpurun_out/$t/probe.log 2>&1 || exit $?
done
grep ms_per gpurun_out/$t/probe.log
