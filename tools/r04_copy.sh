#!/bin/bash
# Saved-block second pass (copy64) vs blind and 2-byte second passes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04o}
mkdir -p gpurun_out/$t
L=read,lib_plain,lib_fused,read+w2,read+blind64,copy64,read+copy64,blind64
for fam in 4 6; do
  for lay in packed umem; do
    timeout -k 10 240 python -u tools/inplace_probe.py --family $fam --layout $lay --legs $L --rounds 3 \
      >> gpurun_out/$t/probe.log 2>&1 || exit $?
  done
done
grep ms_per gpurun_out/$t/probe.log
