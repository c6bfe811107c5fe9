#!/bin/bash
# Host-resident end-to-end rates on the final tree (tools/bench_e2e.py), in a
# libxudp-style UMEM mapping: config 2 packed and in xudp's slots, config 4.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04v}
mkdir -p gpurun_out/$t
for a in "--config 2" "--config 2 --layout umem" "--config 4"; do
  echo "== $a" >> gpurun_out/$t/e2e.log
  timeout -k 10 300 python -u tools/bench_e2e.py $a --reps 5 >> gpurun_out/$t/e2e.log 2>&1 || { tail -5 gpurun_out/$t/e2e.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/$t/e2e.log
