#!/bin/bash
# What IPHDR costs on config 2: plain / in place, with and without the IPv4 header.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04q}
mkdir -p gpurun_out/$t
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-order-ab"
for r in 1 2; do
  for fl in none iphdr inplace inplace,iphdr; do
    a=""; [ $fl != none ] && a="--flags $fl"
    timeout -k 10 200 $B $a > gpurun_out/$t/c2_${fl/,/_}_$r.log 2>&1 || { tail -5 gpurun_out/$t/c2_${fl/,/_}_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/$t/c2_${fl/,/_}_$r.log
  done
done
