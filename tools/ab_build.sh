#!/bin/bash
# build-kernel geometry sweep (tuning): each geometry in its own process
set -e
for g in auto 16,6 32,3 16,3 64,2; do
  if [ $g = auto ]; then unset XCSUM_BUILD_GEOMETRY; else export XCSUM_BUILD_GEOMETRY=$g; fi
  tools/gpu_run.sh s1/build_${g/,/_} 200 python tools/bench_build.py
done
