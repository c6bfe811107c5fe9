#!/bin/bash
# A/B of kernel libraries (tuning only): the parity subset on the current
# build, then the same sweeps per library, each in its own process.
#   tools/ab_libs.sh <tag> <name>=<path/libxcsum.so|cur> ...
set -e
tag="$1"; shift
tools/gpu_run.sh par_$tag 700 python -m pytest tests -m gpu -q -x -p no:cacheprovider
for spec in "$@"; do
  name="${spec%%=*}"; lib="${spec#*=}"
  if [ "$lib" = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=$lib; fi
  tools/gpu_run.sh ${tag}_3_$name 200 python tools/sweep.py --config 3 --rounds 4 --geoms "4,1,2;8,1,2;2,1,4"
  tools/gpu_run.sh ${tag}_2_$name 200 python tools/sweep.py --config 2 --rounds 4 --geoms "16,1,6;16,2,6" --bpc 0,3
  tools/gpu_run.sh ${tag}_4_$name 200 python tools/sweep.py --config 4 --rounds 3 --geoms "16,1,6" --bpc 3
  tools/gpu_run.sh ${tag}_5_$name 200 python tools/sweep.py --config 5 --rounds 2 --geoms "64,1,9"
done
