#!/bin/bash
# A/B of RX kernel build variants (tuning only): make -C libxudp_amd variant
# NAME=rxN DEFS=-DXCSUM_RX_EXP=N, then   tools/ab_rx.sh <tag> <geoms> cur rx8 ...
set -e
tag="$1"; geoms="$2"; shift 2
for v in "$@"; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  tools/gpu_run.sh s1/${tag}_$v 200 python tools/bench_rx.py --configs 3 --geoms "$geoms"
done
