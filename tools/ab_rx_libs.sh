#!/bin/bash
# Receive-kernel A/B across library builds in ONE gpurun call (box-to-box
# spread on this kernel is up to 20 %): current, and each named variant under
# libxudp_amd/variants/, interleaved over two rounds.
#   [ROUNDS=3] [EXTRA="--layout umem"] tools/ab_rx_libs.sh <outdir> <configs> <geoms> <variant>...
set -e
out="$1"; cfgs="$2"; geoms="$3"; shift 3; mkdir -p $out
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python tools/bench_rx.py --configs $cfgs --only verify,csum_verify --geoms "$geoms" $EXTRA > $out/cur_$r.log 2>&1
  for v in "$@"; do
    XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so timeout -k 10 300 python tools/bench_rx.py --configs $cfgs --only verify,csum_verify --geoms "$geoms" $EXTRA > $out/${v}_$r.log 2>&1
  done
done
