#!/bin/bash
# A/B of the receive kernel between the current library and a variant build
# (libxudp_amd/variants/<name>), interleaved processes, bench_rx VERIFY modes.
#   tools/ab_rx_lib.sh <variant> <outdir> [configs]
set -e
v="$1"; out="$2"; cfgs="${3:-2,4,5}"; mkdir -p $out
for r in 1 2; do
  timeout -k 10 300 python tools/bench_rx.py --configs $cfgs --only plain,verify,csum_verify > $out/cur_$r.log 2>&1
  XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so timeout -k 10 300 python tools/bench_rx.py --configs $cfgs --only plain,verify,csum_verify > $out/${v}_$r.log 2>&1
done
