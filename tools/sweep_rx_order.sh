#!/bin/bash
# The XCSUM_* tuning variables are read only by the A/B build (`make -C
# libxudp_amd variant NAME=ab`, -DXCSUM_ENV_TUNING): run with
# XCSUM_LIB=libxudp_amd/variants/ab/libxcsum.so; libxcsum.so takes them
# through xcsum_ctx_set_tuning only.
# RX visiting-order sweep on xudp's UMEM layout: tools/bench_rx.py under each
# XCSUM_RX_ORDER value ("0" off, "R,T" 2^R regions of 2^T-frame tiles).
#   tools/sweep_rx_order.sh <outdir under gpurun_out> "0;5,6;3,6" [configs]
set -e
out="gpurun_out/$1"; mkdir -p "$out"
IFS=';' read -ra ORDERS <<< "$2"
for o in "${ORDERS[@]}"; do
  XCSUM_RX_ORDER="$o" timeout -k 10 200 python tools/bench_rx.py --configs "${3:-2,3}" --layout umem \
      --only plain,verify,csum_verify --reps 5 > "$out/order_${o/,/_}.log" 2>&1
done
