#!/bin/bash
# Checksum kernel with flags across library builds in ONE gpurun call:
# tools/sweep.py per (config, layout, flags) for the current build and each
# named variant under libxudp_amd/variants/, ROUNDS interleaved rounds.
#   [ROUNDS=2] [CASES="2:packed:inplace,iphdr 2:umem:inplace,iphdr"] tools/ab_flags_libs.sh <outdir> <variant>...
set -e
out="$1"; shift; mkdir -p $out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in cur "$@"; do
    L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
    for c in ${CASES:-2:packed:inplace,iphdr 2:umem:inplace,iphdr}; do
      IFS=: read cfg lay fl <<< "$c"
      XCSUM_LIB=$L timeout -k 10 300 python tools/sweep.py --config $cfg --layout $lay --flags "$fl" \
          --rounds 3 --launches 10 > $out/${v}_c${cfg}_${lay}_${fl//,/+}_$r.log 2>&1
    done
  done
done
