#!/bin/bash
# Checksum-kernel A/B across library builds in ONE gpurun call: plain and
# VERIFY on configs 2, 4, 5 (tools/verify_probe.py), current build and each
# named variant under libxudp_amd/variants/, two interleaved rounds.
#   tools/ab_csum_libs.sh <outdir> <variant>...
set -e
out="$1"; shift; mkdir -p $out
for r in 1 2; do
  for v in cur "$@"; do
    L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
    for c in ${CFGS:-2 4 5}; do
      XCSUM_LIB=$L timeout -k 10 300 python tools/verify_probe.py --config $c --checks valid > $out/${v}_c${c}_$r.log 2>&1
    done
  done
done
