#!/bin/bash
# checksum kernel under each flag combination, current build vs a variant
#   tools/ab_flags.sh <tag> <variant> [config]
set -e
tag="$1"; var="$2"; cfg="${3:-2}"
for v in cur $var; do
  if [ $v = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so; fi
  for f in none inplace,rfc inplace,iphdr,rfc verify verify,iphdr; do
    tools/gpu_run.sh s1/${tag}_${v}_$f 120 python tools/sweep.py --config $cfg --rounds 3 --geoms "${GEOM:-16,2,6}" --bpc ${BPC:-1} --flags $f
  done
done
