#!/bin/bash
# A/B of the checksum kernel's VERIFY mode: current library vs the round-1
# build (libxudp_amd/variants/r01, built from git dcd7f00), interleaved
# sweeps in separate processes, configs 2 and 5.
set -e
out=${1:-gpurun_out/abv}; mkdir -p $out
for r in 1 2; do
for v in cur r01; do
  if [ $v = cur ]; then L=libxudp_amd/libxcsum.so; else L=libxudp_amd/variants/$v/libxcsum.so; fi
  for c in 2 5; do
    XCSUM_LIB=$L timeout -k 10 200 python tools/sweep.py --config $c --geoms "16,2,6;64,1,9" --flags verify --rounds 3 > $out/${v}_c${c}_v_$r.log 2>&1
    XCSUM_LIB=$L timeout -k 10 200 python tools/sweep.py --config $c --geoms "16,2,6;64,1,9" --rounds 3 > $out/${v}_c${c}_n_$r.log 2>&1
  done
done
done
