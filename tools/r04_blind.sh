#!/bin/bash
# Blind whole-block write probe: do full-sector stores avoid
# the memory-side merge cost of 2-byte / partial stores?
set -e
mkdir -p gpurun_out/r04l
L=read,w2,read+w2,read+w32,blind16,blind32,blind64,read+blind16,read+blind32,read+blind64,read+blind128,lib_fused,lib_plain
for fam in 4 6; do
  timeout -k 10 240 python -u tools/inplace_probe.py --family $fam --legs $L --rounds 2 >> gpurun_out/r04l/blind.log 2>&1
done
