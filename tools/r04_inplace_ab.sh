#!/bin/bash
# Round 4 in-place A/B on one box, alternating: the fused pass as shipped,
# with each frame's first 2 / 4 chunks loaded temporally (XCSUM_INPLACE_TL),
# and with nontemporal IPv4-header loads (variant build ihnt).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04g}
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
V=$PWD/libxudp_amd/variants/ihnt/libxcsum.so
for r in 1 2; do
  tools/gpu_run.sh $t/c2_fused_$r 300 $B --flags inplace,iphdr &&
  XCSUM_INPLACE_TL=2 tools/gpu_run.sh $t/c2_tl2_$r 300 $B --flags inplace,iphdr &&
  XCSUM_LIB=$V tools/gpu_run.sh $t/c2_ihnt_$r 300 $B --flags inplace,iphdr &&
  tools/gpu_run.sh $t/c4_fused_$r 300 $B --config 4 --flags inplace &&
  XCSUM_INPLACE_TL=4 tools/gpu_run.sh $t/c4_tl4_$r 300 $B --config 4 --flags inplace || exit $?
done
