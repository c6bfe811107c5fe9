#!/bin/bash
# Same-box A/B of library builds through bench.py: for each round, each
# config, each library (name=path pairs), one bench process; logs under
# gpurun_out/$TAG/.  Usage:
#   tools/ab_bench.sh TAG ROUNDS "CONFIG_ARGS;..." name=lib.so ...
# e.g. tools/ab_bench.sh ab1 2 "--config 2;--config 3" new=libxudp_amd/libxcsum.so \
#      r02=libxudp_amd/variants/r02/libxcsum.so
set -u
cd "${GRAFT_REPO_ROOT:-.}"
tag=$1; rounds=$2; IFS=';' read -ra cfgs <<< "$3"; shift 3
for r in $(seq 1 "$rounds"); do
  for c in "${cfgs[@]}"; do
    cn=$(echo "$c" | tr -c 'a-zA-Z0-9\n' '_' | sed 's/__*/_/g;s/^_//;s/_$//')
    for nl in "$@"; do
      name=${nl%%=*}; lib=${nl#*=}
      XCSUM_LIB=$PWD/$lib tools/gpu_run.sh "$tag/${cn}_${name}_$r" 240 \
        python bench.py --steps 100 --warmup 5 --no-cpu-baseline $c || exit $?
    done
  done
done
