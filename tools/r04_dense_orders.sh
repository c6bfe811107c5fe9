#!/bin/bash
# Dense (packed) batches with flags: the automatic order vs forced ones.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04do}
mkdir -p gpurun_out/$t
i=0
while read -r a; do
  for r in 1 2; do
    for o in auto 0,0 3,4 4,4 4,5 2,5 3,3; do
      i=$((i+1))
      if [ $o = auto ]; then env_o=""; else env_o="XCSUM_ORDER=$o"; fi
      env $env_o timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-order-ab --no-calibrate $a > gpurun_out/$t/b$i.log 2>&1 || { echo "FAIL: $a $o"; tail -5 gpurun_out/$t/b$i.log; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], '|', d['ms_per_step'], d['roofline'].get('frac_vs_ceiling'))" gpurun_out/$t/b$i.log "$a $o"
    done
  done
done <<'LIST'
--config 2 --flags verify
--config 4 --flags verify
--config 2 --flags inplace,iphdr
--config 4 --flags inplace
LIST
