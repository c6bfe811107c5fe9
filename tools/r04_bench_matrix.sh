#!/bin/bash
# bench.py across its modes on the final tree (calibration on): one line each.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04m2}
mkdir -p gpurun_out/$t
i=0
while read -r a; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $a > gpurun_out/$t/b$i.log 2>&1 || { echo "FAIL: $a"; tail -5 gpurun_out/$t/b$i.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], '|', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('frac_vs_ceiling'), d['config'].get('order_calibration'), d.get('parity_ok'))" gpurun_out/$t/b$i.log "$a"
done <<'LIST'
--config 2 --layout umem
--config 3
--config 4
--config 2 --flags inplace,iphdr
--config 4 --flags inplace
--config 2 --flags verify
--config 2 --flags inplace,iphdr --layout umem
--config 2 --no-graph
LIST
