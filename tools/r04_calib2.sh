#!/bin/bash
# Does the calibrated order ever lose to the automatic one? Alternating
# bench runs with and without xcsum_ctx_calibrate_order, per workload.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04cal2}
mkdir -p gpurun_out/$t
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k calibrat --timeout 300 \
  --timeout-method thread > gpurun_out/$t/pytest.log 2>&1 || { tail -20 gpurun_out/$t/pytest.log; exit 1; }
tail -1 gpurun_out/$t/pytest.log
i=0
while read -r a; do
  for r in 1 2; do
    for c in cal nocal; do
      i=$((i+1)); x=""; [ $c = nocal ] && x="--no-calibrate"
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-order-ab $a $x > gpurun_out/$t/b$i.log 2>&1 || { echo "FAIL: $a $x"; tail -5 gpurun_out/$t/b$i.log; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], '|', d['ms_per_step'], d['roofline'].get('frac_vs_ceiling'), d['config'].get('order_calibration'))" gpurun_out/$t/b$i.log "$a $c"
    done
  done
done <<'LIST'
--config 2
--config 2 --flags verify
--config 3
--config 2 --flags inplace,iphdr --layout umem
--config 2 --layout umem
--config 5
LIST
