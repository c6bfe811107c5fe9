#!/bin/bash
# VERIFY's new dense order (descriptor order) vs the old automatic (3,4).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04vo}
mkdir -p gpurun_out/$t
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rx.py tests/test_gpu_fuzz.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/$t/pytest.log 2>&1 || { tail -20 gpurun_out/$t/pytest.log; exit 1; }
tail -1 gpurun_out/$t/pytest.log
i=0
while read -r a; do
  for r in 1 2 3; do
    for o in auto 3,4; do
      i=$((i+1))
      if [ $o = auto ]; then env_o=""; else env_o="XCSUM_ORDER=$o"; fi
      env $env_o timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-order-ab --no-calibrate $a > gpurun_out/$t/b$i.log 2>&1 || { echo "FAIL: $a $o"; tail -5 gpurun_out/$t/b$i.log; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], '|', d['ms_per_step'], d['roofline'].get('frac_vs_ceiling'), d.get('parity_ok'))" gpurun_out/$t/b$i.log "$a $o"
    done
  done
done <<'LIST'
--config 2 --flags verify
--config 4 --flags verify
LIST
