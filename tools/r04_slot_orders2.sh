#!/bin/bash
# The new automatic in-place order for sparse batches vs the old one (5,4)
# forced, alternating; plus the in-place tests.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04so2}
mkdir -p gpurun_out/$t
timeout -k 10 400 python -u -m pytest tests/test_gpu_inplace.py tests/test_gpu_host_path.py tests/test_gpu_config1.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/$t/pytest.log 2>&1 || { tail -20 gpurun_out/$t/pytest.log; exit 1; }
tail -1 gpurun_out/$t/pytest.log
i=0
while read -r a; do
  for r in 1 2; do
    for o in auto 5,4; do
      i=$((i+1))
      if [ $o = auto ]; then env_o=""; else env_o="XCSUM_ORDER=$o"; fi
      env $env_o timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-order-ab --no-calibrate --layout umem $a > gpurun_out/$t/b$i.log 2>&1 || { echo "FAIL: $a $o"; tail -5 gpurun_out/$t/b$i.log; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], '|', d['ms_per_step'], d['roofline'].get('frac_vs_ceiling'), d.get('parity_ok'))" gpurun_out/$t/b$i.log "$a $o"
    done
  done
done <<'LIST'
--config 2 --flags inplace,iphdr
--config 4 --flags inplace
--config 2 --flags inplace
LIST
