#!/bin/bash
# Order calibration: its tests, then the driver's command with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04u}
mkdir -p gpurun_out/$t
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_abi.py -x -q -k "calibrat or export or symbol" \
  --timeout 300 --timeout-method thread > gpurun_out/$t/pytest.log 2>&1 || { tail -30 gpurun_out/$t/pytest.log; exit 1; }
tail -1 gpurun_out/$t/pytest.log
for r in 1 2; do
  for c in cal nocal; do
    a=""; [ $c = nocal ] && a="--no-calibrate"
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $a > gpurun_out/$t/c2_${c}_$r.log 2>&1 || { tail -5 gpurun_out/$t/c2_${c}_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['frac_vs_ceiling'], d['config'].get('order_calibration'), d['roofline']['order_ab']['fastest'], d['roofline']['order_ab']['auto_vs_fastest'])" gpurun_out/$t/c2_${c}_$r.log
  done
done
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$t/c5_cal.log 2>&1 || { tail -5 gpurun_out/$t/c5_cal.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['frac'], d['config'].get('order_calibration'))" gpurun_out/$t/c5_cal.log
