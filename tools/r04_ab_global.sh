#!/bin/bash
# Same-box A/B, HEAD's library (variants/head: flat loads in the IPHDR,
# VERIFY, resident and receive kernels) vs the working tree's (global loads):
# RX bench, in-place and plain config 2, after the GPU tests of those paths.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04p}
mkdir -p gpurun_out/$t
V=$PWD/libxudp_amd/variants/head/libxcsum.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inplace.py tests/test_gpu_rx.py \
  tests/test_gpu_resident.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/$t/pytest.log 2>&1 || { tail -30 gpurun_out/$t/pytest.log; exit 1; }
tail -1 gpurun_out/$t/pytest.log
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-order-ab"
run() {
  local n=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then XCSUM_LIB=$lib timeout -k 10 200 "$@" > gpurun_out/$t/$n.log 2>&1
  else timeout -k 10 200 "$@" > gpurun_out/$t/$n.log 2>&1; fi
  local rc=$?
  [ $rc -eq 0 ] || { echo "$n rc $rc"; tail -5 gpurun_out/$t/$n.log; exit $rc; }
}
for r in 1 2; do
  run rx_head_$r $V python -u tools/bench_rx.py --configs 2,3,4 --reps 5
  run rx_new_$r "" python -u tools/bench_rx.py --configs 2,3,4 --reps 5
  run c2ip_head_$r $V $B --flags inplace,iphdr
  run c2ip_new_$r "" $B --flags inplace,iphdr
  run c2_head_$r $V $B
  run c2_new_$r "" $B
done
for f in gpurun_out/$t/c2*.log; do
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['roofline']['frac'])" $f
done
for f in gpurun_out/$t/rx_*.log; do
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[1].split('/')[-1], d.get('config'), d.get('kernel'), d.get('flags'), d.get('geometry'), d['ms'], d['pct_hbm_peak'])" $f
done
