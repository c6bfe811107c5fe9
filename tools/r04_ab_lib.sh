#!/bin/bash
# (Historical: needs libxudp_amd/variants/head/libxcsum.so built from commit
# 38cefbc, not kept in the tree; it produced profiles/r04/inplace/r04n_* and r04p_*.)
# Same-box A/B of the in-place passes: HEAD's library (variants/head) vs the
# working tree's, alternating bench runs, then the interleaved probe.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04n}
mkdir -p gpurun_out/$t
V=$PWD/libxudp_amd/variants/head/libxcsum.so
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-order-ab"
run() { # name, lib or "", args...
  local n=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    XCSUM_LIB=$lib timeout -k 10 200 $B "$@" > gpurun_out/$t/$n.log 2>&1
  else
    timeout -k 10 200 $B "$@" > gpurun_out/$t/$n.log 2>&1
  fi
  local rc=$?
  [ $rc -eq 0 ] || { echo "$n rc $rc"; tail -5 gpurun_out/$t/$n.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['ms_per_step'], d.get('roofline',{}).get('frac'))" gpurun_out/$t/$n.log $n
}
timeout -k 10 400 python -u -m pytest tests/test_gpu_inplace.py tests/test_gpu_parity.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/$t/pytest.log 2>&1 || { tail -30 gpurun_out/$t/pytest.log; exit 1; }
tail -1 gpurun_out/$t/pytest.log
for r in 1 2; do
  run c2ip_head_$r $V --flags inplace,iphdr
  run c2ip_new_$r "" --flags inplace,iphdr
  run c4ip_head_$r $V --config 4 --flags inplace
  run c4ip_new_$r "" --config 4 --flags inplace
done
L=lib_plain,lib_fused,read+blind64,read+copy64
for fam in 4 6; do
  timeout -k 10 240 python -u tools/inplace_probe.py --family $fam --legs $L --rounds 3 \
    >> gpurun_out/$t/probe.log 2>&1 || exit $?
done
grep ms_per gpurun_out/$t/probe.log
