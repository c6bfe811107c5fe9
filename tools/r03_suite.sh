#!/bin/bash
# Round 3 GPU check: a pinning diagnostic (does the runtime pin pageable
# buffers in place), the product suite, the suite under the bounds-checked
# debug build, a same-box A/B of this library against round 2's on configs 2
# and 3, and the in-place bench.  Each step under its own time limit; the
# chain stops at a fault.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/${R03_TAG:-r03c}
mkdir -p "$out"
AMD_LOG_LEVEL=4 timeout -k 10 120 python tools/diag_pinning.py > "$out/diag_pinning.out" \
    2> "$out/diag_pinning.raw" ; rc=$?
grep -aE "=== MARK|Pinned|pinned|Staged|staged|Unpinned" "$out/diag_pinning.raw" | cut -c1-300 \
    > "$out/diag_pinning.log" || true
rm -f "$out/diag_pinning.raw"
echo "diag exit=$rc" >> "$out/diag_pinning.log"
case $rc in 0|1) ;; *) exit $rc ;; esac
P="python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
tools/gpu_run.sh "${out#gpurun_out/}/pytest_gpu" 600 $P &&
XCSUM_LIB=$PWD/libxudp_amd/debug/libxcsum.so tools/gpu_run.sh "${out#gpurun_out/}/pytest_gpu_debug" 900 $P &&
tools/ab_bench.sh "${out#gpurun_out/}/ab" 2 "--config 2;--config 3" new=libxudp_amd/libxcsum.so \
    r02=libxudp_amd/variants/r02/libxcsum.so &&
tools/gpu_run.sh "${out#gpurun_out/}/bench_inplace_c2" 240 python bench.py --steps 100 --warmup 5 \
    --no-cpu-baseline --flags inplace,iphdr
