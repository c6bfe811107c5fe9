#!/bin/bash
# In-place write cost on one box: the probe legs (whole-block stores
# included), then PMC passes on single legs -- FETCH_SIZE, WRITE_SIZE and the
# L2's memory-side request counts -- each in its own rocprofv3 run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t=${R04_TAG:-r04h}
mkdir -p gpurun_out/$t/pmc
tools/gpu_run.sh $t/inplace_probe_c2 300 python tools/inplace_probe.py --family 4 &&
tools/gpu_run.sh $t/inplace_probe_c4 300 python tools/inplace_probe.py --family 6 || exit $?
for leg in lib_plain lib_fused read read+w2 fused_nt fused_blk64 fused_blk128; do
  for pmc in FETCH_SIZE WRITE_SIZE "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    tag=$(echo "$pmc" | cut -d' ' -f1)
    d=gpurun_out/$t/pmc/${leg/+/_}_$tag
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $d -o run -- \
      python3 tools/inplace_probe.py --family 4 --legs "$leg" --rounds 1 > $d.log 2>&1
    rc=$?
    echo "pmc $leg $tag rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
