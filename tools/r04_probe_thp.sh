#!/bin/bash
# In-place schedule probes (no registered memory), then the THP-disabled suite.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04d}
mkdir -p gpurun_out/$t
tools/gpu_run.sh $t/inplace_probe_c2 300 python tools/inplace_probe.py --family 4 &&
tools/gpu_run.sh $t/inplace_probe_c4 300 python tools/inplace_probe.py --family 6 &&
tools/gpu_run.sh $t/inplace_probe_c2_umem 300 python tools/inplace_probe.py --family 4 --layout umem &&
R04_TAG=$t bash tools/r04_thp.sh
