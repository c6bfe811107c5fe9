#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04e}
mkdir -p gpurun_out/$t
tools/gpu_run.sh $t/inplace_probe_c2 300 python tools/inplace_probe.py --family 4 &&
tools/gpu_run.sh $t/inplace_probe_c4 300 python tools/inplace_probe.py --family 6 &&
R04_TAG=$t bash tools/r04_thp.sh
