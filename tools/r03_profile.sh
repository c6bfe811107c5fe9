#!/bin/bash
# Round 3 end-of-work refresh: host path end to end (threaded staging), then
# the round profile (tools/profile_round.sh).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R03_TAG:-r03p}
tools/gpu_run.sh $t/e2e_config2 300 python tools/bench_e2e.py &&
tools/profile_round.sh $t
