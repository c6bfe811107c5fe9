#!/bin/bash
# GPU-box runner: each step under its own timeout; stop at the first step that
# faults, aborts, segfaults or times out (124/134/137/139), keep going after a
# plain test failure (exit 1) so the bench still runs.  Logs -> gpurun_out/.
#   tools/gpu_run.sh "<name>" <timeout_s> <cmd...>   (one step)
set -u
mkdir -p gpurun_out
name="$1"; shift
tmo="$1"; shift
log="gpurun_out/${name}.log"
mkdir -p "$(dirname "$log")"
echo "=== $name: $*" > "$log"
start=$(date +%s)
timeout -k 10 "$tmo" "$@" >> "$log" 2>&1
rc=$?
echo "=== $name exit=$rc secs=$(( $(date +%s) - start ))" >> "$log"
echo "$name exit=$rc"
case $rc in
  0|1|5) exit 0 ;;     # ok / test failures / no tests collected
  *) exit $rc ;;       # fault, abort, timeout: stop the chain
esac
