#!/bin/bash
# HBM bytes of one command's kernels: separate FETCH_SIZE and WRITE_SIZE
# passes (MI355X_MICROARCH.md: one TCC counter family per pass), kernel trace
# only.  Summarise with tools/sq_summary.py <outdir>/fetch <outdir>/write.
#   tools/pmc_bytes.sh <outdir> <command...>
set -eu
out="$1"; shift
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- "$@" > "$out.fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- "$@" > "$out.write.log" 2>&1
