#!/bin/bash
# HBM bytes of the receive kernel next to the checksum kernel's VERIFY mode
# (FETCH_SIZE and WRITE_SIZE in separate passes).
#   tools/pmc_rx_bytes.sh <config> <outdir> [extra bench_rx args]
set -eu
cfg="$1"; out="$2"; shift 2
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$out/$c" -o run -- \
      python3 tools/bench_rx.py --configs "$cfg" --reps 3 "$@"
done
