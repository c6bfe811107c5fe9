#!/bin/bash
# SQ instruction/wave-cycle counters for the receive kernel next to the
# checksum kernel's VERIFY mode on the same frames (one --pmc pass).
#   tools/pmc_rx.sh <config> <outdir> [extra bench_rx args]
set -eu
cfg="$1"; out="$2"; shift 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$out" -o run -- \
    python3 tools/bench_rx.py --configs "$cfg" --reps 3 "$@"
