#!/bin/bash
# SQ instruction/wave-cycle counters for the checksum kernel of one config
# (one --pmc pass, kernel-trace only; see MI355X_MICROARCH.md PMC slots).
#   tools/pmc_sq.sh <config> <outdir> [extra bench args]
set -eu
cfg="$1"; out="$2"; shift 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$out" -o run -- \
    python3 bench.py --config "$cfg" --steps 10 --warmup 2 --no-cpu-baseline --no-graph "$@"
