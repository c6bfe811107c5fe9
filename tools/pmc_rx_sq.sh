#!/bin/bash
# Two SQ counter passes (instruction mix, then LDS/wait cycles) for the receive
# kernel's VERIFY mode and the checksum kernel's VERIFY mode on the same
# frames.  tools/pmc_rx_sq.sh <config> <outdir>
set -eu
cfg="$1"; out="$2"
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
    --output-format csv -d "$out/p1" -o run -- \
    python3 tools/bench_rx.py --configs "$cfg" --reps 2 --only verify,csum_verify
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM \
    --output-format csv -d "$out/p2" -o run -- \
    python3 tools/bench_rx.py --configs "$cfg" --reps 2 --only verify,csum_verify
