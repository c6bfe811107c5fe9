#!/bin/bash
# SQ counters and HBM bytes: wide receive kernel vs group kernel vs checksum
# kernel VERIFY, config 2 (MTU) and config 5 (jumbo).  Each pass its own run.
set -e
d=${1:-pmcwide}
tools/gpu_run.sh $d/sq2 200 bash tools/pmc_rx.sh 2 gpurun_out/$d/sq2 --geoms "16,6,1,2;32,3,0"
tools/gpu_run.sh $d/sq5 300 bash tools/pmc_rx.sh 5 gpurun_out/$d/sq5 --geoms "64,9,1;64,9,0"
tools/gpu_run.sh $d/bytes2 300 bash tools/pmc_rx_bytes.sh 2 gpurun_out/$d/bytes2 --geoms "16,6,1,2;32,3,0"
