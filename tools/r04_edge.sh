#!/bin/bash
# Config 5 A/B: frame-edge chunks temporal (XCSUM_EDGE_TL=1) vs shipped,
# alternating bench runs (parity digest checked by bench.py each run).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
t=${R04_TAG:-r04s}
mkdir -p gpurun_out/$t
B="python -u bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline --no-order-ab"
for r in 1 2; do
  for v in 0 1; do
    XCSUM_EDGE_TL=$v timeout -k 10 300 $B > gpurun_out/$t/c5_edge${v}_$r.log 2>&1 || { tail -5 gpurun_out/$t/c5_edge${v}_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('frac_vs_ceiling'), d.get('parity_digest',{}).get('ok'))" gpurun_out/$t/c5_edge${v}_$r.log
  done
done
