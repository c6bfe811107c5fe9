#!/usr/bin/env python3
"""Per-leg PMC summary of the per-leg rocprofv3 passes (round 4:
profiles/run_scripts.bundle.txt r04_inplace_pmc.sh; round 5: tools/run_session.sh
<tag> iphdr_pmc): for every
<leg>_<counter>/run_counter_collection.csv under a directory, the mean per
dispatch of each counter, per kernel (FETCH_SIZE / WRITE_SIZE in KiB as
rocprofv3 reports them; FETCH_SIZE counts half the bytes of a wide streaming
read on gfx950, MI355X_MICROARCH.md).  Prints JSON.

    python tools/pmc_legs.py gpurun_out/r04h/pmc > profiles/r04/inplace/r04h_pmc_legs.json
"""
import collections
import csv
import glob
import json
import os
import sys


def main(root):
    out = {}
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        leg = os.path.basename(os.path.dirname(f))
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not any(t in k for t in ("stream_read", "csum_kernel", "scatter", "iphdr_kernel", "line_halves",
                                        "header_touch",
                                        "build_hdr_kernel")):
                continue
            per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for (k, _), cs in per.items():
            for c, v in cs.items():
                agg[k][c].append(v)
        for k, cs in agg.items():
            out.setdefault(leg, {})[k] = {c: round(sum(v) / len(v), 1) for c, v in cs.items()}
            out[leg][k]["dispatches"] = len(next(iter(cs.values())))
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
