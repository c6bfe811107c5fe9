#!/usr/bin/env python3
"""Summarise tools/ab_*_libs.sh output: one row per (layout, config, kernel,
flags, geometry), one column per library log (<lib>_<round>.log), ms.
Usage: python tools/ab_summary.py <dir>..."""
import collections
import glob
import json
import os
import sys

for d in sys.argv[1:]:
    rows = collections.OrderedDict()
    cols = []
    for path in sorted(glob.glob(os.path.join(d, "*.log"))):
        col = os.path.basename(path)[:-4]
        cols.append(col)
        for line in open(path):
            if not line.startswith("{"):
                continue
            r = json.loads(line)
            key = (r.get("layout", ""), r.get("config"), r.get("kernel"), r.get("flags"),
                   r.get("geometry", ""))
            rows.setdefault(key, {})[col] = r.get("ms")
    print(f"== {d}")
    print(" ".join(f"{c:>10}" for c in ["layout", "cfg", "kernel", "flags", "geom"] + cols))
    for key, v in rows.items():
        print(" ".join(f"{str(k):>10}" for k in key) + " " +
              " ".join(f"{v.get(c, float('nan')):>10}" for c in cols))
