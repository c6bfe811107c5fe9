#!/usr/bin/env python3
"""Per-kernel medians of rocprofv3 --pmc counters (one CSV dir or file per
argument): prints one JSON line per (file, kernel).
Usage: python tools/sq_summary.py <counter_collection.csv | dir>... [--kernel REGEX]"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import statistics


def rows(path):
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*counter_collection*.csv"), recursive=True)
    for fp in files:
        with open(fp) as f:
            yield from csv.DictReader(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--kernel", default=r"csum_(stream_|seg_)?kernel|rx_(wide_)?kernel")
    args = ap.parse_args()
    kre = re.compile(args.kernel)
    for p in args.paths:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in rows(p):
            k = r.get("Kernel_Name", "")
            if not kre.search(k):
                continue
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            names[key] = k
        byk = collections.defaultdict(list)
        for key, c in per.items():
            byk[names[key]].append(c)
        for k, lst in byk.items():
            cn = sorted({n for c in lst for n in c})
            med = {n: statistics.median(c.get(n, 0.0) for c in lst) for n in cn}
            print(json.dumps({"file": p, "kernel": k[:80], "dispatches": len(lst), **med}))


if __name__ == "__main__":
    main()
