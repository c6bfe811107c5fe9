#!/usr/bin/env python3
"""Print the medians of tools/ab_libs.sh logs: python tools/ab_show.py <tag>"""
import glob
import json
import sys

tag = sys.argv[1]
for path in sorted(glob.glob(f"gpurun_out/{tag}_*.log")):
    rows = [json.loads(x) for x in open(path) if x.startswith("{")]
    print(path.split("/")[-1][:-4], " ".join(
        f"{tuple(r['geometry'])}/{r['bpc']}:{r['GBps_median']:.0f}" for r in rows))
