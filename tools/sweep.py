#!/usr/bin/env python3
"""Kernel-geometry sweep for one BASELINE config, in ONE process with
interleaved rounds (cdna_hip_programming.md 5.4 rule 24).  Prints one JSON
line per geometry: median / min kernel time and GB/s of algorithmic bytes.

Usage: python tools/sweep.py --config 2 [--rounds 5] [--launches 20]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libxudp_amd as X  # noqa: E402
import bench  # noqa: E402

GEOMS = X.GEOMETRIES


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--geoms", default="")
    ap.add_argument("--bpc", default="0", help="blocks per CU to try, e.g. 2,3,4 (0: default)")
    ap.add_argument("--orders", default="-1,0",
                    help="visiting orders to try, 'R,T;R,T' (log2 regions, log2 tile frames; "
                         "-1,0 = automatic)")
    ap.add_argument("--claims", default="64,0",
                    help="claimed-tail settings to try, 'S,C;S,C' (XCSUM_TUNE_CLAIM: static "
                         "share in 64ths, wave steps per claim; 64 = static only)")
    ap.add_argument("--shard", default="", help="r/N: time shard r of N of a sharded config")
    ap.add_argument("--layout", default="packed", choices=["packed", "umem"])
    ap.add_argument("--flags", default="", help="comma list of inplace,iphdr,verify,rfc")
    ap.add_argument("--payload", default="", help="MIN,MAX payload bytes instead of the config's")
    args = ap.parse_args()
    fl = {"inplace": X.F_INPLACE, "iphdr": X.F_IPHDR, "verify": X.F_VERIFY}
    flags = sum(fl[f] for f in args.flags.split(",") if f in fl)
    import torch
    dev = torch.device("cuda:0")
    cfg = dict(bench.CONFIGS[args.config], id=args.config, layout=args.layout)
    if args.payload:
        cfg["pmin"], cfg["pmax"] = (int(v) for v in args.payload.split(","))
    eng = X.Engine(0)
    s = torch.cuda.current_stream(dev)
    sr, sn = bench.parse_shard(args.shard) or (0, 1)
    desc, d_desc, bufs, out, first, count = bench.build_batch(cfg, sr, sn, torch, dev, eng,
                                                              s.cuda_stream)
    alg = X.alg_bytes(desc, cfg["family"])
    mode = cfg["mode"]
    if "rfc" in args.flags.split(",") and cfg["family"] == 4:
        mode = X.MODE_V4_RFC
    # "auto": the library's own pick from the batch's mean frame length
    geoms = GEOMS if not args.geoms else [(0, 0, 0) if g == "auto" else
                                          tuple(int(v) for v in g.split(","))
                                          for g in args.geoms.split(";")]
    len_hint = int(desc["len"].mean()) if len(desc) else 0
    bpcs = [int(b) for b in args.bpc.split(",")]
    orders = [tuple(int(v) for v in o.split(",")) for o in args.orders.split(";")]
    claims = [tuple(int(v) for v in c.split(",")) for c in args.claims.split(";")]
    geoms = [(g, b, o, c) for g in geoms for b in bpcs for o in orders for c in claims]
    times = {g: [] for g in geoms}
    for r in range(args.rounds):
        for g, b, o, c in geoms:
            eng.set_geometry(*g) if g[0] else eng.set_geometry(0)
            eng.set_launch(b)
            eng.set_order(*o)
            eng.set_tuning(X.TUNE_CLAIM, *c)
            for k in range(3):
                eng.batch_device(bufs[k % len(bufs)], d_desc, count, out, mode, flags,
                                 len_hint, stream=s.cuda_stream)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.launches)]
            for k in range(args.launches):
                evs[k][0].record(s)
                eng.batch_device(bufs[k % len(bufs)], d_desc, count, out, mode, flags,
                                 len_hint, stream=s.cuda_stream)
                evs[k][1].record(s)
            torch.cuda.synchronize()
            times[(g, b, o, c)] += [e0.elapsed_time(e1) for e0, e1 in evs]
    for g, b, o, c in geoms:
        t = np.array(times[(g, b, o, c)])
        print(json.dumps({"config": args.config, "payload": [cfg["pmin"], cfg["pmax"]],
                          "layout": args.layout, "flags": args.flags,
                          "geometry": g, "bpc": b, "claim": c,
                          "order": o, "median_ms": round(float(
            np.median(t)), 4), "min_ms": round(float(t.min()), 4), "GBps_median": round(
            alg / (np.median(t) * 1e-3) / 1e9, 1), "GBps_best": round(alg / (t.min() * 1e-3) / 1e9,
                                                                      1)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
