#!/usr/bin/env python3
"""A/B probe for the checksum kernel's VERIFY mode on config-2 frames whose
check fields are (a) 0 as generated, (b) valid RFC checksums written in place
(the receive-side case), (c) written and then zeroed again.  Interleaved
rounds in one process; K back-to-back launches between two events.
Usage: python tools/verify_probe.py [--config 2]   (XCSUM_LIB picks the build)"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import libxudp_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--checks", default="zero,valid,rezeroed",
                    help="which check-field contents to build (comma list)")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    eng = X.Engine(0)
    s = torch.cuda.current_stream(dev)
    cfg = bench.CONFIGS[args.config]
    n, fam = cfg["n"], cfg["family"]
    seed = bench.SEED_BASE ^ args.config
    desc, nbytes = X.gen_layout(n, fam, cfg["pmin"], cfg["pmax"], seed=seed)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    mode = X.MODE_V6 if fam == 6 else X.MODE_V4_RFC
    hint = int(desc["len"].mean())
    bufs = {}
    for name in args.checks.split(","):
        b = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
        eng.gen_fill_device(b, d_desc, n, fam, seed, 0)
        if name != "zero":
            eng.batch_device(b, d_desc, n, None, mode, X.F_INPLACE | X.F_IPHDR, hint)
        if name == "rezeroed":
            off = torch.from_numpy(desc["addr"].astype(np.int64)).to(dev) + (60 if fam == 6 else 40)
            b[off] = 0
            b[off + 1] = 0
        bufs[name] = b
    out = torch.empty(n, dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    first = next(iter(bufs.values()))
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:   # clock ramp
        for _ in range(10):
            eng.batch_device(first, d_desc, n, out, mode, 0, hint, stream=s.cuda_stream)
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    runs = [(b, f) for b in bufs for f in ("none", "verify")]
    times = {r: [] for r in runs}
    K = 20 if args.config != 5 else 3
    for _ in range(args.rounds):
        for (b, f) in runs:
            fl = X.F_VERIFY if f == "verify" else 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(K):
                eng.batch_device(bufs[b], d_desc, n, out, mode, fl, hint, stream=s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            times[(b, f)].append(e0.elapsed_time(e1) / K)
    for (b, f), ts in times.items():
        print(json.dumps({"lib": os.environ.get("XCSUM_LIB", "current"), "config": args.config,
                          "checks": b, "flags": f, "ms": round(float(np.median(ts)), 4)}))


if __name__ == "__main__":
    main()
