#!/usr/bin/env python3
"""Is the in-place check write cheaper as a second pass?  Times, on config 2
(1M x 1472 B, packed layout, one buffer set): the checksum kernel writing to a
separate array, the same kernel writing udp->check in place, and a scatter of
the separate array's 2-byte results into the frames (torch index_put, an
upper bound for a dedicated kernel).  Timing only.
Usage: python tools/scatter_probe.py [--config 2] [--layout packed|umem]"""
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
    ap.add_argument("--layout", default="packed", choices=["packed", "umem"])
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    cfg = dict(bench.CONFIGS[args.config], id=args.config, layout=args.layout)
    eng = X.Engine(0)
    s = torch.cuda.current_stream(dev)
    desc, d_desc, bufs, out, first, n = bench.build_batch(cfg, 0, 1, torch, dev, eng,
                                                          s.cuda_stream)
    mode = X.MODE_V6 if cfg["family"] == 6 else X.MODE_V4_RFC
    hint = int(desc["len"].mean())
    coff = 60 if cfg["family"] == 6 else 40
    addr = torch.from_numpy(desc["addr"].astype(np.int64)).to(dev)
    assert bool(((addr + coff) % 2 == 0).all().item())
    idx16 = (addr + coff) // 2
    for k in range(200):
        eng.batch_device(bufs[k % len(bufs)], d_desc, n, out, mode, 0, hint, stream=s.cuda_stream)
    torch.cuda.synchronize()

    def timed(fn):
        for k in range(10):
            fn(k)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.reps)]
        for k, (e0, e1) in enumerate(evs):
            e0.record(s)
            fn(k)
            e1.record(s)
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in evs]))

    def to_array(k):
        eng.batch_device(bufs[k % len(bufs)], d_desc, n, out, mode, 0, hint, stream=s.cuda_stream)

    def inplace(k):
        eng.batch_device(bufs[k % len(bufs)], d_desc, n, None, mode, X.F_INPLACE, hint,
                         stream=s.cuda_stream)

    def scatter(k):
        bufs[k % len(bufs)].view(torch.int16)[idx16] = out

    def two_pass(k):
        to_array(k)
        scatter(k)

    for name, fn in (("to_array", to_array), ("inplace", inplace), ("scatter_only", scatter),
                     ("two_pass", two_pass), ("to_array", to_array), ("inplace", inplace)):
        print(json.dumps({"config": args.config, "layout": args.layout, "what": name,
                          "ms": round(timed(fn), 4)}), flush=True)


if __name__ == "__main__":
    main()
