#!/usr/bin/env python3
"""Receive kernel (config 2, VERIFY) with the record buffer and the frame
buffer at different offsets inside larger allocations, in one process: is
the box-to-box / process-to-process spread a placement effect?
Usage: python tools/rx_offset_probe.py [--config 2] [--layout packed|umem]"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import libxudp_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--layout", default="packed", choices=["packed", "umem"])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    eng = X.Engine(0)
    s = torch.cuda.current_stream(dev)
    cfg = bench.CONFIGS[args.config]
    n, fam = cfg["n"], cfg["family"]
    seed = bench.SEED_BASE ^ args.config
    kw = dict(stride=4096, offset=322 if fam == 6 else 342) if args.layout == "umem" else {}
    desc, nbytes = X.gen_layout(n, fam, cfg["pmin"], cfg["pmax"], seed=seed, **kw)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    SLACK = 8 << 20
    nrot = max(1, math.ceil((1 << 30) / nbytes))
    big = [torch.empty(nbytes + SLACK + 64, dtype=torch.uint8, device=dev) for _ in range(nrot)]
    eng.gen_fill_device(big[0], d_desc, n, fam, seed, 0)
    mode = X.MODE_V6 if fam == 6 else X.MODE_V4_RFC
    eng.batch_device(big[0], d_desc, n, None, mode, X.F_INPLACE | X.F_IPHDR)
    src = big[0][:nbytes + 64].clone()
    msgs_big = torch.empty(n * 64 + SLACK, dtype=torch.uint8, device=dev)
    d_out = torch.empty(n, dtype=torch.int16, device=dev)
    hint = int(desc["len"].mean())
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(10):
            eng.batch_device(src, d_desc, n, d_out, mode, X.F_VERIFY, hint, stream=s.cuda_stream)
        torch.cuda.synchronize()
    K = 20
    for foff in (0, 4096, 1 << 20):
        for b in big:
            b[foff:foff + nbytes + 64].copy_(src)
        umems = [b[foff:] for b in big]
        for moff in (0, 256, 4096, 65536, 1 << 20, (3 << 20) + 4096):
            msgs = msgs_big[moff:moff + n * 64]
            ts = []
            for r in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for k in range(K):
                    eng.rx_device(umems[k % nrot], d_desc, n, msgs, None, X.F_VERIFY, hint,
                                  stream=s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / K)
            print(json.dumps({"config": args.config, "layout": args.layout, "frames_off": foff,
                              "msgs_off": moff, "ms": round(float(np.median(ts)), 4),
                              "umem_addr_mod_2M": umems[0].data_ptr() % (2 << 20),
                              "msgs_addr_mod_2M": msgs.data_ptr() % (2 << 20)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
