#!/usr/bin/env python3
"""The header-only access pattern alone (tools/hbm_probe.hip
probe_header_touch_mode): per frame the 16-byte descriptor, the seven header
dwords at (eth+12)&~3 and optionally a 2-byte store at eth+24 (write 1) or a blind store of the
whole 32-byte sector / 64-byte block / 128-byte line holding it (write 2/3/4), or
the 2-byte store nontemporal / sc0 sc1 / nt (write 5/6/7), no arithmetic,
over BASELINE config 2's frames packed and in xudp's slots -- with the
header loads plain (mode 0, as the library's XCSUM_F_IPHDR_ONLY kernel),
nontemporal (1) or with the cache-policy bits nt / sc1 / sc0 sc1 (2-4).
Legs interleaved over rounds, `per` launches between two events, median of
`reps`, the lowest median kept.  One JSON line per layout.

    python tools/header_probe.py [--modes 0,1,2,3,4] [--layouts packed,slots]
"""
import argparse
import ctypes
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
    ap.add_argument("--layouts", default="packed,slots")
    ap.add_argument("--modes", default="0,1,2,3,4")
    ap.add_argument("--writes", default="0,1")
    ap.add_argument("--per", type=int, default=50)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rot", type=int, default=8,
                    help="buffers rotated between launches: the header lines of one batch "
                         "(~130 MB) would stay in the 256 MiB Infinity Cache")
    ap.add_argument("--warm", type=int, default=2000)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbmprobe.so"))
    fn = L.probe_header_touch_mode
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_void_p]
    eng = X.Engine(0)
    s = torch.cuda.current_stream(dev)
    n = bench.CONFIGS[2]["n"]
    scratch = torch.zeros((n + 1023) // 1024, dtype=torch.int32, device=dev)
    modes = [int(m) for m in args.modes.split(",")]
    writes = [int(w) for w in args.writes.split(",")]
    for layout in args.layouts.split(","):
        kw = dict(stride=4096, offset=342) if layout == "slots" else {}
        desc, nbytes = X.gen_layout(n, 4, 1472, 1472, seed=bench.SEED_BASE ^ 2, **kw)
        d_desc = torch.from_numpy(desc.view(np.uint8)).pin_memory().to(dev)
        bufs = [torch.zeros(nbytes + 64, dtype=torch.uint8, device=dev) for _ in range(args.rot)]
        eng.gen_fill_device(bufs[0], d_desc, n, 4, bench.SEED_BASE ^ 2, 0, stream=s.cuda_stream)
        for b in bufs[1:]:
            b.copy_(bufs[0])
        for k in range(args.warm):
            assert fn(bufs[k % len(bufs)].data_ptr(), d_desc.data_ptr(), n, 1, 0, scratch.data_ptr(),
                      s.cuda_stream) == 0
        torch.cuda.synchronize(dev)
        best = {}
        for rnd in range(args.rounds):
            for m in modes:
                for w in writes:
                    ts = []
                    for r in range(args.reps):
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(s)
                        for k in range(args.per):
                            assert fn(bufs[k % len(bufs)].data_ptr(), d_desc.data_ptr(), n, w, m,
                                      scratch.data_ptr(), s.cuda_stream) == 0
                        e1.record(s)
                        torch.cuda.synchronize(dev)
                        ts.append(e0.elapsed_time(e1) / args.per)
                    k = f"mode{m}_w{w}"
                    best[k] = min(best.get(k, 1e9), float(np.median(ts)))
        print(json.dumps({"layout": layout, "frames": n, "rotating_buffers": args.rot,
                          "us": {k: round(v * 1e3, 2) for k, v in best.items()}}), flush=True)
        del bufs
    eng.close()


if __name__ == "__main__":
    main()
