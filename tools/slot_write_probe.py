#!/usr/bin/env python3
"""The IPv4 in-place build's stores alone (tools/hbm_probe.hip
probe_slot_write): 1M xudp slots (4096 bytes, eth at F+342), per slot the 42
header bytes (one 64-byte block), optionally the coalesced 16-byte
descriptor write and 16-byte message load the build kernel also makes.
UMEMs rotated between launches (the touched blocks would stay in the
Infinity Cache), `per` launches between two events, median of `reps`, best
of `rounds`.  Beside it, xcsum_build_device in place (build_hdr_kernel) on
the same UMEMs, interleaved.  One JSON line.

    python tools/slot_write_probe.py [--rot 4]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libxudp_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--rot", type=int, default=4)
    ap.add_argument("--per", type=int, default=20)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    n = args.n
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbmprobe.so"))
    fn = L.probe_slot_write
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_void_p]
    umems = [torch.zeros(n * 4096, dtype=torch.uint8, device=dev) for _ in range(args.rot)]
    d_desc = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    eng = X.Engine(0)
    route = X.make_route(4, b"\x02\0\0\0\0\x01", b"\x02\0\0\0\0\x02", bytes([10, 0, 35, 2]), 3486,
                         bytes([10, 0, 35, 1]), 40000)
    msgs = np.zeros(n, dtype=X.MSG_DTYPE)
    msgs["len"] = 1472
    msgs["slot"] = np.arange(n, dtype=np.uint32)
    d_msgs = torch.from_numpy(msgs.view(np.uint8)).to(dev)
    s = torch.cuda.current_stream(dev)

    def leg(name, k):
        u = umems[k % len(umems)]
        if name == "build":
            eng.build_device(route, d_msgs, d_msgs, n, u, 4096, 384, d_desc, None,
                             X.F_BUILD_INPLACE, 1472, s.cuda_stream)
            return
        desc, m = {"hdr": (0, 0), "hdr_desc": (1, 0), "hdr_desc_msg": (1, 1)}[name]
        assert fn(u.data_ptr(), n, desc, m, d_msgs.data_ptr(), d_desc.data_ptr(),
                  s.cuda_stream) == 0

    legs = ["hdr", "hdr_desc", "hdr_desc_msg", "build"]
    for k in range(200):
        for g in legs:
            leg(g, k)
    torch.cuda.synchronize(dev)
    best = {}
    for _ in range(args.rounds):
        for g in legs:
            ts = []
            for _ in range(args.reps):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for k in range(args.per):
                    leg(g, k)
                e1.record(s)
                torch.cuda.synchronize(dev)
                ts.append(e0.elapsed_time(e1) / args.per)
            best[g] = min(best.get(g, 1e9), float(np.median(ts)))
    print(json.dumps({"frames": n, "rotating_umems": args.rot,
                      "us": {g: round(v * 1e3, 2) for g, v in best.items()},
                      "build_vs_probe": round(best["build"] / best["hdr_desc_msg"], 3)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
