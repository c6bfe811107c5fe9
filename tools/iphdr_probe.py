#!/usr/bin/env python3
"""Same-run legs of libxudp's IPv4 TX call on the device (xcsum_batch_device
with XCSUM_F_IPHDR_ONLY, csrc/xcsum_iphdr.hip) on BASELINE config 2's frames,
packed (1520-byte stride) and in xudp's 4096-byte slots: in place and/or
into a result array, frames per thread (XCSUM_TUNE_IPHDR_FPT), visiting orders.
Each leg: `per` back-to-back launches between two events, median of `reps`,
legs interleaved over `rounds` rounds, the lowest median kept.
One JSON line per layout.

    python tools/iphdr_probe.py [--layouts packed,slots] [--legs ...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import libxudp_amd as X  # noqa: E402

# name -> (flags, with result array, FPT, order or None)
LEGS = {
    "inplace": (X.F_INPLACE, False, "4", None),
    "inplace_out": (X.F_INPLACE, True, "4", None),
    "out_only": (0, True, "4", None),
    "fpt1": (X.F_INPLACE, False, "1", None),
    "fpt2": (X.F_INPLACE, False, "2", None),
    "fpt8": (X.F_INPLACE, False, "8", None),
    "ord0": (X.F_INPLACE, False, "4", (0, 0)),
    "ord54": (X.F_INPLACE, False, "4", (5, 4)),
    "ord34": (X.F_INPLACE, False, "4", (3, 4)),
    "ord46": (X.F_INPLACE, False, "4", (4, 6)),
    "ord28": (X.F_INPLACE, False, "4", (2, 8)),
}
# sweep legs "f<FPT>o<R>_<T>": in place, FPT frames per thread, order R,T
for _f in ("1", "2", "4", "8"):
    for _o in ((0, 0), (3, 4), (5, 4), (4, 6)):
        LEGS[f"f{_f}o{_o[0]}_{_o[1]}"] = (X.F_INPLACE, False, _f, _o)
        LEGS[f"out_f{_f}o{_o[0]}_{_o[1]}"] = (0, True, _f, _o)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layouts", default="packed,slots")
    ap.add_argument("--legs", default=",".join(LEGS))
    ap.add_argument("--per", type=int, default=50)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--mode", type=int, default=X.MODE_V4_LEGACY)
    ap.add_argument("--rot", type=int, default=8,
                    help="buffers rotated between launches: the header lines of one batch "
                         "(~130 MB) would stay in the 256 MiB Infinity Cache")
    ap.add_argument("--warm", type=int, default=2000, help="launches to bring the clocks up")
    ap.add_argument("--no-ref", dest="ref", action="store_false",
                    help="no reference pass (PMC runs: only the legs' dispatches)")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    eng = X.Engine(0)
    cfg = dict(bench.CONFIGS[2], id=2)
    s = torch.cuda.current_stream(dev)
    legs = [k for k in args.legs.split(",") if k]
    for layout in args.layouts.split(","):
        kw = dict(stride=4096, offset=342) if layout == "slots" else {}
        desc, nbytes = X.gen_layout(cfg["n"], 4, 1472, 1472, seed=bench.SEED_BASE ^ 2, **kw)
        d_desc = torch.from_numpy(desc.view(np.uint8)).pin_memory().to(dev)
        bufs = [torch.zeros(nbytes + 64, dtype=torch.uint8, device=dev) for _ in range(args.rot)]
        eng.gen_fill_device(bufs[0], d_desc, cfg["n"], 4, bench.SEED_BASE ^ 2, 0,
                            stream=s.cuda_stream)
        for b in bufs[1:]:
            b.copy_(bufs[0])
        buf = bufs[0]
        out = torch.zeros(cfg["n"], dtype=torch.int16, device=dev)
        ref = torch.zeros_like(out)
        if args.ref:
            eng.batch_device(buf, d_desc, cfg["n"], ref, args.mode, X.F_IPHDR_ONLY, 0,
                             stream=s.cuda_stream)
        # clocks up
        for k in range(args.warm):
            eng.batch_device(bufs[k % len(bufs)], d_desc, cfg["n"], None, args.mode,
                             X.F_IPHDR_ONLY | X.F_INPLACE, 0, stream=s.cuda_stream)
        torch.cuda.synchronize(dev)
        best = {}
        for rnd in range(args.rounds):
            for leg in legs:
                flags, with_out, fpt, order = LEGS[leg]
                eng.set_tuning(X.TUNE_IPHDR_FPT, int(fpt))
                eng.set_order(*(order or (-1, 0)))
                o = out if with_out else None
                ts = []
                for r in range(args.reps):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for k in range(args.per):
                        eng.batch_device(bufs[k % len(bufs)], d_desc, cfg["n"], o, args.mode,
                                         X.F_IPHDR_ONLY | flags, 0, stream=s.cuda_stream)
                    e1.record(s)
                    torch.cuda.synchronize(dev)
                    ts.append(e0.elapsed_time(e1) / args.per)
                best[leg] = min(best.get(leg, 1e9), float(np.median(ts)))
                if with_out and args.ref:
                    assert torch.equal(out, ref), leg
        eng.set_order(-1, 0)
        eng.set_tuning(X.TUNE_IPHDR_FPT, 4)
        real = bench.real_bytes(desc, X.F_IPHDR_ONLY)
        print(json.dumps({"layout": layout, "frames": cfg["n"], "real_bytes": real,
                          "rotating_buffers": args.rot,
                          "us": {k: round(v * 1e3, 2) for k, v in best.items()},
                          "gpps": {k: round(cfg["n"] / (v * 1e-3) / 1e9, 2)
                                   for k, v in best.items()}}), flush=True)
        del buf, bufs
    eng.close()


if __name__ == "__main__":
    main()
