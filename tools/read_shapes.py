#!/usr/bin/env python3
"""Is the same-run ceiling the chip's read rate or one pattern's?  (DESIGN.md
§9 item 1.)  One process, one 4 GiB buffer (far past the 256 MiB Infinity
Cache): bench.py's stream-read ceiling (tools/hbm_probe.hip stream_read, grid
stride, 8 blocks/CU, nontemporal) against wave-contiguous reads
(wave_region_read: each wave streams its own region, 1 KiB per load
instruction, U in flight) over regions, unrolls, blocks per CU and load
policy.  Each leg: `per` back-to-back launches between two events, median
of `reps`, legs interleaved over `rounds`, the lowest median kept.  One JSON
line per leg, sorted, then the best.

    python tools/read_shapes.py [--rounds 3]
"""
import argparse
import ctypes
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--per", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    L = ctypes.CDLL(os.path.join(HERE, "libhbmprobe.so"))
    L.probe_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.probe_wave_region_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nbytes = args.gib << 30
    buf = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=dev)
    out = torch.empty(cus * 64, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    legs = {"grid_stride_8bpc_nt_u1": lambda: L.probe_stream_read(
        buf.data_ptr(), nbytes, out.data_ptr(), cus * 8, 1, 1, s.cuda_stream)}
    for region in (8 << 10, 32 << 10, 128 << 10, 512 << 10):
        for unroll in (4, 8, 16):
            for bpc in (1, 2, 4):
                for nt in (0, 1):
                    name = f"wave_region_{region >> 10}k_u{unroll}_{bpc}bpc{'_nt' if nt else ''}"
                    legs[name] = (lambda r=region, u=unroll, b=bpc, n=nt: L.probe_wave_region_read(
                        buf.data_ptr(), nbytes, r, cus * b, n, u, out.data_ptr(), s.cuda_stream))
    # clocks up
    for _ in range(200):
        legs["grid_stride_8bpc_nt_u1"]()
    torch.cuda.synchronize(dev)
    best = {}
    for rnd in range(args.rounds):
        for name, fn in legs.items():
            ts = []
            for r in range(args.reps + 1):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for k in range(args.per):
                    assert fn() == 0, name
                b.record(s)
                torch.cuda.synchronize(dev)
                ts.append(a.elapsed_time(b) / args.per)
            best[name] = min(best.get(name, 1e9), float(np.median(ts[1:])))
    rows = sorted(best.items(), key=lambda kv: kv[1])
    for name, ms in rows:
        print(json.dumps({"leg": name, "ms": round(ms, 4),
                          "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1)}), flush=True)
    ref = best["grid_stride_8bpc_nt_u1"]
    print(json.dumps({"best": rows[0][0], "best_GBps": round(nbytes / (rows[0][1] * 1e-3) / 1e9, 1),
                      "grid_stride_GBps": round(nbytes / (ref * 1e-3) / 1e9, 1),
                      "best_over_grid_stride": round(ref / rows[0][1], 4)}), flush=True)


if __name__ == "__main__":
    main()
