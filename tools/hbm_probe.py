#!/usr/bin/env python3
"""Achievable streaming-read HBM rate on this GPU (context for the roofline).
Prints one JSON line per (blocks/CU, nt, unroll) and a best line."""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    L = ctypes.CDLL(os.path.join(HERE, "libhbmprobe.so"))
    L.probe_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "--copy":
        return copy_probe(L, dev, cus)
    small = len(sys.argv) > 1 and sys.argv[1] == "--small"
    # --small: a config-3-sized pass (134 MB) rotated over 10 buffers, so
    # nothing is served from the 256 MiB Infinity Cache; else one 2 GiB buffer
    nbytes = (134 << 20) if small else (2 << 30)
    nrot = 10 if small else 1
    bufs = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=dev)
            for _ in range(nrot)]
    out = torch.empty(cus * 32 * 256, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    best = None
    for per_cu in (2, 4, 8, 16):
        for nt in (0, 1):
            for unroll in (1, 2, 4, 8):
                blocks = cus * per_cu
                ts = []
                for r in range(8 * nrot):
                    buf = bufs[r % nrot]
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
                        enable_timing=True)
                    a.record(s)
                    L.probe_stream_read(buf.data_ptr(), nbytes, out.data_ptr(), blocks, nt,
                                        unroll, s.cuda_stream)
                    b.record(s)
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b))
                t = sorted(ts)[len(ts) // 2]
                gbs = nbytes / (t * 1e-3) / 1e9
                rec = {"blocks_per_cu": per_cu, "nt": nt, "unroll": unroll, "ms": round(t, 4),
                       "GBps": round(gbs, 1)}
                print(json.dumps(rec), flush=True)
                if best is None or gbs > best["GBps"]:
                    best = rec
    print(json.dumps({"best_stream_read": best}))


def copy_probe(L, dev, cus):
    """--copy: hand-written read+write stream (the build kernel's copy-mode
    ceiling): 1.5 GB source -> 1.5 GB destination, bytes moved = 2 x size."""
    L.probe_stream_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    nbytes = (1 << 20) * 1472
    src = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    s = torch.cuda.current_stream(dev)
    best = None
    for per_cu in (1, 2, 4, 8):
        for nts in (0, 1):
            for unroll in (1, 2, 4, 8):
                blocks = cus * per_cu
                ts = []
                for r in range(12):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
                        enable_timing=True)
                    a.record(s)
                    rc = L.probe_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, blocks,
                                             nts, unroll, s.cuda_stream)
                    b.record(s)
                    torch.cuda.synchronize()
                    assert rc == 0
                    ts.append(a.elapsed_time(b))
                t = sorted(ts[2:])[len(ts[2:]) // 2]
                gbs = 2 * nbytes / (t * 1e-3) / 1e9
                rec = {"blocks_per_cu": per_cu, "nts": nts, "unroll": unroll, "ms": round(t, 4),
                       "GBps_moved": round(gbs, 1)}
                print(json.dumps(rec), flush=True)
                if best is None or gbs > best["GBps_moved"]:
                    best = rec
    assert torch.equal(src, dst)
    print(json.dumps({"best_stream_copy": best}))


if __name__ == "__main__":
    main()
