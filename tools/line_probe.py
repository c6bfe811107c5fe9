#!/usr/bin/env python3
"""Request-size calibration for scattered accesses (tools/hbm_probe.hip
probe_line_halves): N lines at a fixed stride, one dword read from the first
64-byte half, the second, or both, of each 128-byte line.  Run under
rocprofv3 --pmc with the L2's memory-side request counters (tools/
run_session.sh <tag> line_probe): requests per line for one half vs both
say how many bytes a scattered access fetches; timings printed as JSON.

    python tools/line_probe.py [--lines 4194304] [--stride 1536] [--halves 1,2,3]
"""
import argparse
import ctypes
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=4 << 20)
    ap.add_argument("--stride", type=int, default=1536)
    ap.add_argument("--halves", default="1,2,3")
    ap.add_argument("--per", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbmprobe.so"))
    fn = L.probe_line_halves
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_void_p]
    buf = torch.ones(args.lines * args.stride + 256, dtype=torch.uint8, device=dev)
    out = torch.zeros((args.lines + 255) // 256, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    res = {}
    for h in [int(x) for x in args.halves.split(",")]:
        ts = []
        for r in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.per):
                assert fn(buf.data_ptr(), args.lines, args.stride, h, out.data_ptr(),
                          s.cuda_stream) == 0
            e1.record(s)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1) / args.per)
        ms = float(np.median(ts))
        res[f"halves{h}"] = {"us": round(ms * 1e3, 2),
                             "Glines_per_s": round(args.lines / (ms * 1e-3) / 1e9, 2)}
    print(json.dumps({"lines": args.lines, "stride": args.stride, **res}), flush=True)


if __name__ == "__main__":
    main()
