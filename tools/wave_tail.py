#!/usr/bin/env python3
"""The persistent checksum grid's tail: every
wave's start and end stamp (the `make variant NAME=stamps
DEFS=-DXCSUM_WAVE_STAMPS` build, s_memrealtime at the top and bottom of
csum_loop) for one launch on a bench workload, after the clocks are up.

Per launch: span = last end - first start; busy = sum of (end - start);
occupancy loss = 1 - busy / (waves x span), the share of the launch's
wave-slots left idle by waves that finished early -- the tail; plus when
the first wave ended, when 50 / 90 % had, and the kernel's event time.
Median of `--reps` launches.  One JSON line per workload.

    XCSUM_LIB=libxudp_amd/variants/stamps/libxcsum.so \\
        python tools/wave_tail.py --work c2 c5 c5s0/8 c5s7/8
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STAMPS = os.path.join(ROOT, "libxudp_amd", "variants", "stamps", "libxcsum.so")
os.environ.setdefault("XCSUM_LIB", STAMPS)

import bench  # noqa: E402
import libxudp_amd as X  # noqa: E402


def parse_work(w):
    """c2 -> (2, None); c5s7/8 -> (5, (7, 8))"""
    cid = int(w[1:].split("s")[0])
    shard = None
    if "s" in w:
        r, n = w.split("s")[1].split("/")
        shard = (int(r), int(n))
    return cid, shard


def stats(st, tick_ns=10.0):
    st = st.reshape(-1, 2)
    st = st[(st[:, 0] != 0) & (st[:, 1] >= st[:, 0])]
    t0, t1 = int(st[:, 0].min()), int(st[:, 1].max())
    span = (t1 - t0) * tick_ns / 1e3                       # us
    busy = float((st[:, 1] - st[:, 0]).sum()) * tick_ns / 1e3
    ends = np.sort((st[:, 1] - t0) * tick_ns / 1e3)
    starts = (st[:, 0] - t0) * tick_ns / 1e3
    n = len(st)
    return {"waves": n, "span_us": round(span, 2),
            "occupancy_loss": round(1 - busy / (n * span), 4) if span else None,
            "last_start_us": round(float(starts.max()), 2),
            "first_end_us": round(float(ends[0]), 2),
            "p50_end_us": round(float(ends[n // 2]), 2),
            "p90_end_us": round(float(ends[int(n * 0.9)]), 2),
            "tail_after_p90_frac": round(float((span - ends[int(n * 0.9)]) / span), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--work", nargs="+", default=["c2", "c5", "c5s0/8", "c5s7/8"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warm", type=int, default=40)
    ap.add_argument("--claim", default="64,0",
                    help="XCSUM_TUNE_CLAIM static share in 64ths, wave steps per claim")
    args = ap.parse_args()
    import torch
    L = X.lib()
    fn = getattr(L, "xcsum_wave_stamps", None)
    if fn is None:
        sys.exit(f"{X.LIB_PATH} has no wave stamps: make -C libxudp_amd variant NAME=stamps "
                 f"DEFS=-DXCSUM_WAVE_STAMPS")
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    eng = X.Engine(0)
    eng.set_tuning(X.TUNE_CLAIM, *[int(v) for v in args.claim.split(",")])
    s = torch.cuda.current_stream(dev)
    for w in args.work:
        cid, shard = parse_work(w)
        cfg = dict(bench.CONFIGS[cid], id=cid, layout="packed")
        r, n = shard if shard else (0, 1)
        desc, d_desc, bufs, out, first, count = bench.build_batch(cfg, r, n, torch, dev, eng,
                                                                  s.cuda_stream)
        hint = int(desc["len"].mean())
        for k in range(args.warm):
            eng.batch_device(bufs[k % len(bufs)], d_desc, count, out, cfg["mode"], 0, hint,
                             stream=s.cuda_stream)
        host = np.zeros(2 * 65536, dtype=np.uint64)
        rows = []
        for k in range(args.reps):
            assert fn(None, 65536, 1) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            eng.batch_device(bufs[k % len(bufs)], d_desc, count, out, cfg["mode"], 0, hint,
                             stream=s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize(dev)
            assert fn(host.ctypes.data, 65536, 0) == 0
            st = stats(host)
            st["event_ms"] = round(e0.elapsed_time(e1), 4)
            # the stamps' clock is taken as 100 MHz: span / event time checks it
            st["span_over_event"] = round(st["span_us"] / 1e3 / st["event_ms"], 4)
            rows.append(st)
        med = {k: float(np.median([r_[k] for r_ in rows])) for k in rows[0]}
        frames_per_wave = count / med["waves"]
        print(json.dumps({"work": w, "claim": args.claim, "frames": count, "frames_per_wave": round(frames_per_wave, 1),
                          "median": med, "reps": rows}), flush=True)
        del bufs, d_desc, out
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
