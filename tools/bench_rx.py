#!/usr/bin/env python3
"""Throughput of xcsum_rx_device (xudp_nic_recv_channel's per-frame work on
the GPU, csrc/xcsum_rx.hip) on BASELINE-sized batches of received frames.

Frames: the bench generator's packed layout (configs 2/3/4: 1M x 1472 B
IPv4, 1M x 64 B IPv4, 1M x 1472 B IPv6), checksummed in place by the TX
kernel (RFC rules, IPv4 header too) so every frame verifies.  Batches under
1 GiB are replicated and rotated (no pass served by the Infinity Cache).

Bytes moved per frame: descriptor 16 + record 64 + the frame bytes the
kernel must read -- the whole frame with XCSUM_F_VERIFY, the 64-byte header
line without.  For comparison the checksum kernel's VERIFY mode (2-byte
result instead of the 64-byte record) runs on the same buffers.
One JSON line per (config, flags, geometry), all modes timed in interleaved
rounds in one process after a >= 300 ms clock ramp; vs_csum_verify = time /
the checksum kernel's VERIFY time in the same rounds.
Usage: python tools/bench_rx.py [--configs 2,3,4] [--geoms "auto;4,2,1;16,6,1"]"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import libxudp_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,4")
    ap.add_argument("--geoms", default="auto")
    ap.add_argument("--reps", type=int, default=7, help="interleaved rounds")
    ap.add_argument("--no-count", action="store_true", help="pass d_count = NULL")
    ap.add_argument("--reverse", action="store_true", help="time the modes in reverse order")
    ap.add_argument("--layout", default="packed", choices=["packed", "umem"],
                    help="frames packed (default) or one per 4096-byte chunk as in xudp's "
                         "UMEM (eth at chunk + 342 / + 322, SURVEY a14)")
    ap.add_argument("--only", default="", help="comma list of modes to run: plain, verify, "
                    "verify_iphdr, csum_verify, csum (default: all)")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    eng = X.Engine(0)
    s = torch.cuda.current_stream(dev)
    for cid in [int(c) for c in args.configs.split(",")]:
        cfg = bench.CONFIGS[cid]
        n, fam = cfg["n"], cfg["family"]
        seed = bench.SEED_BASE ^ cid
        kw = dict(stride=4096, offset=322 if fam == 6 else 342) if args.layout == "umem" else {}
        if args.layout == "umem" and cfg["pmax"] > 3700:
            continue   # jumbo frames do not fit a 4096-byte chunk
        desc, nbytes = X.gen_layout(n, fam, cfg["pmin"], cfg["pmax"], seed=seed, **kw)
        d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
        nrot = max(1, math.ceil((1 << 30) / nbytes))
        bufs = [torch.empty(nbytes + 64, dtype=torch.uint8, device=dev) for _ in range(nrot)]
        eng.gen_fill_device(bufs[0], d_desc, n, fam, seed, 0)
        mode = X.MODE_V6 if fam == 6 else X.MODE_V4_RFC
        eng.batch_device(bufs[0], d_desc, n, None, mode, X.F_INPLACE | X.F_IPHDR)
        for b in bufs[1:]:
            b.copy_(bufs[0])
        d_msgs = torch.empty(n * 64, dtype=torch.uint8, device=dev)
        d_count = torch.zeros(1, dtype=torch.int32, device=dev)
        d_out = torch.empty(n, dtype=torch.int16, device=dev)
        frame_bytes = int(desc["len"].astype(np.int64).sum())
        hint = int(desc["len"].mean())
        # clock ramp: >= 300 ms of launches before anything is timed (the
        # clocks take tens of milliseconds to reach their working point)
        import time
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 0.3:
            for _ in range(20):
                eng.batch_device(bufs[k % nrot], d_desc, n, d_out, mode, X.F_VERIFY, hint,
                                 stream=s.cuda_stream)
                k += 1
            torch.cuda.synchronize()

        def rx_fn(flags, gname):
            def rx(k):
                if gname == "auto":
                    eng.set_tuning(X.TUNE_RX_GEOMETRY, 0)
                else:
                    eng.set_tuning(X.TUNE_RX_GEOMETRY, *[int(v) for v in gname.split(",")])
                eng.rx_device(bufs[k % nrot], d_desc, n, d_msgs,
                              None if args.no_count else d_count, flags, hint,
                              stream=s.cuda_stream)
            return rx

        def csum_fn(flags):
            def ver(k):
                eng.batch_device(bufs[k % nrot], d_desc, n, d_out, mode, flags, hint,
                                 stream=s.cuda_stream)
            return ver

        runs = []   # (record, fn, check)
        names = (("plain", 0), ("verify", X.F_VERIFY), ("verify_iphdr", X.F_VERIFY | X.F_IPHDR))
        for gname in args.geoms.split(";"):
            for fname, flags in (names[::-1] if args.reverse else names):
                read = frame_bytes if flags else 64 * n
                runs.append(({"kernel": "rx", "config": cid, "flags": fname, "geometry": gname,
                              "layout": args.layout,
                              "moved": read + n * (16 + 64)}, rx_fn(flags, gname), flags))
        runs.append(({"kernel": "csum_verify", "config": cid, "flags": "verify",
                      "moved": frame_bytes + n * 18}, csum_fn(X.F_VERIFY), None))
        runs.append(({"kernel": "csum", "config": cid, "flags": "none",
                      "moved": frame_bytes + n * 18}, csum_fn(0), None))
        if args.only:
            keep = set(args.only.split(","))
            runs = [r for r in runs if (r[0]["flags"] if r[0]["kernel"] == "rx" else
                                        ("csum_verify" if r[0]["kernel"] == "csum_verify"
                                         else "csum")) in keep]
        # interleaved rounds in one process: every mode sees the same clocks;
        # per round K back-to-back launches between two events
        K = max(5, min(50, int(0.02 / max(frame_bytes / 5e12, 1e-6))))
        times = [[] for _ in runs]
        for r in range(args.reps):
            for i, (rec, fn, _) in enumerate(runs):
                fn(0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for k in range(K):
                    fn(k)
                e1.record(s)
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) / K * 1e-3)
        eng.set_tuning(X.TUNE_RX_GEOMETRY, 0)
        # clocks while kernels run: the boxes differ on this kernel far more
        # than on the checksum kernel, and SCLK is the first suspect
        for k in range(3 * K):
            runs[0][1](k)
        clocks = bench.gpu_clocks(dev)
        torch.cuda.synchronize()
        cv = [i for i, r in enumerate(runs) if r[0]["kernel"] == "csum_verify"]
        t_csum = float(np.median(times[cv[0]])) if cv else float("nan")
        for (rec, fn, flags), ts in zip(runs, times):
            t = float(np.median(ts))
            if rec["kernel"] == "rx":
                if args.no_count:
                    ok = bool((d_msgs.view(-1, 64)[:, 20].cpu() == 0).all().item())
                else:
                    fn(0)
                    torch.cuda.synchronize()
                    ok = int(d_count.item()) == n
                rec["all_delivered"] = ok
            else:
                fn(0)
                torch.cuda.synchronize()
                if rec["flags"] == "verify":
                    rec["all_valid"] = bool((d_out == 0).all().item())
            moved = rec.pop("moved")
            rec.update({"frames": n, "ms": round(t * 1e3, 4), "mpps": round(n / t / 1e6, 1),
                        "GBps_moved": round(moved / t / 1e9, 1),
                        "pct_hbm_peak": round(100 * moved / t / 8e12, 1),
                        "vs_csum_verify": round(t / t_csum, 3), "launches_per_round": K,
                        "rounds": args.reps, "clocks_under_load": clocks})
            print(json.dumps(rec), flush=True)
        del bufs, d_msgs
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
