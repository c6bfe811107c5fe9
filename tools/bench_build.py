#!/usr/bin/env python3
"""Throughput of xcsum_build_device (xudp_frame_send on the GPU): 1M messages
of one payload size into xudp's TX frame layout (4096-byte slots, data at
+384).  Modes: copy from a packed payload buffer (aligned /
unaligned sources) and in place (payload already in its slot, the
xudp_frame_alloc path).  Bytes moved per frame: copy = payload read + frame
(headers + payload) written + 16-byte message + 16-byte descriptor; in place
= payload read + headers written + message + descriptor.
Mode d2d_copy: the payload bytes copied device to device (torch's copy,
contiguous) into the same UMEMs, the copy modes' bound.
One JSON line per mode.  Usage: python tools/bench_build.py [--payload 1472]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libxudp_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--payload", type=int, default=1472)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--family", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--modes", default="copy_aligned,copy_unaligned,inplace")
    ap.add_argument("--rot", type=int, default=4, help="UMEM buffers rotated between launches")
    ap.add_argument("--orders", default="auto",
                    help="comma list of visiting orders to time, 'auto' or R_T "
                         "(xcsum_ctx_set_order: 2^R regions of 2^T-message tiles)")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    n, L, fam = args.n, args.payload, args.family
    hdr = 42 if fam == 4 else 62
    FRAME, DATA_OFF = 4096, 384
    eng = X.Engine(0)
    route = X.make_route(fam, b"\x02\0\0\0\0\x01", b"\x02\0\0\0\0\x02",
                         bytes(range(16)) if fam == 6 else bytes([10, 0, 35, 2]), 3486,
                         bytes(range(16, 32)) if fam == 6 else bytes([10, 0, 35, 1]), 40000)
    # rotated UMEMs: the header lines one launch writes (~128 MB for 1M
    # slots) would otherwise stay in the 256 MiB Infinity Cache between launches
    d_umems = [torch.zeros(n * FRAME, dtype=torch.uint8, device=dev) for _ in range(args.rot)]
    d_desc = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_out = torch.zeros(n, dtype=torch.int16, device=dev)
    res = {}
    for mode in args.modes.split(","):
        stride = L + (1 if mode == "copy_unaligned" else 0)
        stride = stride if mode == "copy_unaligned" else (L + 15) // 16 * 16
        msgs = np.zeros(n, dtype=X.MSG_DTYPE)
        msgs["src"] = np.arange(n, dtype=np.uint64) * stride
        msgs["len"] = L
        msgs["slot"] = np.arange(n, dtype=np.uint32)
        d_msgs = torch.from_numpy(msgs.view(np.uint8)).to(dev)
        d_src = torch.randint(0, 255, (n * stride + 16,), dtype=torch.uint8, device=dev)
        if mode == "d2d_copy":
            # the copy bound of the copy modes: the payload bytes copied
            # device to device, contiguous (torch's copy kernel), into the
            # rotated UMEMs; moved = read + write
            s = torch.cuda.current_stream(dev)
            src = d_src[:n * L]
            for k in range(20):
                d_umems[k % args.rot][:n * L].copy_(src)
            torch.cuda.synchronize()
            evs = []
            for k in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                d_umems[k % args.rot][:n * L].copy_(src)
                e1.record(s)
                evs.append((e0, e1))
            torch.cuda.synchronize()
            t = float(np.median([a.elapsed_time(b) for a, b in evs])) * 1e-3
            print(json.dumps({"mode": mode, "rotating_umems": args.rot, "payload": L,
                              "frames": n, "ms": round(t * 1e3, 4),
                              "GBps_moved": round(2 * n * L / t / 1e9, 1),
                              "pct_hbm_peak": round(100 * 2 * n * L / t / 8e12, 1)}), flush=True)
            del d_src
            continue
        flags = {"inplace": X.F_BUILD_INPLACE, "inplace_sum": X.F_BUILD_INPLACE,
                 "copy_aligned": X.F_SRC_ALIGNED}.get(mode, 0)
        # inplace_sum (A/B): IPv4 in place through the payload-summing build
        # kernel (xcsum_ctx_set_tuning XCSUM_TUNE_BUILD_HDR 0), as before round 5
        eng.set_tuning(X.TUNE_BUILD_HDR, 0 if mode == "inplace_sum" else 1)
        for order in args.orders.split(","):
            if order == "auto":
                eng.set_order(-1, 0)
            else:
                eng.set_order(*[int(v) for v in order.split("_")])
            s = torch.cuda.current_stream(dev)
            # clock ramp: >= 300 ms of launches before anything is timed
            import time
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                for k in range(10):
                    eng.build_device(route, d_src, d_msgs, n, d_umems[k % args.rot], FRAME, DATA_OFF,
                                     d_desc, d_out, flags, L, s.cuda_stream)
                torch.cuda.synchronize()
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.reps)]
            for k, (e0, e1) in enumerate(evs):
                e0.record(s)
                eng.build_device(route, d_src, d_msgs, n, d_umems[k % args.rot], FRAME, DATA_OFF,
                                 d_desc, d_out, flags, L, s.cuda_stream)
                e1.record(s)
            torch.cuda.synchronize()
            t = float(np.median([a.elapsed_time(b) for a, b in evs])) * 1e-3
            if mode == "inplace" and fam == 4:
                # libxudp's IPv4 send in place: headers only, no payload byte read
                # (packet.c:43-66, :125; build_hdr_kernel)
                moved = n * (hdr + 32)
            elif mode.startswith("inplace"):
                moved = n * (L + hdr + 32)
            else:
                moved = n * (L + hdr + L + 32)
            rec = {"mode": mode, "order": order, "rotating_umems": args.rot,
                   "geometry": "auto",
                   "payload": L, "family": fam, "frames": n, "ms": round(t * 1e3, 4),
                   "mpps": round(n / t / 1e6, 1), "GBps_moved": round(moved / t / 1e9, 1),
                   "pct_hbm_peak": round(100 * moved / t / 8e12, 1)}
            if mode == "inplace":
                # the checksum call on the frames just built (headers in place):
                # checksums + in-place writes only, the same slots, same process;
                # IPv4: libxudp's call, iph->check alone (XCSUM_F_IPHDR_ONLY)
                d_bdesc = d_desc.clone()
                cs = []
                for k in range(args.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    eng.batch_device(d_umems[k % args.rot], d_bdesc, n, d_out,
                                     X.MODE_V6 if fam == 6 else X.MODE_V4_LEGACY,
                                     X.F_INPLACE | (X.F_IPHDR_ONLY if fam == 4 else 0), L + hdr,
                                     stream=s.cuda_stream)
                    e1.record(s)
                    cs.append((e0, e1))
                torch.cuda.synchronize()
                tc = float(np.median([a.elapsed_time(b) for a, b in cs])) * 1e-3
                rec["csum_inplace_ms"] = round(tc * 1e3, 4)
                rec["vs_csum_inplace"] = round(t / tc, 3)
            print(json.dumps(rec), flush=True)
        del d_src, d_msgs
    eng.set_order(-1, 0)
    eng.close()


if __name__ == "__main__":
    main()
