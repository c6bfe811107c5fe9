#!/usr/bin/env python3
"""End-to-end rate of the host-resident path (frames start and end in host
memory, like xudp's AF_XDP UMEM): xcsum_batch_host() = chunked double-buffered
hipMemcpyAsync H2D -> kernel -> 2-byte results D2H, for
  pageable   -- plain malloc'ed UMEM (runtime stages the copies),
  registered -- UMEM page-locked with xcsum_register_umem (direct DMA),
  zerocopy   -- registered UMEM read in place by the kernel over PCIe,
and each of them with XCSUM_F_INPLACE (udp->check written into the host
frames); then the receive side, xcsum_rx_host with VERIFY on the same frames
(checksums written in first), in the same three variants.  Also the raw
pinned H2D copy rate for context.  One JSON line per variant.
--layout umem puts one frame per 4096-byte chunk (xudp's UMEM, SURVEY a14;
256K frames, 1 GiB), the layout an AF_XDP RX ring hands over.
--iphdr-only times libxudp's IPv4 TX call instead (XCSUM_F_IPHDR_ONLY:
iph->check alone; 42 bytes per frame gathered, or read in place over PCIe)
against the reference's own xudp_checksum_half on the host (oracle/_ref
through bench.cpu_baseline: 1 and 16 threads on a 65,536-frame sample of
the config), and skips the receive side.
Usage: python tools/bench_e2e.py [--config 2] [--reps 5] [--layout umem] [--iphdr-only]"""
import argparse
import json
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--layout", default="packed", choices=["packed", "umem"])
    ap.add_argument("--iphdr-only", action="store_true")
    args = ap.parse_args()
    import torch
    cfg = dict(bench.CONFIGS[args.config], id=args.config)
    n = min(cfg["n"], 1 << 20)
    lay = {}
    if args.layout == "umem":
        n = min(n, 1 << 18)
        lay = dict(stride=4096, offset=322 if cfg["family"] == 6 else 342)
    umem, desc = X.gen_frames_host(n, cfg["family"], cfg["pmin"], cfg["pmax"],
                                   seed=bench.SEED_BASE ^ args.config, **lay)
    # in a mapping like libxudp's UMEM (anon_map: MAP_SHARED, no transparent
    # huge pages), which xcsum_register_umem GPU-maps; a numpy
    # array of this size is THP-eligible and would be staged instead
    umem = X.as_umem(umem)
    alg = X.alg_bytes(desc, cfg["family"])
    out = np.zeros(n, dtype=np.uint16)
    eng = X.Engine(0)
    import oracle
    mode, extra = cfg["mode"], 0
    if args.iphdr_only:
        assert cfg["family"] == 4, "--iphdr-only: an IPv4 config"
        mode, extra = X.MODE_V4_LEGACY, X.F_IPHDR_ONLY
        alg = 22 * n
        for a in desc["addr"]:           # as iph_build leaves it
            umem[int(a) + 24:int(a) + 26] = 0
    exp = oracle.batch(umem, desc, mode, extra)
    if args.iphdr_only:
        # the reference on the host (bench.cpu_baseline's legs, its own
        # 65,536-frame sample of the config)
        cb = bench.cpu_baseline(cfg, seconds=10.0, flags=X.F_IPHDR_ONLY)
        print(json.dumps({"variant": "reference_cpu", "frames": n, **cb}), flush=True)

    # raw pinned H2D rate of the same bytes
    pin = torch.empty(umem.nbytes, dtype=torch.uint8).pin_memory()
    pin.numpy()[:] = umem
    dst = torch.empty(umem.nbytes, dtype=torch.uint8, device="cuda:0")
    dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    h2d = umem.nbytes * args.reps / (time.perf_counter() - t0) / 1e9
    print(json.dumps({"variant": "raw_pinned_h2d_copy", "GBps": round(h2d, 1),
                      "bytes": umem.nbytes}), flush=True)
    del pin, dst

    for variant in ("pageable", "registered", "zerocopy"):
        for inplace in (False, True):
            flags = (X.F_INPLACE if inplace else 0) | extra
            if variant != "pageable":
                eng.register_umem(umem)
                assert eng.umem_mapped(umem), "registered UMEM not GPU-mapped"
            if variant == "zerocopy":
                flags |= X.F_ZEROCOPY
            eng.batch_host(umem, desc, out, mode, flags)  # warm-up
            ok = bool(np.array_equal(out, exp))
            t0 = time.perf_counter()
            for _ in range(args.reps):
                eng.batch_host(umem, desc, out, mode, flags)
            dt = (time.perf_counter() - t0) / args.reps
            if variant != "pageable":
                eng.unregister_umem(umem)
            if inplace:  # restore check fields for the next variant
                umem2, _ = X.gen_frames_host(n, cfg["family"], cfg["pmin"], cfg["pmax"],
                                             seed=bench.SEED_BASE ^ args.config, **lay)
                umem[:] = umem2
                if args.iphdr_only:
                    for a in desc["addr"]:
                        umem[int(a) + 24:int(a) + 26] = 0
            print(json.dumps({"variant": variant, "inplace": inplace, "frames": n,
                              "layout": args.layout,
                              "ms": round(dt * 1e3, 3),
                              "GiBps_alg": round(alg / dt / 2**30, 1),
                              "GBps_frames": round(umem.nbytes / dt / 1e9, 1),
                              "mpps": round(n / dt / 1e6, 1), "parity": ok}), flush=True)
    if args.iphdr_only:
        eng.close()
        return

    # receive side: the same frames with valid checksums written in
    # (RFC rules, IPv4 header too), verified by xcsum_rx_host
    rfc = X.MODE_V6 if cfg["family"] == 6 else X.MODE_V4_RFC
    eng.batch_host(umem, desc, out, rfc, X.F_INPLACE | X.F_IPHDR)
    msgs = np.zeros(n, dtype=X.RX_MSG_DTYPE)
    flags_rx = X.F_VERIFY | X.F_IPHDR
    exp_rx = oracle.rx_batch(umem, desc, flags_rx)
    for variant in ("pageable", "registered", "zerocopy"):
        flags = flags_rx | (X.F_ZEROCOPY if variant == "zerocopy" else 0)
        if variant != "pageable":
            eng.register_umem(umem)
        cnt = eng.rx_host(umem, desc, msgs, flags)  # warm-up
        ok = bool(np.array_equal(msgs.view(np.uint8), exp_rx.view(np.uint8))) and cnt == n
        t0 = time.perf_counter()
        for _ in range(args.reps):
            eng.rx_host(umem, desc, msgs, flags)
        dt = (time.perf_counter() - t0) / args.reps
        if variant != "pageable":
            eng.unregister_umem(umem)
        print(json.dumps({"variant": "rx_" + variant, "verify": True, "frames": n,
                          "layout": args.layout, "frame_bytes": int(desc["len"].sum()),
                          "ms": round(dt * 1e3, 3),
                          "GBps_frames": round(umem.nbytes / dt / 1e9, 1),
                          "mpps": round(n / dt / 1e6, 1), "parity": ok}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
