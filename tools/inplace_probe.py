#!/usr/bin/env python3
"""In-place write schedules on one box (measuring stick).

Config-2 (IPv4, fields at eth+24 and eth+40) and config-4 (IPv6, eth+60)
frames, packed (1520-B stride) or in xudp's 4096-B slots, 1M frames in a
>= 1 GiB rotation: per launch, medians of 5 x 10 back-to-back launches:
  read            the plain stream read (tools/hbm_probe.hip)
  w2              2-byte field stores alone (second pass of two-pass)
  w32 / w64       the same as whole 32-B sector / 64-B line read-patch-write
  read+w2/32/64   the read, then that second pass (two launches)
  lib_plain       the library's checksum pass with a result array
  lib_fused       the library's in-place pass, FUSED schedule
  lib_two_pass    the library's in-place pass, TWO_PASS schedule
  fused_nt        the read with each field stored by the thread that read it
  fused_tl        the same, the chunks holding a field loaded temporally
  [read+]blindW   whole W-byte blocks holding the fields written with junk,
                  no load first (after the read pass, or alone)
  [read+]copy64   the 64-B blocks holding the fields copied whole from a
                  compact side array (a first pass's saved blocks)
  lib_plain+X     the library's plain pass, then second pass X (copy64,
                  blind64, w2)
  lib_two_pass_wW[_out]  the library's TWO_PASS schedule with second-pass
                  store width W (XCSUM_TUNE_INPLACE_BLOCK; 0: 2-byte stores);
                  _out: with a result array (no scratch)
  fused_blkW      the read, each W-byte block holding a field stored back
                  whole by the wave that read it (W = 16/32/64/128)
  lib_fused_tl2/4 the library's fused pass with each frame's first 2 / 4
                  chunks loaded temporally (XCSUM_TUNE_INPLACE_TL)
Prints one JSON line per layout and family."""
import argparse
import ctypes
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import libxudp_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", type=int, default=4)
    ap.add_argument("--layout", default="packed", choices=["packed", "umem"])
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--legs", default="", help="comma list of legs to run (default: all)")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    fam = args.family
    off = (322 if fam == 6 else 342) if args.layout == "umem" else 0
    kw = dict(stride=4096, offset=off) if args.layout == "umem" else {}
    desc, nbytes = X.gen_layout(args.n, fam, 1472, 1472, seed=7, **kw)
    a = desc["addr"].astype(np.int64)
    fstride, a0 = int(a[1] - a[0]), int(a[0])
    nrot = max(1, math.ceil((1 << 30) / nbytes))
    bufs = [torch.empty(nbytes + 128, dtype=torch.uint8, device=dev) for _ in range(nrot)]
    d_desc = torch.from_numpy(desc.view(np.uint8)).pin_memory().to(dev)
    eng = X.Engine(0)
    s = torch.cuda.current_stream(dev)
    sp = s.cuda_stream
    for b in bufs:
        eng.gen_fill_device(b, d_desc, len(desc), fam, 7, 0, stream=sp)
    out = torch.empty(len(desc), dtype=torch.int16, device=dev)
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbmprobe.so"))
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    blocks = cus * 8
    scratch = torch.empty(blocks * 256, dtype=torch.int32, device=dev)
    f1 = 60 if fam == 6 else 40
    f2 = 60 if fam == 6 else 24
    V, U64, U32, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.probe_stream_read.argtypes = [V, U64, V, I, I, I, V]
    L.probe_scatter_fields.argtypes = [V, U64, U64, U64, U64, U32, U32, I, V]
    L.probe_stream_read_twopass.argtypes = [V, U64, U64, U64, U64, U32, U32, V, I, V]
    L.probe_stream_read_twopass_blocks.argtypes = [V, U64, U64, U64, U64, U32, U32, V, I, I, I,
                                                   V]
    nb = nbytes & ~15
    mode = X.MODE_V6 if fam == 6 else X.MODE_V4_LEGACY
    iph = 0 if fam == 6 else X.F_IPHDR
    legs = {
        "read": lambda b: L.probe_stream_read(b, nb, scratch.data_ptr(), blocks, 1, 4, sp),
        "w2": lambda b: L.probe_scatter_fields(b, nb, fstride, a0, len(a), f1, f2, blocks, sp),
        "w32": lambda b: L.probe_stream_read_twopass_blocks(b, nb, fstride, a0, len(a), f1, f2,
                                                             scratch.data_ptr(), blocks, 32, 0,
                                                             sp),
        "w64": lambda b: L.probe_stream_read_twopass_blocks(b, nb, fstride, a0, len(a), f1, f2,
                                                             scratch.data_ptr(), blocks, 64, 0,
                                                             sp),
        "read+w2": lambda b: L.probe_stream_read_twopass(b, nb, fstride, a0, len(a), f1, f2,
                                                         scratch.data_ptr(), blocks, sp),
        "read+w32": lambda b: L.probe_stream_read_twopass_blocks(b, nb, fstride, a0, len(a), f1,
                                                                  f2, scratch.data_ptr(), blocks,
                                                                  32, 1, sp),
        "read+w64": lambda b: L.probe_stream_read_twopass_blocks(b, nb, fstride, a0, len(a), f1,
                                                                  f2, scratch.data_ptr(), blocks,
                                                                  64, 1, sp),
    }

    L.probe_stream_read_inplace.argtypes = [V, U64, U64, U64, U64, U32, U32, V, I, I, V]
    L.probe_stream_read_inplace_tl.argtypes = [V, U64, U64, U64, U64, U32, U32, V, I, V]
    legs["fused_nt"] = lambda b: L.probe_stream_read_inplace(b, nb, fstride, a0, len(a), f1, f2,
                                                            scratch.data_ptr(), blocks, 1, sp)
    legs["fused_tl"] = lambda b: L.probe_stream_read_inplace_tl(b, nb, fstride, a0, len(a), f1,
                                                               f2, scratch.data_ptr(), blocks, sp)

    L.probe_stream_read_inplace_blk.argtypes = [V, U64, U64, U64, U64, U32, U32, V, I, I, V]
    for W in (16, 32, 64, 128):
        legs[f"fused_blk{W}"] = (lambda W_: lambda b: L.probe_stream_read_inplace_blk(
            b, nb, fstride, a0, len(a), f1, f2, scratch.data_ptr(), blocks, W_, sp))(W)

    L.probe_stream_read_blind.argtypes = [V, U64, U64, U64, U64, U32, U32, V, I, I, I, V]
    for W in (16, 32, 64, 128):
        for rf in (0, 1):
            legs[f"{'read+' if rf else ''}blind{W}"] = (lambda W_, rf_: lambda b:
                L.probe_stream_read_blind(b, nb, fstride, a0, len(a), f1, f2, scratch.data_ptr(),
                                          blocks, W_, rf_, sp))(W, rf)

    side = torch.zeros(len(desc) * 128, dtype=torch.uint8, device=dev)
    L.probe_stream_read_copy.argtypes = [V, U64, U64, U64, U64, U32, U32, V, U64, V, I, I, V]
    for rf in (0, 1):
        legs[f"{'read+' if rf else ''}copy64"] = (lambda rf_: lambda b: L.probe_stream_read_copy(
            b, nb, fstride, a0, len(a), f1, f2, side.data_ptr(), side.numel(),
            scratch.data_ptr(), blocks, rf_, sp))(rf)

    def lib(sched, flags, o):
        def f(b):
            eng.set_inplace(sched)
            eng.batch_device(b, d_desc, len(desc), o, mode, flags, 1500, stream=sp)
            return 0
        return f
    engs_tl = {}
    for tl in (2, 4):
        engs_tl[tl] = X.Engine(0)
        engs_tl[tl].set_tuning(X.TUNE_INPLACE_TL, tl)

    def lib_tl(tl):
        def f(b):
            engs_tl[tl].batch_device(b, d_desc, len(desc), None, mode, X.F_INPLACE | iph, 1500,
                                     stream=sp)
            return 0
        return f
    engs_blk = {}
    for w in (0, 32, 64):
        engs_blk[w] = X.Engine(0)
        engs_blk[w].set_tuning(X.TUNE_INPLACE_BLOCK, w)
        engs_blk[w].set_inplace(X.INPLACE_TWO_PASS)

    def lib_blk(w, o):
        def f(b):
            engs_blk[w].batch_device(b, d_desc, len(desc), o, mode, X.F_INPLACE | iph, 1500,
                                     stream=sp)
            return 0
        return f
    for w in (0, 32, 64):
        legs[f"lib_two_pass_w{w}"] = lib_blk(w, None)
        legs[f"lib_two_pass_w{w}_out"] = lib_blk(w, out)
    legs["lib_fused_tl2"] = lib_tl(2)
    legs["lib_fused_tl4"] = lib_tl(4)
    legs["lib_plain"] = lib(X.INPLACE_AUTO, iph, out)

    def lib_plain_then(second):
        def f(b):
            eng.set_inplace(X.INPLACE_AUTO)
            eng.batch_device(b, d_desc, len(desc), out, mode, iph, 1500, stream=sp)
            return second(b)
        return f
    legs["lib_plain+copy64"] = lib_plain_then(lambda b: L.probe_stream_read_copy(
        b, nb, fstride, a0, len(a), f1, f2, side.data_ptr(), side.numel(), scratch.data_ptr(),
        blocks, 0, sp))
    legs["lib_plain+blind64"] = lib_plain_then(lambda b: L.probe_stream_read_blind(
        b, nb, fstride, a0, len(a), f1, f2, scratch.data_ptr(), blocks, 64, 0, sp))
    legs["lib_plain+w2"] = lib_plain_then(lambda b: L.probe_scatter_fields(
        b, nb, fstride, a0, len(a), f1, f2, blocks, sp))
    legs["lib_fused"] = lib(X.INPLACE_FUSED, X.F_INPLACE | iph, None)
    legs["lib_two_pass"] = lib(X.INPLACE_TWO_PASS, X.F_INPLACE | iph, None)
    if args.legs:
        legs = {k: legs[k] for k in args.legs.split(",")}
    res = {}
    for rnd in range(args.rounds):   # rounds of interleaved legs; the min of the medians
        for name, fn in legs.items():
            ts = []
            for r in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for k in range(10):
                    if fn(bufs[k % len(bufs)].data_ptr()) != 0:
                        raise SystemExit(f"{name} failed")
                e1.record(s)
                torch.cuda.synchronize(dev)
                ts.append(e0.elapsed_time(e1) / 10)
            m = float(np.median(ts[1:]))
            res[name] = round(min(res.get(name, 1e9), m), 4)
    print(json.dumps({"family": fam, "layout": args.layout, "n": len(desc), "fstride": fstride,
                      "eth0": a0, "fields": [f2, f1], "rotating_buffers": nrot,
                      "ms_per_launch": res}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
