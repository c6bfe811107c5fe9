#!/usr/bin/env python3
"""Strong scaling of config 5 from one GPU:
the 8M-frame job split by bytes into N shards (xcsum_shard_by_bytes, as
bench.py's ranks split it), every shard of N = 1, 2, 4, 8 timed alone on
this GPU over the same device-resident frames, and its output checked
against the reference's digest of exactly that shard.  With no collective on
the data path, an N-GPU job takes as long as its slowest shard, so
T(1) / max_r T_r(N) is the whole job's speedup if the N GPUs run like this
one (the driver's 8-GPU node measures the real thing, SCALE_r*.json).

Per shard: `per` back-to-back launches between two events, median of
`reps`; shards and N interleaved over `rounds` rounds, the lower median
kept.  One JSON line per N, then a summary line.

    python tools/shard_scan.py [--ns 1,2,4,8] [--rounds 2]
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import libxudp_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--per", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--warm-ms", type=float, default=300.0)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    eng = X.Engine(0)
    s = torch.cuda.current_stream(dev)
    sp = s.cuda_stream
    cfg = dict(bench.CONFIGS[5], id=5, layout="packed")
    desc, d_desc, bufs, out, first, count = bench.build_batch(cfg, 0, 1, torch, dev, eng, sp)
    umem = bufs[0]
    digests = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))["config5"]
    ns = [int(v) for v in args.ns.split(",")]
    shards = {}
    for n in ns:
        for r in range(n):
            f, c = X.shard_by_bytes(desc, n, r)
            sub = desc[f:f + c]
            shards[(n, r)] = dict(first=f, count=c, alg=X.alg_bytes(sub, 4),
                                  hint=int(sub["len"].mean()),
                                  d_desc=d_desc[16 * f:16 * (f + c)], out=out[f:f + c])

    def launch(sh):
        eng.batch_device(umem, sh["d_desc"], sh["count"], sh["out"], cfg["mode"], 0, sh["hint"],
                         stream=sp)

    # clocks up: whole-job launches for warm-ms
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    spent = 0.0
    while spent < args.warm_ms:
        e0.record(s)
        launch(shards[(ns[0], 0)])
        e1.record(s)
        torch.cuda.synchronize(dev)
        spent += e0.elapsed_time(e1)
    best = {}
    for rnd in range(args.rounds):
        for key, sh in shards.items():
            ts = []
            for rep in range(args.reps + 1):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for k in range(args.per):
                    launch(sh)
                b.record(s)
                torch.cuda.synchronize(dev)
                ts.append(a.elapsed_time(b) / args.per)
            best[key] = min(best.get(key, 1e9), float(np.median(ts[1:])))
    # parity: one pass per shard into a zeroed output, against its digest
    rows = []
    t1 = None
    for n in ns:
        ok = []
        for r in range(n):
            sh = shards[(n, r)]
            sh["out"].zero_()
            launch(sh)
            torch.cuda.synchronize(dev)
            h = torch.empty(sh["count"], dtype=torch.int16, pin_memory=True)
            h.copy_(sh["out"])
            got = hashlib.sha256(h.numpy().tobytes()).hexdigest()
            want = digests["sha256_out"] if n == 1 else digests[f"sha256_out_shards{n}"][r]
            ok.append(got == want)
        ms = [round(best[(n, r)], 4) for r in range(n)]
        slow = max(ms)
        if n == 1:
            t1 = slow
        alg_all = sum(shards[(n, r)]["alg"] for r in range(n))
        row = {"n": n, "shard_ms": ms, "slowest_ms": slow,
               "shard_GBps": [round(shards[(n, r)]["alg"] / (best[(n, r)] * 1e-3) / 1e9, 1)
                              for r in range(n)],
               "frames": [shards[(n, r)]["count"] for r in range(n)],
               "projected_job_GiBps": round(alg_all / (slow * 1e-3) / 2**30, 1),
               "projected_speedup": round(t1 / slow, 3) if t1 else None,
               "projected_efficiency": round(t1 / slow / n, 4) if t1 else None,
               "parity_digests_ok": all(ok)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"summary": "config 5 strong scaling projected from shards timed alone "
                                 "on one GPU (no collective on the data path)",
                      "speedup_by_n": {str(r["n"]): r["projected_speedup"] for r in rows},
                      "parity_ok": all(r["parity_digests_ok"] for r in rows)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
