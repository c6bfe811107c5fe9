#!/usr/bin/env python3
"""Headline benchmark: device-resident UDP checksum GiB/s (BASELINE.json metric).

A step = one xcsum_batch_device() launch over one batch of synthetic frames
already resident in HBM: by default BASELINE config 2, 1,048,576 x 1472-byte
UDP/IPv4 frames (1.6 GB), checksummed bit-exactly like xudp/checksum.h's
udp_checksum().  N>1: one process per GPU (torch.distributed.run), each rank
checksums its own batch (weak scaling, no collective on the data path; the
only collectives are the timing barrier and the max-over-ranks of the elapsed
time).

value    = algorithmic bytes of all ranks / max-over-ranks wall time, GiB/s
           (algorithmic bytes per frame = UDP length + pseudo-header address
           bytes + 2-byte result)
roofline = the checksum kernel's algorithmic bytes per launch / its average
           launch duration (HIP events on the launch stream), vs 8 TB/s HBM3E
cpu_baseline = the reference's own checksum.h (oracle/_ref, compiled from
           /root/reference in the build container) on a bounded sample of the
           same workload on this host's cores (rank 0, N=1 only)

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C]
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import libxudp_amd as X  # noqa: E402

SEED_BASE = 0x78756470  # "xudp"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    2: dict(n=1 << 20, family=4, pmin=1472, pmax=1472, mode=X.MODE_V4_LEGACY, shard=False,
            name="1M x 1472B UDP/IPv4, device-resident (BASELINE config 2)"),
    3: dict(n=1 << 20, family=4, pmin=64, pmax=64, mode=X.MODE_V4_LEGACY, shard=False,
            name="1M x 64B UDP/IPv4, device-resident (BASELINE config 3)"),
    4: dict(n=1 << 20, family=6, pmin=1472, pmax=1472, mode=X.MODE_V6, shard=False,
            name="1M x 1472B UDP/IPv6, device-resident (BASELINE config 4)"),
    5: dict(n=8 << 20, family=4, pmin=64, pmax=9000, mode=X.MODE_V4_LEGACY, shard=True,
            name="8M x U[64,9000]B UDP/IPv4 sharded by bytes over the GPUs (BASELINE config 5)"),
}
MODE_NAMES = {0: "v4_legacy", 1: "v4_rfc", 2: "v6", 3: "auto"}


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def rank_slice(cfg, rank, world):
    """(first global frame index, frame count) owned by `rank`.  Config 5 is
    one 8M-frame job split by bytes over the ranks (strong scaling); the others
    give every rank its own full batch (weak scaling).  No data-path
    collective: a frame's checksum depends on that frame only."""
    n = cfg["n"]
    if cfg["shard"]:
        full, _ = X.gen_layout(n, cfg["family"], cfg["pmin"], cfg["pmax"],
                               seed=SEED_BASE ^ cfg["id"])
        return X.shard_by_bytes(full, world, rank)
    return rank * n, n


def build_batch(cfg, rank, world, torch, dev, eng, stream):
    """Descriptors + frames for this rank, generated on the device."""
    seed = SEED_BASE ^ cfg["id"]
    first, count = rank_slice(cfg, rank, world)
    if cfg.get("layout") == "umem":
        # xudp's own TX layout: one frame per 4096-byte chunk, eth at F+342
        # (IPv4) / F+322 (IPv6), SURVEY a14
        off = 322 if cfg["family"] == 6 else 342
        desc, nbytes = X.gen_layout(count, cfg["family"], cfg["pmin"], cfg["pmax"], seed=seed,
                                    first_index=first, stride=4096, offset=off)
    else:
        desc, nbytes = X.gen_layout(count, cfg["family"], cfg["pmin"], cfg["pmax"], seed=seed,
                                    first_index=first)
    d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
    # rotate buffers so each pass streams >= 1 GiB: nothing is served from the
    # 256 MiB Infinity Cache (SURVEY.md 7 hard part iv)
    nrot = max(1, math.ceil((1 << 30) / max(nbytes, 1)))
    bufs = [torch.empty(nbytes + 64, dtype=torch.uint8, device=dev) for _ in range(nrot)]
    eng.gen_fill_device(bufs[0], d_desc, count, cfg["family"], seed, first, stream=stream)
    for b in bufs[1:]:
        b.copy_(bufs[0])
    out = torch.empty(max(count, 1), dtype=torch.int16, device=dev)
    torch.cuda.synchronize(dev)
    return desc, d_desc, bufs, out, first, count


def cpu_baseline(cfg, seconds=10.0):
    """The reference checksum.h timed on this host over a bounded sample."""
    import oracle  # test infrastructure, used here only as the CPU baseline
    seed = SEED_BASE ^ cfg["id"]
    m = min(cfg["n"], 1 << 16)
    umem, desc = X.gen_frames_host(m, cfg["family"], cfg["pmin"], cfg["pmax"], seed=seed)
    out = np.zeros(m, dtype=np.uint16)
    alg = X.alg_bytes(desc, cfg["family"])
    mode = 2 if cfg["family"] == 6 else 0
    if oracle.have_ref():
        kind, L = "reference", oracle.ref()
        timed = lambda th, reps: L.ref_batch_timed(umem.ctypes.data, desc.ctypes.data, m,
                                                   out.ctypes.data, mode, th, reps)
    else:
        kind, L = "port", oracle.port()
        timed = lambda th, reps: L.orc_batch_timed(umem.ctypes.data, desc.ctypes.data, m,
                                                   out.ctypes.data, mode, 0, th, reps)
    threads = max(1, min(16, os.cpu_count() or 1))
    res = {}
    for th, budget in ((1, seconds * 0.35), (threads, seconds * 0.65)):
        t1 = timed(th, 1)
        reps = max(1, int(budget / max(t1, 1e-6)))
        t = timed(th, reps)
        res[th] = alg * reps / t / 2**30
    exp = oracle.ref_batch(umem, desc, mode) if kind == "reference" else oracle.batch(umem, desc,
                                                                                        mode)
    assert np.array_equal(out, exp)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f
                          if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": round(res[threads], 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "value_1core": round(res[1], 3), "cpu_model": model,
            "host_cpus": os.cpu_count(),
            "sample": f"{m} frames of the same config ({alg / 1e6:.1f} MB algorithmic), "
                      f"repeated for ~{seconds:.0f} s; xudp/checksum.h "
                      f"{'udp_csum6' if mode == 2 else 'udp_checksum'} compiled -O2 from the "
                      f"reference, static frame partition over {threads} pthreads"}


def pmc_traffic(cid):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", f"pmc_config{cid}.json")
    if os.path.exists(path):
        try:
            return json.load(open(path)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--geometry", default="", help="G,U,K override (tuning)")
    ap.add_argument("--layout", default="packed", choices=["packed", "umem"],
                    help="frames packed at 8-byte boundaries (default) or one per 4096-byte "
                         "chunk as in xudp's TX UMEM")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="time eager launches")
    ap.add_argument("--dist-backend", default="nccl",
                    help="process group for the barrier / timing reductions (nccl = RCCL)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on cuda:0 (1-GPU box)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world, rank, local = dist_env()
    if world != args.gpus and rank == 0:
        print(f"note: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
    dev = torch.device(f"cuda:{0 if args.same_device else local}")
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    def barrier():
        if world > 1:
            dist.barrier()

    cfg = dict(CONFIGS[args.config], id=args.config, layout=args.layout)
    eng = X.Engine(dev.index)
    if args.geometry:
        eng.set_geometry(*[int(v) for v in args.geometry.split(",")])
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    desc, d_desc, bufs, out, first, count = build_batch(cfg, rank, world, torch, dev, eng, sptr)
    alg = X.alg_bytes(desc, cfg["family"])
    len_hint = int(desc["len"].mean()) if count else 0

    def step(k):
        eng.batch_device(bufs[k % len(bufs)], d_desc, count, out, cfg["mode"], 0, len_hint,
                         stream=sptr)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)

    # The K timed launches are captured once into a HIP graph and replayed:
    # the host enqueues one graph instead of K ctypes launches, so short
    # kernels (config 3) are not host-bound.  Every replay runs all K
    # checksum launches.  --no-graph times eager launches instead.
    graph = None
    if not args.no_graph:
        try:
            graph = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(stream)
            with torch.cuda.graph(graph, stream=cap):
                cptr = torch.cuda.current_stream(dev).cuda_stream
                for k in range(args.steps):
                    eng.batch_device(bufs[k % len(bufs)], d_desc, count, out, cfg["mode"], 0,
                                     len_hint, stream=cptr)
            stream.wait_stream(cap)
            graph.replay()  # warm replay
            torch.cuda.synchronize(dev)
        except Exception as e:  # capture unsupported: fall back to eager launches
            print(f"note: graph capture failed ({e}); timing eager launches", file=sys.stderr)
            graph = None
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(1 if graph is not None else args.steps)]
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if graph is not None:
        evs[0][0].record(stream)
        graph.replay()
        evs[0][1].record(stream)
    else:
        for k in range(args.steps):
            evs[k][0].record(stream)
            step(k)
            evs[k][1].record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if graph is not None:
        # HIP events around the replayed launches on the stream they run on;
        # per launch = region / K (includes the ~1 us graph node boundaries)
        kern_ms = evs[0][0].elapsed_time(evs[0][1]) / args.steps
    else:
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))

    # whole-job numbers: max elapsed over ranks, sum of bytes over ranks
    sdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    stats = torch.tensor([elapsed, float(alg), float(count), kern_ms], dtype=torch.float64,
                         device=sdev)
    if world > 1:
        tmax = stats[0:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tot = stats[1:3].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed_max, alg_all, frames_all = float(tmax[0]), float(tot[0]), float(tot[1])
    else:
        elapsed_max, alg_all, frames_all = elapsed, float(alg), float(count)

    # parity spot check of the timed output (rank's last buffer pass)
    ok = None
    if rank == 0 and count:
        import oracle  # checker only
        m = min(count, 4096)
        got = out[:m].cpu().numpy().view(np.uint16)
        ubytes = int(desc["addr"][m - 1]) + int(desc["len"][m - 1])
        hu = bufs[0][:ubytes].cpu().numpy()
        ok = bool(np.array_equal(got, oracle.batch(hu, desc[:m], cfg["mode"])))

    if rank == 0:
        value = alg_all * args.steps / elapsed_max / 2**30
        achieved = alg / (kern_ms * 1e-3) / 1e9  # GB/s, this rank's kernel
        traffic = pmc_traffic(args.config) if args.config in CONFIGS else None
        line = {
            "metric": "device-resident UDP checksum GiB/s + %HBM-peak, 1M x 1472B IPv4 packets"
                      if args.config == 2 else f"device-resident UDP checksum GiB/s (config "
                                                f"{args.config})",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if cfg["shard"] else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SplitMix64 frames generated on device, xudp_packet_udp layout)",
            "config": {"workload": cfg["name"], "frames_per_gpu": count,
                       "frames_total": int(frames_all), "payload_bytes": [cfg["pmin"], cfg["pmax"]],
                       "family": cfg["family"], "mode": MODE_NAMES[cfg["mode"]],
                       "layout": "packed, 8-byte aligned frames" if args.layout == "packed"
                       else "xudp TX UMEM: one frame per 4096-byte chunk",
                       "visiting_order": "automatic (region order if the batch is sparse in "
                                         "the UMEM, else descriptor order)",
                       "rotating_buffers": len(bufs),
                       "alg_bytes_per_step": int(alg_all), "parallelism": f"dp{world}"},
            "pct_hbm_peak": round(100 * achieved / HBM_PEAK_GBS, 2),
            "mpps": round(frames_all * args.steps / elapsed_max / 1e6, 1),
            "kernel_ms": round(kern_ms, 4),
            "timing": "hipGraph replay of the K launches" if graph is not None else "eager",
            "parity_spot_check": ok,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        print(json.dumps(line), flush=True)

    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
