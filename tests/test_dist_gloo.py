"""CPU, world_size 2 and 8 (gloo): the multi-GPU path's partitioning, exercised
exactly as bench.py does it (rank_slice -> per-rank generation -> per-rank
checksums, no data-path collective), checked against one single-process run.
Only the timing reduction (MAX of elapsed) and the byte count (SUM) cross
ranks, as in bench.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import libxudp_amd as X
import oracle

CFG_SMALL = dict(n=6000, family=4, pmin=64, pmax=9000, mode=0, shard=True, id=5, name="t")
CFG_WEAK = dict(n=500, family=6, pmin=1472, pmax=1472, mode=2, shard=False, id=4, name="t")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_outputs(cfg, rank, world):
    first, count = bench.rank_slice(cfg, rank, world)
    umem, desc = X.gen_frames_host(count, cfg["family"], cfg["pmin"], cfg["pmax"],
                                   seed=bench.SEED_BASE ^ cfg["id"], first_index=first)
    return first, oracle.batch(umem, desc, cfg["mode"]), X.alg_bytes(desc, cfg["family"])


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    for name, cfg in (("strong", CFG_SMALL), ("weak", CFG_WEAK)):
        first, out, alg = rank_outputs(cfg, rank, world)
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        b = torch.tensor([float(alg), float(len(out))], dtype=torch.float64)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        res[name] = (first, out, float(t[0]), b.tolist())
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_partition_matches_single_process(world):
    """world 2, and 8 as in the driver's 8-GPU run (gloo processes on the CPU)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # strong scaling (config-5 style): shards tile the job in rank order,
    # outputs concatenate to the single-process run, byte counts sum
    firsts = [got[r]["strong"][0] for r in range(world)]
    outs = [got[r]["strong"][1] for r in range(world)]
    assert firsts == [int(sum(len(o) for o in outs[:r])) for r in range(world)]
    assert all(got[r]["strong"][2] == float(world) for r in range(world))   # MAX over ranks
    whole = rank_outputs(CFG_SMALL, 0, 1)
    assert np.array_equal(np.concatenate(outs), whole[1])
    assert got[0]["strong"][3] == [float(whole[2]), float(CFG_SMALL["n"])]
    # byte-balanced: no shard carries more than its share plus one frame
    per = [float(X.alg_bytes(*_shard_desc(CFG_SMALL, r, world))) for r in range(world)]
    assert max(per) - min(per) <= 2 * (CFG_SMALL["pmax"] + 16)
    # weak scaling: each rank owns its own n frames, rank r starts at r*n
    assert [got[r]["weak"][0] for r in range(world)] == [r * CFG_WEAK["n"] for r in range(world)]
    big = dict(CFG_WEAK, n=world * CFG_WEAK["n"])
    whole = rank_outputs(big, 0, 1)
    assert np.array_equal(np.concatenate([got[r]["weak"][1] for r in range(world)]), whole[1])


def _shard_desc(cfg, rank, world):
    first, count = bench.rank_slice(cfg, rank, world)
    desc, _ = X.gen_layout(count, cfg["family"], cfg["pmin"], cfg["pmax"],
                           seed=bench.SEED_BASE ^ cfg["id"], first_index=first)
    return desc, cfg["family"]


def test_bench_helpers_present_and_real_bytes():
    """bench.py's helpers exist (the GPU-only main() calls them) and the real
    byte count is the union of touched 64-byte lines + 18 bytes per frame."""
    import bench
    for name in ("digest_check", "stream_ceiling", "gpu_clocks", "cpu_baseline", "pmc_traffic",
                 "host_cpu_facts", "real_bytes", "rank_slice", "build_batch", "inplace_ceiling",
                 "lib_sha16", "parse_flags", "alg_bytes_flags", "order_ab", "span_ceiling",
                 "launch_plan", "launch_ranks", "parse_shard"):
        assert callable(getattr(bench, name)), name
    d = np.zeros(3, dtype=X.DESC_DTYPE)
    d["addr"] = [0, 100, 4096]
    d["len"] = [100, 28, 64]
    assert bench.real_bytes(d) == (2 + 1) * 64 + 3 * 18
    # the visiting-order A/B: descriptor order and forced region orders
    assert (0, 0) in bench.ORDER_AB and (3, 4) in bench.ORDER_AB
    # the in-place kernel without IPHDR (csrc/xcsum_csum_tl.hip) is found
    # by name in the library's code objects, so PMC counters can key on it
    assert bench.kernel_sha16("void xcsum::csum_kernel_tl<16, 2, 6, 0, 4>(xcsum::CsumArgs)")


def test_bench_flags_and_algorithmic_bytes():
    """--flags parsing and the algorithmic bytes per mode:
    span + 2-byte result; in place without a result array, + 2 per written
    check field, + the 12 IPv4 header bytes before the addresses with IPHDR."""
    import bench
    assert bench.parse_flags("") == 0
    assert bench.parse_flags("inplace,iphdr") == X.F_INPLACE | X.F_IPHDR
    with pytest.raises(SystemExit):
        bench.parse_flags("bogus")
    d = np.zeros(2, dtype=X.DESC_DTYPE)
    d["len"] = [1514, 106]                       # IPv4 payloads 1472 and 64
    span = (1472 + 16) + (64 + 16)
    assert bench.alg_bytes_flags(d, 4, 0, True) == span + 4
    assert bench.alg_bytes_flags(d, 4, X.F_INPLACE, False) == span + 4
    assert bench.alg_bytes_flags(d, 4, X.F_INPLACE | X.F_IPHDR, False) == span + 24 + 8
    assert bench.alg_bytes_flags(d, 4, X.F_VERIFY | X.F_IPHDR, True) == span + 24 + 4
    d6 = np.zeros(1, dtype=X.DESC_DTYPE)
    d6["len"] = [1534]
    assert bench.alg_bytes_flags(d6, 6, X.F_INPLACE | X.F_IPHDR, False) == 1472 + 40 + 2


def test_pmc_traffic_only_from_the_same_library(tmp_path, monkeypatch):
    """roofline.traffic comes from a committed PMC summary only when it was
    taken on this very code: the counted kernel's machine-code hash
    (kernel_sha16) when the summary has one, else the whole device code
    (lib_sha16); otherwise null + reason."""
    import json
    import bench
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    d = tmp_path / "profiles" / "r03"
    d.mkdir(parents=True)
    (d / "pmc_config2.json").write_text(json.dumps({"hbm_bytes_per_launch": 123,
                                                    "lib_sha16": "aaaa"}))
    assert bench.pmc_traffic(2, "packed", 0, "aaaa")[0] == 123
    t, src, why, _ = bench.pmc_traffic(2, "packed", 0, "bbbb")
    assert t is None and src.endswith("pmc_config2.json") and "aaaa" in why
    t, src, why, _ = bench.pmc_traffic(3, "packed", 0, "aaaa")
    assert t is None and src is None and why
    (d / "pmc_config2_f3.json").write_text(json.dumps({"hbm_bytes_per_launch": 7,
                                                       "lib_sha16": "aaaa"}))
    assert bench.pmc_traffic(2, "packed", X.F_INPLACE | X.F_IPHDR, "aaaa")[0] == 7
    # kernel-keyed: the library's own csum_kernel<16, 2, 6, 0> code decides,
    # whatever the whole-library hash says
    kern = "void xcsum::csum_kernel<16, 2, 6, 0>(xcsum::CsumArgs)"
    ksha = bench.kernel_sha16(kern)
    assert ksha and ksha != bench.kernel_sha16(
        "void xcsum::csum_kernel<16, 2, 6, 2>(xcsum::CsumArgs)")
    (d / "pmc_config4.json").write_text(json.dumps({"hbm_bytes_per_launch": 9, "kernel": [kern],
                                                    "kernel_sha16": ksha,
                                                    "lib_sha16": "zzzz"}))
    t, _, why, got = bench.pmc_traffic(4, "packed", 0, "aaaa")
    assert t == 9 and why is None and got == ksha
    (d / "pmc_config4.json").write_text(json.dumps({"hbm_bytes_per_launch": 9, "kernel": [kern],
                                                    "kernel_sha16": "0000"}))
    t, _, why, got = bench.pmc_traffic(4, "packed", 0, "aaaa")
    assert t is None and "0000" in why and got == ksha


def test_kernel_sha16_reads_the_fatbin():
    """kernel_sha16 finds every product checksum kernel in libxcsum.so's
    gfx950 code objects (no GPU needed) and tells them apart."""
    import bench
    names = ["void xcsum::csum_kernel<16, 2, 6, 0>(xcsum::CsumArgs)",
             "void xcsum::csum_kernel<16, 2, 6, 2>(xcsum::CsumArgs)",
             "void xcsum::csum_kernel<64, 1, 9, 0>(xcsum::CsumArgs)",
             "void xcsum::csum_stream_kernel<8>(xcsum::CsumArgs)"]
    hs = [bench.kernel_sha16(n) for n in names]
    assert all(hs) and len(set(hs)) == len(hs)
    assert bench.kernel_sha16("void xcsum::no_such_kernel<1>(xcsum::CsumArgs)") is None


def test_cpu_baseline_legs_report_their_seconds():
    """cpu_baseline times every leg after an untimed warm repetition and
    reports each leg's measured seconds and the usable cores; the sample
    text is generated from those numbers."""
    import bench
    cfg = dict(bench.CONFIGS[3], id=3, n=4096)
    r = bench.cpu_baseline(cfg, seconds=0.6)
    assert r["unit"] == "GiB/s" and r["value"] > 0 and r["cores"] >= 1
    assert set(r["seconds_by_threads"]) == set(r["by_threads"])
    assert r["cores_usable"] >= 1
    assert r["seconds_total"] < 10
    for th, sec in r["seconds_by_threads"].items():
        assert f"{th} thread" in r["sample"] and sec > 0
