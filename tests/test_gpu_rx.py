"""GPU: xcsum_rx_device (the receive path, csrc/xcsum_rx.hip) through the C ABI
against the fixture records (tests/golden/rx_fixtures.npz: the reference's
packet_parse() + the oracle's fill/verify), against the oracle on generated
batches, and as a size-independent round trip at BASELINE sizes: frames the
TX kernel checksummed in place all verify; one flipped bit in each fails."""
import os
import sys

import numpy as np
import pytest

import bench
import libxudp_amd as X
from conftest import h2d, d2h
import oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
import rx_frames  # noqa: E402

FLAGS = {"plain": 0, "verify": X.F_VERIFY, "iphdr": X.F_VERIFY | X.F_IPHDR}


@pytest.fixture(scope="module")
def rx():
    z = np.load(os.path.join(GOLDEN, "rx_fixtures.npz"))
    d = {k: z[k] for k in z.files}
    d["desc"] = d["desc"].view(X.DESC_DTYPE)
    return d


def run_rx(torch, eng, umem, desc, flags, len_hint=0, geometry=None):
    dev = torch.device("cuda:0")
    d_umem = h2d(torch, umem, dev)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    d_msgs = torch.full((max(len(desc), 1) * 64,), 0xA5, dtype=torch.uint8, device=dev)
    d_count = torch.full((1,), 77, dtype=torch.int32, device=dev)
    if geometry:
        # the context's forced receive geometry (XCSUM_TUNE_RX_GEOMETRY: G, K, U)
        eng.set_tuning(X.TUNE_RX_GEOMETRY, *[int(v) for v in str(geometry).split(",")])
    try:
        eng.rx_device(d_umem, d_desc, len(desc), d_msgs, d_count, flags, len_hint)
        torch.cuda.synchronize()
    finally:
        if geometry:
            eng.set_tuning(X.TUNE_RX_GEOMETRY, 0)
    recs = d2h(d_msgs)[:len(desc) * 64].view(X.RX_MSG_DTYPE)
    return recs, int(d_count.cpu().item())


GEOMETRIES = ["2,4,1", "2,4,2", "4,2,1", "4,2,2", "8,1,2", "8,2,1", "16,2,1", "16,3,1", "16,6,1", "16,6,2", "64,9,1",
              "4,2,0", "8,2,0", "16,3,0", "16,6,0", "32,3,0", "64,2,0", "64,9,0", "64,8,3"]


def test_rx_geometry_list_matches_kernel():
    src = open(os.path.join(os.path.dirname(GOLDEN), "..", "libxudp_amd", "csrc",
                            "xcsum_rx.hip")).read()
    i = src.index("#define XCSUM_RX_GEOMETRIES")
    block = src[i:src.index("\n\n", i)]
    import re
    assert sorted(GEOMETRIES) == sorted(",".join(t) for t in
                                        re.findall(r"X\((\d+), (\d+), (\d+)\)", block))


@pytest.mark.parametrize("geometry", GEOMETRIES)
@pytest.mark.parametrize("name", sorted(FLAGS))
def test_rx_matches_fixtures(torch_cuda, engine, rx, name, geometry):
    recs, count = run_rx(torch_cuda, engine, rx["umem"], rx["desc"], FLAGS[name],
                         geometry=geometry)
    exp = rx[f"rec_{name}"].view(X.RX_MSG_DTYPE)
    bad = np.nonzero(recs.view(np.uint8).reshape(-1, 64) != exp.view(np.uint8).reshape(-1, 64))
    assert len(bad[0]) == 0, f"records differ: {sorted(set(bad[0].tolist()))[:10]}"
    assert count == int((exp["status"] == X.RX_OK).sum())


@pytest.mark.parametrize("geometry", [None] + GEOMETRIES)
def test_rx_generated_vs_oracle(torch_cuda, engine, geometry):
    """6k frames: the corpus under three seeds, at irregular offsets."""
    frames = []
    for seed in (1, 2, 3):
        frames += [f for f, _ in rx_frames.corpus(seed=seed)]
    rng = np.random.default_rng(5)
    frames = [frames[i] for i in rng.permutation(len(frames))] * 10
    umem, offs, lens = rx_frames.layout(frames, rng)
    desc = np.zeros(len(frames), dtype=X.DESC_DTYPE)
    desc["addr"], desc["len"] = offs, lens
    exps = {flags: oracle.rx_batch(umem, desc, flags) for flags in FLAGS.values()}
    for flags in FLAGS.values():
        for hint in ((0, 100, 1500, 9000) if geometry is None else (0,)):
            recs, count = run_rx(torch_cuda, engine, umem, desc, flags, hint, geometry)
            exp = exps[flags]
            assert np.array_equal(recs.view(np.uint8), exp.view(np.uint8)), (flags, hint)
            assert count == int((exp["status"] == X.RX_OK).sum())


@pytest.mark.parametrize("geometry", [None, "64,8,3"])
def test_rx_stream_small_frames_vs_oracle(torch_cuda, engine, geometry):
    """Packed small frames, the stream receive kernel's fast path (one 8 KiB
    region per 64 frames): every corpus frame of at most 128 bytes (padding,
    options, ihl < 5, extension headers, stats requests, corrupted, truncated,
    junk), under four seeds, at irregular offsets, and a batch size that ends
    mid-wave."""
    frames = []
    for seed in (1, 2, 3, 4):
        frames += [f for f, _ in rx_frames.corpus(seed=seed) if len(f) <= 128]
    rng = np.random.default_rng(8)
    frames = [frames[i] for i in rng.permutation(len(frames))] * 20
    frames = frames[:len(frames) - 37]
    umem, offs, lens = rx_frames.layout(frames, rng)
    desc = np.zeros(len(frames), dtype=X.DESC_DTYPE)
    desc["addr"], desc["len"] = offs, lens
    for flags in FLAGS.values():
        exp = oracle.rx_batch(umem, desc, flags)
        recs, count = run_rx(torch_cuda, engine, umem, desc, flags, 100, geometry)
        bad = np.nonzero(recs.view(np.uint8).reshape(-1, 64) != exp.view(np.uint8).reshape(-1, 64))
        assert len(bad[0]) == 0, (flags, sorted(set(bad[0].tolist()))[:10])
        assert count == int((exp["status"] == X.RX_OK).sum())


def umem_chunks(frames, rng, n):
    """n frames one per chunk (xudp's UMEM: frame i in chunk i at a fixed
    headroom plus a small jitter), the layout the region order is for"""
    chunk = 4096
    while chunk < max(len(f) for f in frames) + 512:
        chunk *= 2
    pick = [frames[i] for i in rng.integers(0, len(frames), n)]
    offs = np.arange(n, dtype=np.uint64) * chunk + 256 + rng.integers(0, 8, n).astype(np.uint64)
    umem = np.zeros(n * chunk + 64, dtype=np.uint8)
    for o, f in zip(offs, pick):
        umem[int(o):int(o) + len(f)] = np.frombuffer(f, dtype=np.uint8)
    desc = np.zeros(n, dtype=X.DESC_DTYPE)
    desc["addr"], desc["len"] = offs, [len(f) for f in pick]
    return umem, desc


@pytest.mark.parametrize("order", ["auto", "0"])
@pytest.mark.parametrize("geometry", [None, "4,2,1", "16,3,1", "4,2,0", "32,3,0", "64,9,0", "64,8,3"])
def test_rx_sparse_umem_vs_oracle(torch_cuda, engine, geometry, order):
    """Frames one per UMEM chunk (sparse: the kernels visit them in region
    order, launch_rx) and a batch size that leaves the last tiles partly or
    wholly past the end: the same records and count as the oracle, with the
    order on and off (XCSUM_TUNE_RX_ORDER 0)."""
    frames = [f for f, _ in rx_frames.corpus(seed=11)]
    rng = np.random.default_rng(12)
    umem, desc = umem_chunks(frames, rng, 4099)
    engine.set_tuning(X.TUNE_RX_ORDER, -1 if order == "auto" else int(order))
    try:
        for flags in FLAGS.values():
            exp = oracle.rx_batch(umem, desc, flags)
            recs, count = run_rx(torch_cuda, engine, umem, desc, flags, 1500, geometry)
            bad = np.nonzero(recs.view(np.uint8).reshape(-1, 64) != exp.view(np.uint8).reshape(-1, 64))
            assert len(bad[0]) == 0, (flags, sorted(set(bad[0].tolist()))[:10])
            assert count == int((exp["status"] == X.RX_OK).sum())
    finally:
        engine.set_tuning(X.TUNE_RX_ORDER, -1)


def test_rx_empty_batch(torch_cuda, engine):
    dev = torch_cuda.device("cuda:0")
    d = torch_cuda.zeros(64, dtype=torch_cuda.uint8, device=dev)
    c = torch_cuda.full((1,), 5, dtype=torch_cuda.int32, device=dev)
    engine.rx_device(d, d, 0, d, c, X.F_VERIFY)
    torch_cuda.cuda.synchronize()
    assert int(c.item()) == 0
    with pytest.raises(X.XcsumError):
        engine.rx_device(None, None, 3, None)
    with pytest.raises(X.XcsumError):   # d_umem must be 4-byte aligned
        engine.rx_device(d.data_ptr() + 1, d, 1, d, c, X.F_VERIFY)


@pytest.mark.slow
@pytest.mark.parametrize("cid", [2, 3, 4])
def test_rx_round_trip_full_size(torch_cuda, engine, cid):
    """TX checksums written in place (RFC; IPv4 header too) verify on RX, at
    the BASELINE config's size; a flipped payload bit fails every frame."""
    cfg = dict(bench.CONFIGS[cid], id=cid)
    n = cfg["n"]
    desc, nbytes = X.gen_layout(n, cfg["family"], cfg["pmin"], cfg["pmax"],
                                seed=bench.SEED_BASE ^ cid)
    dev = torch_cuda.device("cuda:0")
    d_desc = h2d(torch_cuda, desc.view(np.uint8), dev)
    d_umem = torch_cuda.empty(nbytes + 64, dtype=torch_cuda.uint8, device=dev)
    engine.gen_fill_device(d_umem, d_desc, n, cfg["family"], bench.SEED_BASE ^ cid, 0)
    mode = X.MODE_V6 if cfg["family"] == 6 else X.MODE_V4_RFC
    engine.batch_device(d_umem, d_desc, n, None, mode, X.F_INPLACE | X.F_IPHDR)
    d_msgs = torch_cuda.empty(n * 64, dtype=torch_cuda.uint8, device=dev)
    d_count = torch_cuda.zeros(1, dtype=torch_cuda.int32, device=dev)
    engine.rx_device(d_umem, d_desc, n, d_msgs, d_count, X.F_VERIFY | X.F_IPHDR,
                     int(desc["len"][0]))
    torch_cuda.cuda.synchronize()
    recs = d2h(d_msgs).view(X.RX_MSG_DTYPE)
    assert int(d_count.item()) == n
    assert (recs["status"] == X.RX_OK).all()
    hdr = 42 if cfg["family"] == 4 else 62
    assert np.array_equal(recs["body"], desc["addr"] + hdr)
    assert np.array_equal(recs["size"], desc["len"] - hdr)
    # flip one bit of the last payload byte of every frame
    last = h2d(torch_cuda, (desc["addr"] + desc["len"] - 1).astype(np.int64), dev)
    d_umem[last] ^= 0x10
    engine.rx_device(d_umem, d_desc, n, d_msgs, d_count, X.F_VERIFY, int(desc["len"][0]))
    torch_cuda.cuda.synchronize()
    recs = d2h(d_msgs).view(X.RX_MSG_DTYPE)
    assert int(d_count.item()) == 0
    assert (recs["status"] == X.RX_CSUM).all()


@pytest.mark.parametrize("zerocopy", [False, True])
def test_rx_host_vs_oracle(torch_cuda, engine, zerocopy):
    """xcsum_rx_host on host-resident frames (staged copies, or zero-copy from
    a registered UMEM): the same records as the oracle, > 65,536 frames so the
    batch is cut into several chunks over both staging slots."""
    frames = []
    for seed in (4, 5):
        frames += [f for f, _ in rx_frames.corpus(seed=seed)]
    rng = np.random.default_rng(9)
    frames = [frames[i] for i in rng.integers(0, len(frames), 70000)]
    umem, offs, lens = rx_frames.layout(frames, rng)
    desc = np.zeros(len(frames), dtype=X.DESC_DTYPE)
    desc["addr"], desc["len"] = offs, lens
    flags_zc = X.F_ZEROCOPY if zerocopy else 0
    if zerocopy:
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        engine.register_umem(umem)
    try:
        for flags in FLAGS.values():
            msgs = np.full(len(desc) * 64, 0xA5, dtype=np.uint8).view(X.RX_MSG_DTYPE)
            count = engine.rx_host(umem, desc, msgs, flags | flags_zc)
            exp = oracle.rx_batch(umem, desc, flags)
            assert np.array_equal(msgs.view(np.uint8), exp.view(np.uint8)), flags
            assert count == int((exp["status"] == X.RX_OK).sum())
    finally:
        if zerocopy:
            engine.unregister_umem(umem)


@pytest.mark.parametrize("register", [False, True])
@pytest.mark.parametrize("n", [100, 5000, 70000])
def test_rx_host_sparse_umem_vs_oracle(engine, n, register):
    """xcsum_rx_host on frames one per UMEM chunk, as an RX ring hands them
    over: from a pageable UMEM gathered frame by frame into the pinned stage
    (copy-free up to 256 KiB of frames, staged copies above, two chunks at
    70,000 frames), from a registered one read in place (zerocopy_pays); the
    records hold UMEM offsets either way."""
    frames = [f for f, _ in rx_frames.corpus(seed=13)]
    rng = np.random.default_rng(14)
    umem, desc = umem_chunks(frames, rng, n)
    if register:
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        engine.register_umem(umem)
    try:
        for flags in FLAGS.values():
            msgs = np.full(n * 64, 0xA5, dtype=np.uint8).view(X.RX_MSG_DTYPE)
            count = engine.rx_host(umem, desc, msgs, flags)
            exp = oracle.rx_batch(umem, desc, flags)
            bad = np.nonzero(msgs.view(np.uint8).reshape(-1, 64) !=
                             exp.view(np.uint8).reshape(-1, 64))
            assert len(bad[0]) == 0, (flags, sorted(set(bad[0].tolist()))[:10])
            assert count == int((exp["status"] == X.RX_OK).sum())
    finally:
        if register:
            engine.unregister_umem(umem)


def test_rx_host_errors(engine):
    umem = np.zeros(4096, dtype=np.uint8)
    desc = np.zeros(1, dtype=X.DESC_DTYPE)
    desc["len"] = 64
    msgs = np.zeros(1, dtype=X.RX_MSG_DTYPE)
    assert engine.rx_host(umem, desc[:0], msgs[:0], X.F_VERIFY) == 0
    with pytest.raises(X.XcsumError):   # zero-copy needs a registered UMEM
        engine.rx_host(umem, desc, msgs, X.F_VERIFY | X.F_ZEROCOPY)
    assert engine.rx_host(umem, desc, msgs, X.F_VERIFY) == 0
    assert msgs["status"][0] == X.RX_PARSE
