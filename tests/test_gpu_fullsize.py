"""GPU: full BASELINE sizes.  Frames generated on the device, checksummed by
the kernel, SHA-256 of the output array compared with the digest the
REFERENCE produced over the same frames (tests/golden/digests.json), plus
size-independent properties (verify-after-write, geometry independence)."""
import hashlib

import numpy as np
import pytest

import bench
import libxudp_amd as X
from conftest import h2d, d2h

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def device_batch(torch, engine, cid, first=0, count=None, umem_layout=False):
    cfg = dict(bench.CONFIGS[cid], id=cid)
    count = cfg["n"] if count is None else count
    # umem_layout: xudp's TX UMEM, one frame per 4096-byte chunk;
    # the generator keys bytes by frame index, so the frames are identical
    kw = dict(stride=4096, offset=322 if cfg["family"] == 6 else 342) if umem_layout else {}
    desc, nbytes = X.gen_layout(count, cfg["family"], cfg["pmin"], cfg["pmax"],
                                seed=bench.SEED_BASE ^ cid, first_index=first, **kw)
    dev = torch.device("cuda:0")
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    d_umem = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
    engine.gen_fill_device(d_umem, d_desc, count, cfg["family"], bench.SEED_BASE ^ cid, first)
    return cfg, desc, d_desc, d_umem


def run(torch, engine, d_umem, d_desc, n, mode, flags=0, hint=0):
    out = torch.empty(n, dtype=torch.int16, device="cuda:0")
    engine.batch_device(d_umem, d_desc, n, out, mode, flags, hint)
    torch.cuda.synchronize()
    return d2h(out).view(np.uint16)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u2").tobytes()).hexdigest()


@pytest.mark.parametrize("cid", [2, 3, 4])
def test_config_digest(torch_cuda, engine, digests, cid):
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, cid)
    dg = digests[f"config{cid}"]
    hint = int(desc["len"].mean())
    assert sha(run(torch_cuda, engine, d_umem, d_desc, len(desc), cfg["mode"], 0, hint)) \
        == dg["sha256_out"]
    if cfg["family"] == 4:
        assert sha(run(torch_cuda, engine, d_umem, d_desc, len(desc), X.MODE_V4_RFC, 0, hint)) \
            == dg["sha256_out_v4_rfc"]
    # the frames themselves equal the host generator's (which equals the
    # reference builder's, tests/test_generator.py)
    h = hashlib.sha256()
    host = d2h(d_umem)
    for d in desc:
        h.update(host[d["addr"]:d["addr"] + d["len"]].tobytes())
    assert h.hexdigest() == dg["sha256_frames"]


def test_config2_every_geometry_same_digest(torch_cuda, engine, digests):
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, 2)
    for g in X.GEOMETRIES:
        engine.set_geometry(*g)
        try:
            got = run(torch_cuda, engine, d_umem, d_desc, len(desc), cfg["mode"])
        finally:
            engine.set_geometry(0)
        assert sha(got) == digests["config2"]["sha256_out"], g


@pytest.mark.parametrize("order", [(4, 6), (6, 3), (3, 8)])
def test_config2_visiting_order_same_digest(torch_cuda, engine, digests, order):
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, 2)
    engine.set_order(*order)
    try:
        got = run(torch_cuda, engine, d_umem, d_desc, len(desc), cfg["mode"])
    finally:
        engine.set_order(-1, 0)
    assert sha(got) == digests["config2"]["sha256_out"]


CAL_CANDIDATES = {(-1, 0), (0, 0), (3, 4), (4, 4), (2, 5), (5, 4)}


@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")
@pytest.mark.parametrize("umem_layout", [False, True])
def test_config2_calibrated_order_same_digest(torch_cuda, engine, digests, umem_layout):
    """xcsum_ctx_calibrate_order on config 2 (packed, and in xudp's slots):
    it picks one of its candidates (automatic unless a forced order is >= 1 %
    faster), leaves the context on it, and the output digest is unchanged;
    refused while the stream is being captured."""
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, 2, umem_layout=umem_layout)
    n = len(desc)
    out = torch_cuda.empty(n, dtype=torch_cuda.int16, device="cuda:0")
    s = torch_cuda.cuda.current_stream().cuda_stream
    try:
        pick = engine.calibrate_order(d_umem, d_desc, n, out, cfg["mode"], 0, 1514, stream=s)
        assert pick in CAL_CANDIDATES, pick
        got = run(torch_cuda, engine, d_umem, d_desc, n, cfg["mode"], 0, 1514)
        assert sha(got) == digests["config2"]["sha256_out"], pick
        g = torch_cuda.cuda.CUDAGraph()
        cap = torch_cuda.cuda.Stream()
        err = None
        with torch_cuda.cuda.graph(g, stream=cap):
            try:   # refused before anything is enqueued: the capture ends empty
                engine.calibrate_order(d_umem, d_desc, n, out, cfg["mode"], 0, 1514,
                                       stream=torch_cuda.cuda.current_stream().cuda_stream)
            except X.XcsumError as e:
                err = e.rc
        assert err == -X.ERR_INVAL
    finally:
        engine.set_order(-1, 0)


@pytest.mark.parametrize("cid,umem_layout", [(2, False), (2, True), (3, False), (5, False)])
def test_iphdr_only_digest(torch_cuda, engine, digests, cid, umem_layout):
    """libxudp's IPv4 TX call (XCSUM_F_IPHDR_ONLY) over whole BASELINE
    configs: the output's SHA-256 equals the digest of the reference's own
    xudp_checksum_half (packet.c:43-66) over the same frames
    (digests.json sha256_iphdr, tests/golden/make_golden.py --only-iphdr)."""
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, cid, umem_layout=umem_layout)
    got = run(torch_cuda, engine, d_umem, d_desc, len(desc), cfg["mode"], X.F_IPHDR_ONLY, 0)
    assert sha(got) == digests[f"config{cid}"]["sha256_iphdr"]


def test_calibration_leaves_error_count(torch_cuda, engine):
    """The thousands of calls xcsum_ctx_calibrate_order makes count their
    malformed frames apart: take_errors after a calibration is
    what the caller's own calls produced."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    umem, desc = X.gen_frames_host(2000, 4, 0, 1472, seed=77)
    desc["len"][::20] = 10                       # 100 malformed frames
    d_umem = h2d(torch, umem, dev)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    out = torch.empty(len(desc), dtype=torch.int16, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    engine.take_errors()
    try:
        engine.calibrate_order(d_umem, d_desc, len(desc), out, X.MODE_V4_LEGACY, 0, 1514, stream=s)
        assert engine.take_errors() == 0
        engine.batch_device(d_umem, d_desc, len(desc), out, X.MODE_V4_LEGACY, 0, 1514, stream=s)
        assert engine.take_errors() == 100
    finally:
        engine.set_order(-1, 0)


@pytest.mark.parametrize("cid", [2, 3, 4])
def test_umem_layout_same_digest(torch_cuda, engine, digests, cid):
    """The same frames in xudp's 4096-byte-chunk UMEM layout: the automatic
    visiting order switches to regions there (sparse batch) -- same output."""
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, cid, umem_layout=True)
    assert int(desc["addr"][1] - desc["addr"][0]) == 4096
    for hint in (0, int(desc["len"][0])):
        got = run(torch_cuda, engine, d_umem, d_desc, len(desc), cfg["mode"], 0, hint)
        assert sha(got) == digests[f"config{cid}"]["sha256_out"], hint


def test_config5_digest_8m_mixed(torch_cuda, engine, digests):
    """8M frames of U[64, 9000] bytes (38 GB algorithmic) on one GPU, and the
    byte-balanced 8-way shards of bench.py concatenated."""
    dg = digests["config5"]
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, 5)
    out = run(torch_cuda, engine, d_umem, d_desc, len(desc), cfg["mode"], 0,
              int(desc["len"].mean()))
    assert sha(out) == dg["sha256_out"]
    assert X.alg_bytes(desc, 4) == dg["alg_bytes"]
    del d_umem, d_desc
    torch_cuda.cuda.empty_cache()
    parts = []
    for r in range(8):
        first, count = bench.rank_slice(cfg, r, 8)
        c, dsc, dd, du = device_batch(torch_cuda, engine, 5, first, count)
        parts.append(run(torch_cuda, engine, du, dd, count, cfg["mode"]))
        del du, dd
    assert sha(np.concatenate(parts)) == dg["sha256_out"]


def test_config5_every_jumbo_geometry_same_digest(torch_cuda, engine, digests):
    """Config 5 through the frame-group kernel (and, in a variants build,
    the segmented stream at every D): the reference's digest each time;
    then INPLACE and a VERIFY pass over the written frames."""
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, 5)
    for g in (X.SEG_GEOMETRIES + X.SEG_ATOM_GEOMETRIES if X.variants_built() else []) + [(64, 1, 9)]:
        engine.set_geometry(*g)
        try:
            got = run(torch_cuda, engine, d_umem, d_desc, len(desc), cfg["mode"])
        finally:
            engine.set_geometry(0)
        assert sha(got) == digests["config5"]["sha256_out"], g
    engine.set_geometry(*(X.SEG_GEOMETRIES[-1] if X.variants_built() else (64, 1, 9)))
    try:
        run(torch_cuda, engine, d_umem, d_desc, len(desc), X.MODE_V4_RFC, X.F_INPLACE)
        ok = run(torch_cuda, engine, d_umem, d_desc, len(desc), X.MODE_V4_RFC, X.F_VERIFY)
    finally:
        engine.set_geometry(0)
    assert (ok == 0).all()


@pytest.mark.parametrize("cid,mode", [(2, X.MODE_V4_RFC), (4, X.MODE_V6)])
def test_verify_after_inplace_write(torch_cuda, engine, cid, mode):
    """RFC property: once udp->check holds the checksum, the one's complement
    sum over the span (check included) is 0xffff, so a second pass yields
    ~0 -> mapped 0xffff for every frame."""
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, cid)
    first = run(torch_cuda, engine, d_umem, d_desc, len(desc), mode, X.F_INPLACE)
    second = run(torch_cuda, engine, d_umem, d_desc, len(desc), mode)
    assert (second == 0xffff).all()
    assert (first != 0).all()


@pytest.mark.parametrize("cid,mode", [(2, X.MODE_V4_RFC), (4, X.MODE_V6)])
def test_verify_flag_after_inplace_write(torch_cuda, engine, cid, mode):
    cfg, desc, d_desc, d_umem = device_batch(torch_cuda, engine, cid)
    run(torch_cuda, engine, d_umem, d_desc, len(desc), mode, X.F_INPLACE | X.F_IPHDR)
    ok = run(torch_cuda, engine, d_umem, d_desc, len(desc), mode, X.F_VERIFY | X.F_IPHDR)
    assert (ok == 0).all()
