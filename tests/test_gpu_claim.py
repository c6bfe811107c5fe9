"""GPU parity of the claimed-tail schedule (XCSUM_TUNE_CLAIM, csrc/xcsum_csum.h
csum_kernel_claim): the first share of a batch's logical frames scheduled as
csum_kernel does, the rest claimed in chunks from a device counter.  Every
frame must be summed exactly once whatever the split, chunk size, geometry,
order, flags or batch size, and the counter ring must come back to zero after
every launch (the last wave resets its slot) -- checked against the oracle
(pinned to the reference by the CPU tests), bit-exact, including over more
launches than the ring has slots and in a captured graph."""
import numpy as np
import pytest

import libxudp_amd as X
import oracle
from conftest import d2h, h2d

pytestmark = pytest.mark.gpu
ab_only = pytest.mark.skipif(not X.variants_built(),
                             reason="claimed tail: A/B build only (make variant; XCSUM_LIB)")

CLAIM_GEOMS = [(64, 1, 9), (64, 1, 2), (16, 2, 6)]


@pytest.fixture
def claim_engine():
    e = X.Engine(0)
    yield e
    e.close()


def run(torch, eng, umem, desc, mode, flags=0, hint=0):
    dev = torch.device("cuda:0")
    d_umem = h2d(torch, umem, dev)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    out = torch.full((max(len(desc), 1),), 0x5a5a, dtype=torch.int32, device=dev).to(torch.int16)
    eng.batch_device(d_umem, d_desc, len(desc), out, mode, flags, hint,
                     stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    return d2h(out[:len(desc)]).view(np.uint16), d2h(d_umem)


@ab_only
@pytest.mark.parametrize("geom", CLAIM_GEOMS)
@pytest.mark.parametrize("static_64,steps", [(0, 1), (0, 16), (32, 3), (56, 16), (63, 1),
                                             (48, 4096)])
@pytest.mark.parametrize("n", [1, 63, 4097, 60001])
def test_claimed_tail_vs_oracle(torch_cuda, claim_engine, geom, static_64, steps, n):
    """Every split (all claimed .. all but a 64th static), chunk sizes from one
    wave step to more than the batch, batch sizes below one grid step to
    several: every frame summed once, mixed sizes."""
    e = claim_engine
    e.set_geometry(*geom)
    e.set_tuning(X.TUNE_CLAIM, static_64, steps)
    umem, desc = X.gen_frames_host(n, 4, 0, 3000, seed=900 + n + static_64)
    exp = oracle.batch(umem, desc, X.MODE_V4_LEGACY)
    for rep in range(3):          # the slot reset: the next launches see zero
        got, _ = run(torch_cuda, e, umem, desc, X.MODE_V4_LEGACY, 0, int(desc["len"].mean()))
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, (geom, static_64, steps, n, rep, bad[:8].tolist())


@ab_only
@pytest.mark.parametrize("geom", CLAIM_GEOMS)
@pytest.mark.parametrize("flags", [X.F_VERIFY, X.F_IPHDR, X.F_INPLACE, X.F_INPLACE | X.F_IPHDR])
def test_claimed_tail_flags(torch_cuda, claim_engine, geom, flags):
    """The VERIFY and IPHDR instantiations and in-place stores under the
    claimed schedule: results and frame bytes as the oracle says."""
    e = claim_engine
    e.set_geometry(*geom)
    e.set_tuning(X.TUNE_CLAIM, 40, 2)
    umem, desc = X.gen_frames_host(20000, 4, 0, 1472, seed=77)
    if flags & X.F_VERIFY:
        # half the frames carry their checksum, half a wrong one
        good = oracle.batch(umem, desc, X.MODE_V4_RFC)
        for k in range(0, len(desc), 2):
            a0 = int(desc["addr"][k])
            umem[a0 + 40:a0 + 42] = np.frombuffer(int(good[k]).to_bytes(2, "little"), np.uint8)
    exp = oracle.batch(umem, desc, X.MODE_V4_RFC, flags & ~X.F_INPLACE)
    got, after = run(torch_cuda, e, umem, desc, X.MODE_V4_RFC, flags, 1500)
    assert np.array_equal(got, exp)
    if flags & X.F_INPLACE:
        a = desc["addr"].astype(np.int64)
        assert np.array_equal(after[a[:, None] + np.array([40, 41])].copy().view("<u2").ravel(),
                              exp)


@ab_only
@pytest.mark.parametrize("order", [(0, 0), (4, 2), (5, 4)])
def test_claimed_tail_orders_and_sparse(torch_cuda, claim_engine, order):
    """Forced visiting orders, and a sparse batch (xudp's slots: the kernel's
    sparse order), under the claimed schedule."""
    e = claim_engine
    e.set_tuning(X.TUNE_CLAIM, 48, 4)
    e.set_order(*order)
    for kw in (dict(), dict(stride=4096, offset=342)):
        umem, desc = X.gen_frames_host(30000, 4, 0, 1472, seed=5 + order[0], **kw)
        exp = oracle.batch(umem, desc, X.MODE_V4_LEGACY)
        e.set_geometry(64, 1, 9)
        got, _ = run(torch_cuda, e, umem, desc, X.MODE_V4_LEGACY, 0, 1500)
        assert np.array_equal(got, exp), (order, kw)
        e.set_geometry(0)
        got, _ = run(torch_cuda, e, umem, desc, X.MODE_V4_LEGACY, 0, 1500)
        assert np.array_equal(got, exp), (order, kw, "auto")


@ab_only
def test_claim_ring_wraps_and_graph_replays(torch_cuda, claim_engine):
    """More launches than the ring has slots (256), eager, then the same
    launches captured in a graph and replayed: every result exact, so every
    slot was back at zero when it was taken again."""
    torch = torch_cuda
    e = claim_engine
    e.set_tuning(X.TUNE_CLAIM, 32, 2)
    dev = torch.device("cuda:0")
    umem, desc = X.gen_frames_host(5000, 4, 64, 9000, seed=31)
    exp = oracle.batch(umem, desc, X.MODE_V4_LEGACY)
    d_umem = h2d(torch, umem, dev)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    outs = [torch.zeros(len(desc), dtype=torch.int16, device=dev) for _ in range(4)]
    s = torch.cuda.current_stream(dev)
    for k in range(300):
        e.batch_device(d_umem, d_desc, len(desc), outs[k % 4], X.MODE_V4_LEGACY, 0, 4500,
                       stream=s.cuda_stream)
        if k % 50 == 49:
            torch.cuda.synchronize(dev)
            for o in outs:
                assert np.array_equal(d2h(o).view(np.uint16), exp), k
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    cap.wait_stream(s)
    for o in outs:
        o.zero_()
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(g, stream=cap):
        cs = torch.cuda.current_stream(dev).cuda_stream
        for k in range(8):
            e.batch_device(d_umem, d_desc, len(desc), outs[k % 4], X.MODE_V4_LEGACY, 0, 4500,
                           stream=cs)
    for r in range(40):            # 320 launches through 8 captured slots
        g.replay()
    torch.cuda.synchronize(dev)
    for o in outs:
        assert np.array_equal(d2h(o).view(np.uint16), exp)
    assert e.take_errors() == 0


@ab_only
def test_claim_setter_bounds_ab(claim_engine):
    e = claim_engine
    with pytest.raises(X.XcsumError):
        e.set_tuning(X.TUNE_CLAIM, 65, 1)
    with pytest.raises(X.XcsumError):
        e.set_tuning(X.TUNE_CLAIM, -1, 1)
    e.set_tuning(X.TUNE_CLAIM, 64, 0)      # off


def test_claim_refused_by_product_library(claim_engine):
    """libxcsum.so carries no claimed-tail kernel: the knob is refused (only
    'static only', 64, is accepted), so no launch takes a missing kernel."""
    if X.variants_built():
        pytest.skip("A/B build loaded")
    with pytest.raises(X.XcsumError) as e:
        claim_engine.set_tuning(X.TUNE_CLAIM, 56, 16)
    assert e.value.rc == -X.ERR_INVAL
    claim_engine.set_tuning(X.TUNE_CLAIM, 64, 0)
