"""GPU parity: the gfx950 kernel (through the C ABI) vs the reference.

Expected values come from the reference's own checksum.h / packet.c
(tests/golden, made by tests/golden/make_golden.py) and, for generated
inputs, from the oracle restatement (oracle/xcsum_oracle.c), itself pinned
to the reference by the CPU tests.  Integer work: bit-exact, no tolerance.
"""
import contextlib

import numpy as np
import pytest

import libxudp_amd as X
import oracle
from conftest import golden_desc, h2d, d2h

pytestmark = pytest.mark.gpu

# every product geometry, plus the A/B kernels when XCSUM_LIB loads a variants
# build (csrc/variants/)
GEOMETRIES = X.GEOMETRIES + X.variant_geometries()
# the default pick plus the stream kernels (and the A/B kernels of a variants
# build): the feature tests below run under each, so every kernel sees
# INPLACE/IPHDR/VERIFY, ragged and maximum sizes
FEATURE_GEOMS = [None] + X.STREAM_GEOMETRIES + X.variant_geometries()


@contextlib.contextmanager
def geometry(engine, geom):
    if geom is not None:
        engine.set_geometry(*geom)
    try:
        yield
    finally:
        engine.set_geometry(0)


def run_device(torch, eng, umem, desc, mode, flags=0, len_hint=0, out=True):
    dev = torch.device("cuda:0")
    d_umem = h2d(torch, umem, dev)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    d_out = torch.full((max(len(desc), 1),), 0x5a5a, dtype=torch.int32,
                       device=dev).to(torch.int16) if out else None
    s = torch.cuda.current_stream(dev).cuda_stream
    eng.batch_device(d_umem, d_desc, len(desc), d_out, mode, flags, len_hint, stream=s)
    torch.cuda.synchronize(dev)
    res = d2h(d_out[:len(desc)]).view(np.uint16) if out else None
    return res, d2h(d_umem)


@pytest.mark.parametrize("geom", GEOMETRIES)
def test_golden_v4_legacy_all_geometries(torch_cuda, engine, golden, geom):
    sel = np.nonzero(golden["family"] == 4)[0]
    engine.set_geometry(*geom)
    try:
        got, _ = run_device(torch_cuda, engine, golden["umem"], golden_desc(golden, sel),
                            X.MODE_V4_LEGACY)
    finally:
        engine.set_geometry(0)
    exp = golden["exp_legacy"][sel]
    assert np.array_equal(got, exp), f"{int((got != exp).sum())} mismatches"


@pytest.mark.parametrize("geom", GEOMETRIES)
def test_golden_v6_all_geometries(torch_cuda, engine, golden, geom):
    sel = np.nonzero(golden["family"] == 6)[0]
    engine.set_geometry(*geom)
    try:
        got, _ = run_device(torch_cuda, engine, golden["umem"], golden_desc(golden, sel),
                            X.MODE_V6)
    finally:
        engine.set_geometry(0)
    assert np.array_equal(got, golden["exp_v6"][sel])


def test_golden_v4_rfc(torch_cuda, engine, golden):
    sel = np.nonzero(golden["family"] == 4)[0]
    got, _ = run_device(torch_cuda, engine, golden["umem"], golden_desc(golden, sel),
                        X.MODE_V4_RFC)
    assert np.array_equal(got, golden["exp_rfc"][sel])


def test_golden_quirk_cases_present_and_exact(torch_cuda, engine, golden):
    """Frames where udp_checksum()'s dropped carry makes legacy != RFC."""
    q = np.nonzero((golden["family"] == 4) & (golden["exp_legacy"] != golden["exp_rfc"]))[0]
    assert len(q) >= 100
    got, _ = run_device(torch_cuda, engine, golden["umem"], golden_desc(golden, q),
                        X.MODE_V4_LEGACY)
    assert np.array_equal(got, golden["exp_legacy"][q])


@pytest.mark.parametrize("len_hint", [0, 100, 200, 500, 1500, 9000])
def test_golden_auto_mixed_families(torch_cuda, engine, golden, len_hint):
    fam = golden["family"]
    exp = np.where(fam == 6, golden["exp_v6"], golden["exp_legacy"])
    got, _ = run_device(torch_cuda, engine, golden["umem"], golden_desc(golden), X.MODE_AUTO,
                        len_hint=len_hint)
    assert np.array_equal(got, exp)
    exp_rfc = np.where(fam == 6, golden["exp_v6"], golden["exp_rfc"])
    got, _ = run_device(torch_cuda, engine, golden["umem"], golden_desc(golden), X.MODE_AUTO,
                        X.F_V4_RFC, len_hint=len_hint)
    assert np.array_equal(got, exp_rfc)


@pytest.mark.parametrize("geom", FEATURE_GEOMS)
def test_golden_inplace_and_iphdr(torch_cuda, engine, golden, geom):
    with geometry(engine, geom):
        _test_golden_inplace_and_iphdr_body(torch_cuda, engine, golden)


def _test_golden_inplace_and_iphdr_body(torch_cuda, engine, golden):
    """INPLACE writes udp->check, IPHDR writes iph->check == xudp_checksum_half."""
    fam = golden["family"]
    umem = golden["umem"].copy()
    desc = golden_desc(golden)
    got, after = run_device(torch_cuda, engine, umem, desc, X.MODE_AUTO,
                            X.F_INPLACE | X.F_IPHDR)
    for i, d in enumerate(desc):
        a = int(d["addr"])
        f = after[a:a + int(d["len"])]
        if fam[i] == 6:
            assert int(f[60:62].view("<u2")[0]) == golden["exp_v6"][i]
        else:
            assert int(f[40:42].view("<u2")[0]) == golden["exp_legacy"][i]
            assert int(f[24:26].view("<u2")[0]) == golden["exp_iphdr"][i]
    # nothing outside the check fields changed
    mask = np.ones(len(umem), dtype=bool)
    for i, d in enumerate(desc):
        a = int(d["addr"])
        if fam[i] == 6:
            mask[a + 60:a + 62] = False
        else:
            mask[a + 40:a + 42] = False
            mask[a + 24:a + 26] = False
    assert np.array_equal(after[mask], golden["umem"][mask])
    # NO_OUT: out == NULL with INPLACE is legal
    _, after2 = run_device(torch_cuda, engine, golden["umem"].copy(), desc, X.MODE_AUTO,
                           X.F_INPLACE | X.F_IPHDR, out=False)
    assert np.array_equal(after2, after)


@pytest.mark.parametrize("family", [4, 6])
@pytest.mark.parametrize("layout", ["packed8", "packed1", "umem_mirror"])
@pytest.mark.parametrize("geom", FEATURE_GEOMS)
def test_generated_vs_oracle(torch_cuda, engine, family, layout, geom):
    with geometry(engine, geom):
        _test_generated_vs_oracle_body(torch_cuda, engine, family, layout)


def _test_generated_vs_oracle_body(torch_cuda, engine, family, layout):
    kw = dict(align=8)
    if layout == "packed1":
        kw = dict(align=1)
    elif layout == "umem_mirror":
        # xudp TX frame layout: 4096-byte chunks, eth at F+342 (v4) / F+322 (v6)
        kw = dict(stride=4096, offset=342 if family == 4 else 322)
    umem, desc = X.gen_frames_host(3000, family, 0, 3000, seed=11 + family, **kw)
    mode = X.MODE_V6 if family == 6 else X.MODE_V4_LEGACY
    for hint in (0, 100, 1500):
        got, _ = run_device(torch_cuda, engine, umem, desc, mode, len_hint=hint)
        assert np.array_equal(got, oracle.batch(umem, desc, mode))


def test_device_generator_matches_host(torch_cuda, engine):
    for family in (4, 6):
        for kw in (dict(align=8), dict(align=1), dict(stride=4096, offset=342)):
            umem, desc = X.gen_frames_host(500, family, 0, 2000, seed=5, first_index=77, **kw)
            dev = torch_cuda.device("cuda:0")
            d_umem = torch_cuda.zeros(len(umem), dtype=torch_cuda.uint8, device=dev)
            d_desc = h2d(torch_cuda, desc.view(np.uint8), dev)
            engine.gen_fill_device(d_umem, d_desc, len(desc), family, 5, 77)
            torch_cuda.cuda.synchronize()
            assert np.array_equal(d2h(d_umem), umem)


@pytest.mark.parametrize("geom", FEATURE_GEOMS)
def test_edge_cases(torch_cuda, engine, geom):
    with geometry(engine, geom):
        _test_edge_cases_body(torch_cuda, engine)


def _test_edge_cases_body(torch_cuda, engine):
    # empty batch
    dev = torch_cuda.device("cuda:0")
    d = torch_cuda.zeros(16, dtype=torch_cuda.uint8, device=dev)
    engine.batch_device(d, d, 0, d, X.MODE_V4_LEGACY)
    # malformed frames: too short, jumbo > 65535 UDP bytes, unknown h_proto
    umem, desc = X.gen_frames_host(8, 4, 10, 10, seed=3)
    desc = desc.copy()
    desc["len"][1] = 41          # < eth+ip+udp
    desc["len"][2] = 34 + 65536  # udp_len > 65535
    umem = np.concatenate([umem, np.zeros(70000, dtype=np.uint8)])
    umem[int(desc["addr"][3]) + 12] = 0x12  # h_proto garbage (AUTO only)
    engine.take_errors()
    got, _ = run_device(torch_cuda, engine, umem, desc, X.MODE_AUTO)
    exp = oracle.batch(umem, desc, X.MODE_AUTO)
    assert got[1] == 0 and got[2] == 0 and got[3] == 0
    assert np.array_equal(got, exp)
    assert engine.take_errors() == 3
    # maximum UDP length: 65535
    umem, desc = X.gen_frames_host(3, 4, 65535 - 8, 65535 - 8, seed=4)
    for hint in (0, 100):
        got, _ = run_device(torch_cuda, engine, umem, desc, X.MODE_V4_LEGACY, len_hint=hint)
        assert np.array_equal(got, oracle.batch(umem, desc, X.MODE_V4_LEGACY))
    umem, desc = X.gen_frames_host(3, 6, 65535 - 8, 65535 - 8, seed=4)
    got, _ = run_device(torch_cuda, engine, umem, desc, X.MODE_V6)
    assert np.array_equal(got, oracle.batch(umem, desc, X.MODE_V6))
    # saturating: all-0xff frames of every small length
    umem, desc = X.gen_frames_host(400, 4, 0, 399, seed=9, align=1)
    for d in desc:
        a = int(d["addr"])
        umem[a + 26:a + int(d["len"])] = 0xff
    got, _ = run_device(torch_cuda, engine, umem, desc, X.MODE_V4_LEGACY, len_hint=100)
    assert np.array_equal(got, oracle.batch(umem, desc, X.MODE_V4_LEGACY))


def test_bad_arguments(engine):
    with pytest.raises(X.XcsumError):
        engine.batch_device(None, None, 5, None, X.MODE_V4_LEGACY)
    with pytest.raises(X.XcsumError):
        engine.batch_device(1, 1, 5, 1, 7)
    with pytest.raises(X.XcsumError):
        engine.set_geometry(7, 1, 1)


# ---- receive-side verify --------------------------------------------------

from test_oracle import filled_golden  # noqa: E402


@pytest.mark.parametrize("len_hint", [0, 100, 1500])
@pytest.mark.parametrize("geom", FEATURE_GEOMS)
def test_verify_matches_oracle(torch_cuda, engine, golden, len_hint, geom):
    with geometry(engine, geom):
        _test_verify_matches_oracle_body(torch_cuda, engine, golden, len_hint)


def _test_verify_matches_oracle_body(torch_cuda, engine, golden, len_hint):
    desc = golden_desc(golden)
    fam = golden["family"]
    good = filled_golden(golden)
    legacy = filled_golden(golden, "exp_legacy")
    rng = np.random.default_rng(2)
    bad = good.copy()
    for i, d in enumerate(desc):
        a, ln = int(d["addr"]), int(d["len"])
        bad[int(rng.integers(a + 22, a + ln))] ^= 0x10
    zero = good.copy()
    for i, d in enumerate(desc):
        a = int(d["addr"])
        zero[a + (60 if fam[i] == 6 else 40):a + (62 if fam[i] == 6 else 42)] = 0
    for umem in (good, legacy, bad, zero):
        for flags in (X.F_VERIFY, X.F_VERIFY | X.F_IPHDR, X.F_VERIFY | X.F_INPLACE):
            got, after = run_device(torch_cuda, engine, umem, desc, X.MODE_AUTO, flags,
                                    len_hint)
            exp = oracle.batch(umem, desc, X.MODE_AUTO, flags & ~X.F_INPLACE)
            assert np.array_equal(got, exp)
            assert np.array_equal(after, umem)   # verify never writes
    assert (run_device(torch_cuda, engine, good, desc, X.MODE_AUTO, X.F_VERIFY | X.F_IPHDR)[0]
            == 0).all()


def test_verify_host_path(engine, golden):
    desc = golden_desc(golden)
    good = filled_golden(golden)
    out = np.full(len(desc), 7, dtype=np.uint16)
    engine.batch_host(good, desc, out, X.MODE_AUTO, X.F_VERIFY | X.F_IPHDR)
    assert (out == 0).all()
    bad = good.copy()
    bad[int(desc["addr"][0]) + 28] ^= 0xff  # saddr byte: inside the span
    engine.batch_host(bad, desc, out, X.MODE_AUTO, X.F_VERIFY)
    assert out[0] != 0 and (out[1:] == 0).all()


# ---- visiting order (xcsum_ctx_set_order): results never depend on it ----

@pytest.mark.parametrize("order", [(0, 0), (1, 0), (2, 3), (4, 0), (3, 5), (6, 2), (12, 16)])
def test_visiting_order_same_result(torch_cuda, engine, golden, order):
    desc = golden_desc(golden)
    engine.set_order(*order)
    try:
        got, after = run_device(torch_cuda, engine, golden["umem"].copy(), desc, X.MODE_AUTO,
                                X.F_INPLACE | X.F_IPHDR)
        for family in (4, 6):
            # ragged: 2999 frames is no multiple of any tile or region count
            umem, gd = X.gen_frames_host(2999, family, 0, 1500, seed=21 + family)
            mode = X.MODE_V6 if family == 6 else X.MODE_V4_LEGACY
            for hint in (0, 100, 1500):
                g2, _ = run_device(torch_cuda, engine, umem, gd, mode, len_hint=hint)
                assert np.array_equal(g2, oracle.batch(umem, gd, mode)), (family, hint)
    finally:
        engine.set_order(-1, 0)
    exp, exp_after = run_device(torch_cuda, engine, golden["umem"].copy(), desc, X.MODE_AUTO,
                                X.F_INPLACE | X.F_IPHDR)
    assert np.array_equal(got, exp)
    assert np.array_equal(after, exp_after)


def test_visiting_order_bad_arguments(engine):
    for bad in ((-2, 0), (13, 0), (2, -1), (2, 17)):
        with pytest.raises(X.XcsumError):
            engine.set_order(*bad)


def test_launch_ignores_stale_hip_error(torch_cuda, engine, golden):
    """A pending event query elsewhere in the thread (hipEventQuery ->
    hipErrorNotReady, which HIP keeps as the thread's last error) must not
    make the next launch report failure."""
    torch = torch_cuda
    x = torch.ones(1 << 27, device="cuda:0")
    for _ in range(4):
        x = x * 1.0001
    ev = torch.cuda.Event()
    ev.record()
    ev.query()   # usually not ready yet
    desc = golden_desc(golden, np.nonzero(golden["family"] == 4)[0][:64])
    got, _ = run_device(torch, engine, golden["umem"].copy(), desc, X.MODE_V4_LEGACY)
    assert np.array_equal(got, golden["exp_legacy"][np.nonzero(golden["family"] == 4)[0][:64]])
    torch.cuda.synchronize()


# ---- VERIFY on received frames: the span ends at udp + ntohs(udp->len) ----

import rx_frames  # noqa: E402  (tests/golden, put on sys.path by conftest)


def received_batch(seed=11):
    """The receive corpus (Ethernet padding with zeros or junk, udp->len that
    does not fit, corrupted bytes, IPv4 options, extension headers, junk)
    plus padded frames of every size class up to jumbo: frames whose
    descriptor length exceeds the UDP datagram."""
    rng = np.random.default_rng(seed)
    frames = [f for f, _ in rx_frames.corpus(seed)]
    for plen in (0, 3, 17, 40, 100, 700, 1472, 3000, 8990):
        for pad in (1, 2, 15, 16, 33, 200):
            frames.append(rx_frames.v4_frame(rng, plen) + rx_frames.rand_bytes(rng, pad))
            frames.append(rx_frames.v6_frame(rng, plen) + rx_frames.rand_bytes(rng, pad))
    umem, addr, ln = rx_frames.layout(frames, rng)
    desc = np.zeros(len(frames), dtype=X.DESC_DTYPE)
    desc["addr"] = addr
    desc["len"] = ln
    return umem, desc


@pytest.mark.parametrize("geom", FEATURE_GEOMS + [(16, 2, 6), (4, 1, 2), (64, 1, 9)])
def test_verify_received_frames(torch_cuda, engine, geom):
    umem, desc = received_batch()
    with geometry(engine, geom):
        for hint in (0, 100, 1500):
            for mode in (X.MODE_AUTO, X.MODE_V4_RFC, X.MODE_V6):
                for flags in (X.F_VERIFY, X.F_VERIFY | X.F_IPHDR):
                    got, after = run_device(torch_cuda, engine, umem, desc, mode, flags, hint)
                    assert np.array_equal(got, oracle.batch(umem, desc, mode, flags)), \
                        (hint, mode, flags)
                    assert np.array_equal(after, umem)


def test_verify_padded_frames_pass(torch_cuda, engine):
    """Valid datagrams in padded frames verify (0); before the fix the pad
    bytes were summed and the frame length used as the UDP length."""
    rng = np.random.default_rng(5)
    frames = []
    for plen in (0, 1, 5, 10, 17):
        frames.append(rx_frames.pad60(rx_frames.v4_frame(rng, plen)))
        frames.append(rx_frames.pad60(rx_frames.v4_frame(rng, plen), rx_frames.rand_bytes(rng, 60)))
    for plen in (64, 1472, 8000):
        frames.append(rx_frames.v4_frame(rng, plen) + b"\xff" * 7)
        frames.append(rx_frames.v6_frame(rng, plen) + b"\x5a" * 24)
    umem, addr, ln = rx_frames.layout(frames, rng)
    desc = np.zeros(len(frames), dtype=X.DESC_DTYPE)
    desc["addr"] = addr
    desc["len"] = ln
    engine.take_errors()   # clear what earlier tests left
    got, _ = run_device(torch_cuda, engine, umem, desc, X.MODE_AUTO, X.F_VERIFY | X.F_IPHDR)
    assert (got == 0).all()
    out = np.full(len(desc), 7, dtype=np.uint16)
    engine.batch_host(umem, desc, out, X.MODE_AUTO, X.F_VERIFY | X.F_IPHDR)
    assert (out == 0).all()
    assert engine.take_errors() == 0


@pytest.mark.parametrize("base_off", [1, 3, 8, 13])
@pytest.mark.parametrize("geom", [None, (4, 1, 2), (16, 2, 6)] + X.STREAM_GEOMETRIES)
def test_unaligned_umem_base(torch_cuda, engine, base_off, geom):
    """d_umem not 16-byte aligned (the ABI allows any base): descriptors are
    offsets from it.  The stream kernel aligns its regions as addresses, so
    no load reaches past the 16-byte block of a frame's last byte.  Small
    packed frames (the stream kernel's case) and MTU frames, every flag set,
    against the oracle; the frame bytes around the batch stay untouched."""
    dev = torch_cuda.device("cuda:0")
    for fam, pmin, pmax in ((4, 0, 80), (6, 0, 80), (4, 1400, 1472)):
        umem, desc = X.gen_frames_host(700, fam, pmin, pmax, seed=fam + pmax + base_off, align=2)
        mode = X.MODE_V6 if fam == 6 else X.MODE_V4_RFC
        for flags in (0, X.F_INPLACE | X.F_IPHDR, X.F_VERIFY):
            buf = np.zeros(len(umem) + 64, np.uint8)
            buf[base_off:base_off + len(umem)] = umem
            d_buf = h2d(torch_cuda, buf, dev)
            d_desc = h2d(torch_cuda, desc.view(np.uint8), dev)
            d_out = torch_cuda.zeros(len(desc), dtype=torch_cuda.int16, device=dev)
            with geometry(engine, geom):
                engine.batch_device(d_buf.data_ptr() + base_off, d_desc, len(desc), d_out, mode,
                                    flags, stream=torch_cuda.cuda.current_stream(dev).cuda_stream)
                torch_cuda.cuda.synchronize(dev)
            got = d2h(d_out).view(np.uint16)
            exp = oracle.batch(umem, desc, mode, flags & ~X.F_INPLACE)
            assert np.array_equal(got, exp), (fam, flags, int((got != exp).sum()))
            after = d2h(d_buf)
            assert not after[:base_off].any() and not after[base_off + len(umem):].any()
