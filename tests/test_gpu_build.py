"""GPU: xcsum_build_device against the reference-built frames and the oracle."""
import numpy as np
import pytest

import libxudp_amd as X
from conftest import h2d, d2h
import oracle
from test_build import ROUTES, bfix, split  # noqa: F401

pytestmark = pytest.mark.gpu

FRAME, DATA_OFF = 16384, 384   # slots big enough for 8999-byte payloads


def route_of(fam, r):
    return X.make_route(fam, r["smac"], r["dmac"], r["saddr"], r["sport"], r["daddr"],
                        r["dport"])


def device_build(torch, engine, route, pays, inplace=False, flags=0, len_hint=0,
                 src_phase=None, slots=None, umem_fill=0x5a, FRAME=FRAME):
    dev = torch.device("cuda:0")
    n = len(pays)
    slots = np.arange(n, dtype=np.uint32) if slots is None else slots
    nslots = int(slots.max()) + 1
    umem = np.full(nslots * FRAME, umem_fill, dtype=np.uint8)
    msgs = np.zeros(n, dtype=X.MSG_DTYPE)
    rng = np.random.default_rng(1)
    if inplace:
        for i, p in enumerate(pays):
            o = int(slots[i]) * FRAME + DATA_OFF
            umem[o:o + len(p)] = p
        src = np.zeros(16, np.uint8)
    else:
        off, chunks = 0, []
        for p in pays:
            ph = int(rng.integers(0, 16)) if src_phase is None else src_phase
            off += ph
            chunks.append((off, p))
            off += len(p)
        src = np.full(off + 16, 0xee, dtype=np.uint8)
        for i, (o, p) in enumerate(chunks):
            src[o:o + len(p)] = p
            msgs["src"][i] = o
        # exact-size device buffer: the last payload ends at the allocation's end
        src = src[:off] if off else src
    msgs["len"] = [len(p) for p in pays]
    msgs["slot"] = slots
    d_umem = h2d(torch, umem, dev)
    d_src = h2d(torch, np.ascontiguousarray(src), dev)
    d_msgs = h2d(torch, msgs.view(np.uint8), dev)
    d_desc = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_out = torch.zeros(n, dtype=torch.int16, device=dev)
    engine.build_device(route, d_src, d_msgs, n, d_umem, FRAME, DATA_OFF, d_desc, d_out,
                        flags | (X.F_BUILD_INPLACE if inplace else 0), len_hint)
    torch.cuda.synchronize()
    return (d2h(d_umem), d2h(d_desc).view(X.DESC_DTYPE),
            d2h(d_out).view(np.uint16), umem)


@pytest.mark.parametrize("fam", [4, 6])
@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("len_hint", [0, 60, 200, 1500, 9000])
def test_build_matches_reference(torch_cuda, engine, bfix, fam, inplace, len_hint):
    hdr = 42 if fam == 4 else 62
    lens = bfix[f"v{fam}_lens"]
    pays = split(bfix[f"v{fam}_payloads"], lens)
    frames = split(bfix[f"v{fam}_frames"], lens + hdr)
    after, desc, out, before = device_build(torch_cuda, engine, route_of(fam, ROUTES[fam]),
                                            pays, inplace=inplace, len_hint=len_hint)
    touched = np.zeros(after.size, dtype=bool)
    for i, f in enumerate(frames):
        eth = i * FRAME + DATA_OFF - hdr
        assert desc["addr"][i] == eth and desc["len"][i] == len(f)
        assert np.array_equal(after[eth:eth + len(f)], f), i
        ck = f[60:62] if fam == 6 else f[40:42]
        assert out[i] == int(ck.view("<u2")[0])
        touched[eth:eth + len(f)] = True
    assert np.array_equal(after[~touched], before[~touched])   # nothing else written


@pytest.mark.parametrize("phase", [0, 1, 2, 3, 5, 8, 13, 15])
def test_build_every_source_alignment(torch_cuda, engine, bfix, phase):
    lens = bfix["v6_lens"]
    pays = split(bfix["v6_payloads"], lens)
    frames = split(bfix["v6_frames"], lens + 62)
    after, desc, out, _ = device_build(torch_cuda, engine, route_of(6, ROUTES[6]), pays,
                                       src_phase=phase, len_hint=1500)
    for i, f in enumerate(frames):
        eth = i * FRAME + DATA_OFF - 62
        assert np.array_equal(after[eth:eth + len(f)], f)


def test_build_random_routes_vs_oracle(torch_cuda, engine):
    rng = np.random.default_rng(9)
    for fam in (4, 6):
        for v4_rfc in (False, True):
            al = 16 if fam == 6 else 4
            r = dict(smac=rng.integers(0, 256, 6, dtype=np.uint8).tobytes(),
                     dmac=rng.integers(0, 256, 6, dtype=np.uint8).tobytes(),
                     saddr=rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                     daddr=rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                     sport=int(rng.integers(0, 65536)), dport=int(rng.integers(0, 65536)))
            pays = [rng.integers(0, 256, int(L), dtype=np.uint8)
                    for L in rng.integers(0, 3000, 400)]
            slots = rng.permutation(600)[:400].astype(np.uint32)     # scattered slots
            after, desc, out, _ = device_build(
                torch_cuda, engine, route_of(fam, r), pays, flags=X.F_V4_RFC if v4_rfc else 0,
                slots=slots)
            hdr = 42 if fam == 4 else 62
            for i, p in enumerate(pays):
                exp = oracle.build_frame(p.tobytes(), fam, r["smac"], r["dmac"], r["saddr"],
                                         r["sport"], r["daddr"], r["dport"], v4_rfc)
                eth = int(slots[i]) * FRAME + DATA_OFF - hdr
                assert np.array_equal(after[eth:eth + len(exp)], exp)


@pytest.mark.parametrize("slot_size", [4096, FRAME])
def test_build_ipv4_inplace_header_kernel(torch_cuda, engine, monkeypatch, slot_size):
    """IPv4 in place without V4_RFC -- libxudp's default send on frames whose
    payload already sits in its slot -- takes the header-only build kernel
    (no payload byte read: iph->check only, udp->check 0, packet.c:43-66,
    :125).  Its slots, descriptors and results equal the payload-summing
    kernel's (XCSUM_TUNE_BUILD_HDR 0) and the oracle's frames, for ragged
    payloads in scattered slots."""
    rng = np.random.default_rng(23)
    n = 3001
    cap = slot_size - DATA_OFF
    pays = [rng.integers(0, 256, int(L), dtype=np.uint8)
            for L in rng.integers(0, min(cap, 1500) + 1, n)]
    slots = rng.permutation(n + 500)[:n].astype(np.uint32)
    r = ROUTES[4]
    res = {}
    try:
        for hdr_kernel in ("1", "0"):
            engine.set_tuning(X.TUNE_BUILD_HDR, int(hdr_kernel))
            engine.take_errors()
            res[hdr_kernel] = device_build(torch_cuda, engine, route_of(4, r), pays,
                                           inplace=True, slots=slots, len_hint=700,
                                           FRAME=slot_size)[:3]
            assert engine.take_errors() == 0
    finally:
        engine.set_tuning(X.TUNE_BUILD_HDR, 1)
    for a, b in zip(res["1"], res["0"]):
        assert np.array_equal(a, b)
    after, desc, out = res["1"]
    assert not out.any()                                        # udp->check 0
    for i in rng.choice(n, 60, replace=False):
        exp = oracle.build_frame(pays[i].tobytes(), 4, r["smac"], r["dmac"], r["saddr"],
                                 r["sport"], r["daddr"], r["dport"], False)
        eth = int(slots[i]) * slot_size + DATA_OFF - 42
        assert np.array_equal(after[eth:eth + len(exp)], exp), i


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 257, 1025, 70001, 300001])
def test_build_ipv4_header_kernel_batch_edges(torch_cuda, engine, monkeypatch, n):
    """The header-only build kernel's persistent grid (4 lanes per message,
    the next message prefetched) at batch tails, and at 300,001 messages
    more than two rounds of a full grid (256 CUs x 8 blocks x 64 messages):
    slots, descriptors and results equal the payload-summing kernel's
    (XCSUM_TUNE_BUILD_HDR 0), in xudp's 4096-byte slots."""
    rng = np.random.default_rng(n)
    pays = [rng.integers(0, 256, int(L), dtype=np.uint8)
            for L in rng.integers(0, 1473, n)]
    res = {}
    try:
        for hdr_kernel in ("1", "0"):
            engine.set_tuning(X.TUNE_BUILD_HDR, int(hdr_kernel))
            res[hdr_kernel] = device_build(torch_cuda, engine, route_of(4, ROUTES[4]), pays,
                                           inplace=True, len_hint=700, FRAME=4096)[:3]
    finally:
        engine.set_tuning(X.TUNE_BUILD_HDR, 1)
    for a, b in zip(res["1"], res["0"]):
        assert np.array_equal(a, b)
    assert np.array_equal(res["1"][1]["len"], np.array([len(p) + 42 for p in pays]))


@pytest.mark.parametrize("inplace", [False, True])   # True: the header-only kernel
def test_build_rejects_oversized(torch_cuda, engine, inplace):
    pays = [np.zeros(100, np.uint8), np.zeros(FRAME - DATA_OFF + 1, np.uint8),
            np.zeros(70000, np.uint8), np.ones(10, np.uint8)]
    engine.take_errors()
    after, desc, out, before = device_build(torch_cuda, engine, route_of(4, ROUTES[4]), pays[:2]
                                            + pays[3:], inplace=inplace)
    assert list(desc["len"]) == [142, 0, 52]
    assert engine.take_errors() == 1


@pytest.mark.parametrize("inplace", [False, True])
def test_build_visiting_order(torch_cuda, engine, inplace):
    """xudp's 4096-byte chunks make the batch sparse: the automatic order
    visits messages region by region.  Frames, descriptors and results must
    be identical to descriptor order, and to the oracle."""
    rng = np.random.default_rng(17)
    pays = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 1500, 3001)]
    r = ROUTES[4]
    res = {}
    for order in ((0, 0), (-1, 0), (5, 4), (3, 2), (7, 0)):
        engine.set_order(*order)
        try:
            res[order] = device_build(torch_cuda, engine, route_of(4, r), pays, inplace=inplace,
                                      len_hint=1472, FRAME=4096)[:3]
        finally:
            engine.set_order(-1, 0)
    base = res[(0, 0)]
    for order, got in res.items():
        for a, b in zip(got, base):
            assert np.array_equal(a, b), order
    after = base[0]
    for i in rng.choice(len(pays), 40, replace=False):
        exp = oracle.build_frame(pays[i].tobytes(), 4, r["smac"], r["dmac"], r["saddr"],
                                 r["sport"], r["daddr"], r["dport"], False)
        eth = int(i) * 4096 + DATA_OFF - 42
        assert np.array_equal(after[eth:eth + len(exp)], exp), i


from test_build import BUILD_GEOMETRIES  # noqa: E402


@pytest.mark.parametrize("geom", BUILD_GEOMETRIES)
def test_build_stage_edges_every_geometry(torch_cuda, engine, geom, monkeypatch):
    """Payloads around one pass's capacity (16*K*G bytes) from every source
    phase: the unaligned path reads the extra block K*G from its LDS stage
    exactly when len + phase > 16*K*G, and longer payloads take the walk."""
    G, K = geom
    cap = 16 * K * G
    monkeypatch.setenv("XCSUM_BUILD_GEOMETRY", f"{G},{K}")
    rng = np.random.default_rng(G * 100 + K)
    lens = sorted({L for L in (1, 15, 16, 17, cap - 17, cap - 16, cap - 15, cap - 1, cap,
                               cap + 1, cap + 15) if 0 < L <= FRAME - DATA_OFF})
    r = ROUTES[4]
    for phase in (0, 1, 3, 4, 7, 12, 15):
        pays = [rng.integers(0, 256, L, dtype=np.uint8) for L in lens]
        after, desc, out, _ = device_build(torch_cuda, engine, route_of(4, r), pays,
                                           src_phase=phase, flags=X.F_V4_RFC)
        for i, p in enumerate(pays):
            exp = oracle.build_frame(p.tobytes(), 4, r["smac"], r["dmac"], r["saddr"],
                                     r["sport"], r["daddr"], r["dport"], True)
            eth = i * FRAME + DATA_OFF - 42
            assert np.array_equal(after[eth:eth + len(exp)], exp), (geom, phase, len(p))
