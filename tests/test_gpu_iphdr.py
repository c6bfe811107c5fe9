"""GPU: XCSUM_F_IPHDR_ONLY -- libxudp's IPv4 TX checksum call on the device.

For IPv4, xudp_packet_udp() computes only iph->check (xudp_checksum_half,
xudp/packet.c:43-66) and leaves udp->check 0 (packet.c:125); the batch call
with XCSUM_F_IPHDR_ONLY does exactly that and reads no payload byte
(csrc/xcsum_iphdr.hip).  Expected values: the reference's own frames and
header checksums (tests/golden: build_fixtures.npz, fixtures.npz exp_iphdr)
and the oracle restatement (orc_ip_checksum_half / orc_ip_header_rfc, pinned
to the reference by tests/test_oracle.py).  Integer work: bit-exact.
"""
import numpy as np
import pytest

import libxudp_amd as X
import oracle
from conftest import golden_desc, h2d, d2h
from test_build import bfix, split  # noqa: F401

pytestmark = pytest.mark.gpu

FPTS = ["1", "2", "4", "8"]


def run(torch, eng, umem, desc, mode=X.MODE_V4_LEGACY, flags=0, out=True):
    dev = torch.device("cuda:0")
    d_umem = h2d(torch, umem, dev)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    d_out = torch.full((max(len(desc), 1),), 0x5a5a, dtype=torch.int32,
                       device=dev).to(torch.int16) if out else None
    s = torch.cuda.current_stream(dev).cuda_stream
    eng.batch_device(d_umem, d_desc, len(desc), d_out, mode, X.F_IPHDR_ONLY | flags, 0,
                     stream=s)
    torch.cuda.synchronize(dev)
    return (d2h(d_out[:len(desc)]).view(np.uint16) if out else None), d2h(d_umem)


def hdr_np(umem, addr, verify=False):
    """RFC 1071 over the 20 header bytes at eth+14 (check as 0 unless
    verify), memory-order u16 -- vectorised; tests pin it to the oracle."""
    a = addr.astype(np.int64)[:, None] + 14 + np.arange(20)[None, :]
    b = umem[a].astype(np.uint32)
    words = (b[:, 0::2] << 8) | b[:, 1::2]
    if not verify:
        words[:, 5] = 0
    s = words.sum(axis=1)
    s = (s & 0xffff) + (s >> 16)
    s = (s & 0xffff) + (s >> 16)
    r = ~s & 0xffff
    return (((r & 0xff) << 8) | (r >> 8)).astype(np.uint16)


def random_frames(rng, n, lmin=42, lmax=1600, align=1, random_header=True):
    """n frames of random bytes (IPv4 h_proto) at random byte phases."""
    lens = rng.integers(lmin, lmax + 1, n)
    addr = np.zeros(n, np.uint64)
    off = int(rng.integers(0, 64))
    for i in range(n):
        off += int(rng.integers(0, 16)) * align if align > 1 else int(rng.integers(0, 9))
        addr[i] = off
        off += int(lens[i])
    umem = rng.integers(0, 256, off + 64, dtype=np.uint8)
    if not random_header:
        umem[:] = 0
    for a in addr:
        umem[int(a) + 12:int(a) + 14] = (0x08, 0x00)
        umem[int(a) + 24:int(a) + 26] = 0        # the check, as iph_build leaves it
    d = np.zeros(n, X.DESC_DTYPE)
    d["addr"], d["len"] = addr, lens
    return umem, d


@pytest.mark.parametrize("fpt", FPTS)
def test_golden_exp_iphdr(torch_cuda, engine, golden, monkeypatch, fpt):
    """fixtures.npz: every IPv4 frame's iph->check == the reference's
    xudp_checksum_half (exp_iphdr); AUTO leaves IPv6 frames at 0."""
    monkeypatch.setenv("XCSUM_IPHDR_FPT", fpt)
    fam = golden["family"]
    v4 = np.nonzero(fam == 4)[0]
    got, after = run(torch_cuda, engine, golden["umem"], golden_desc(golden, v4))
    assert np.array_equal(got, golden["exp_iphdr"][v4])
    assert np.array_equal(after, golden["umem"])          # no INPLACE: nothing written
    engine.take_errors()
    got, _ = run(torch_cuda, engine, golden["umem"], golden_desc(golden), X.MODE_AUTO)
    assert np.array_equal(got, np.where(fam == 6, 0, golden["exp_iphdr"]))
    assert engine.take_errors() == 0                      # IPv6 is not malformed


def test_golden_inplace_touches_only_iph_check(torch_cuda, engine, golden):
    fam = golden["family"]
    desc = golden_desc(golden)
    umem = golden["umem"].copy()
    for d in desc[fam == 4]:
        umem[int(d["addr"]) + 24:int(d["addr"]) + 26] = 0
    for out in (True, False):
        got, after = run(torch_cuda, engine, umem, desc, X.MODE_AUTO, X.F_INPLACE, out=out)
        exp = umem.copy()
        for i, d in enumerate(desc):
            if fam[i] == 4:
                a = int(d["addr"])
                exp[a + 24:a + 26] = np.array([golden["exp_iphdr"][i]], "<u2").view(np.uint8)
        assert np.array_equal(after, exp)                 # udp->check untouched
        if out:
            assert np.array_equal(got, np.where(fam == 6, 0, golden["exp_iphdr"]))


@pytest.mark.parametrize("layout", ["packed", "slots"])
@pytest.mark.parametrize("fpt", ["1", "4", "8"])
def test_reference_built_frames(torch_cuda, engine, bfix, monkeypatch, layout, fpt):
    """The reference's own xudp_packet_udp_payload() frames (build_fixtures,
    139 IPv4 frames, payload 0..8999): with iph->check cleared and the call
    run in place, every byte equals the reference frame -- iph->check from
    xudp_checksum_half, udp->check 0 -- packed at random phases and in
    xudp's 4096-byte slots (eth at F+342)."""
    monkeypatch.setenv("XCSUM_IPHDR_FPT", fpt)
    lens = bfix["v4_lens"] + 42
    frames = split(bfix["v4_frames"], lens)
    rng = np.random.default_rng(5)
    n = len(frames)
    desc = np.zeros(n, X.DESC_DTYPE)
    if layout == "slots":
        stride = 16384                       # payloads up to 8999 bytes
        addr = np.arange(n, dtype=np.uint64) * stride + 342
    else:
        addr = np.cumsum([0] + [int(L) + int(rng.integers(0, 16)) for L in lens[:-1]]).astype(
            np.uint64) + 3
    desc["addr"], desc["len"] = addr, lens
    ref = rng.integers(0, 256, int(addr[-1]) + int(lens[-1]) + 64, dtype=np.uint8)
    for a, f in zip(addr, frames):
        ref[int(a):int(a) + len(f)] = f
        assert f[40] == 0 and f[41] == 0                  # udp->check 0 (packet.c:125)
    start = ref.copy()
    for a in addr:
        start[int(a) + 24:int(a) + 26] = 0
    got, after = run(torch_cuda, engine, start, desc, flags=X.F_INPLACE)
    assert np.array_equal(after, ref)
    exp = np.array([int(f[24:26].view("<u2")[0]) for f in frames], np.uint16)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("seed", range(6))
def test_random_headers_vs_oracle(torch_cuda, engine, seed):
    """Random header bytes (tos, id, ttl, ... not xudp's constants) at every
    byte phase: RFC 1071 over the header as orc_ip_header_rfc computes it;
    xudp-built frames (the generator): orc_ip_checksum_half, the
    restatement of packet.c:43-66."""
    rng = np.random.default_rng(seed)
    umem, desc = random_frames(rng, 3000)
    got, after = run(torch_cuda, engine, umem, desc, flags=X.F_INPLACE)
    exp = hdr_np(umem, desc["addr"])
    assert np.array_equal(got, exp)
    for i in rng.choice(len(desc), 64, replace=False):
        a = int(desc["addr"][i])
        assert exp[i] == oracle.ip_header_rfc(umem[a:a + 42])
    changed = np.nonzero(after != umem)[0]
    fields = set()
    for a in desc["addr"]:
        fields.update((int(a) + 24, int(a) + 25))
    assert set(changed.tolist()) <= fields
    # xudp's own frames
    gumem, gdesc = X.gen_frames_host(2000, 4, 0, 1500, seed=seed)
    got, _ = run(torch_cuda, engine, gumem, gdesc)
    P = oracle.port()
    for i in range(0, 2000, 7):
        a = int(gdesc["addr"][i])
        ip = np.ascontiguousarray(gumem[a + 14:a + 34])
        assert got[i] == P.orc_ip_checksum_half(ip.ctypes.data)
    assert np.array_equal(got, hdr_np(gumem, gdesc["addr"]))


def test_verify(torch_cuda, engine):
    rng = np.random.default_rng(11)
    umem, desc = random_frames(rng, 1000)
    good = umem.copy()
    chk = hdr_np(umem, desc["addr"])
    for a, c in zip(desc["addr"], chk):
        good[int(a) + 24:int(a) + 26] = np.array([c], "<u2").view(np.uint8)
    bad = good.copy()
    flip = rng.choice(len(desc), 300, replace=False)
    for i in flip:
        a = int(desc["addr"][i]) + 14 + int(rng.integers(0, 20))
        bad[a] ^= 1 << int(rng.integers(0, 8))
    for flags in (X.F_VERIFY, X.F_VERIFY | X.F_INPLACE):   # verifying never writes
        got, after = run(torch_cuda, engine, good, desc, flags=flags)
        assert not got.any() and np.array_equal(after, good)
        got, after = run(torch_cuda, engine, bad, desc, flags=flags)
        assert np.array_equal(got, hdr_np(bad, desc["addr"], verify=True))
        assert np.count_nonzero(got) == len(flip) and np.array_equal(after, bad)


def test_malformed_and_auto(torch_cuda, engine):
    """Short frames, UDP length > 65535 and (AUTO) other protocols are
    malformed: out 0 (0xffff under VERIFY), counted, never written.  IPv6
    frames in AUTO are left alone with out 0 and are not errors."""
    rng = np.random.default_rng(3)
    umem = rng.integers(0, 256, 300000, dtype=np.uint8)
    cases = [  # (len, proto, malformed, v4)
        (0, 0x0800, True, False), (13, 0x0800, True, False), (41, 0x0800, True, False),
        (42, 0x0800, False, True), (65569, 0x0800, False, True), (65570, 0x0800, True, False),
        (100, 0x86DD, False, False), (61, 0x86DD, True, False), (100, 0x0806, True, False),
        (100, 0x0000, True, False)]
    desc = np.zeros(len(cases), X.DESC_DTYPE)
    addr = 5
    for i, (ln, proto, _, _) in enumerate(cases):
        desc["addr"][i], desc["len"][i] = addr, ln
        umem[addr + 12:addr + 14] = (proto >> 8, proto & 0xff)
        umem[addr + 24:addr + 26] = 0
        addr += max(ln, 64) + 3
    exp_v4 = hdr_np(umem, desc["addr"])
    mal = np.array([c[2] for c in cases])
    v4 = np.array([c[3] for c in cases])
    engine.take_errors()
    got, after = run(torch_cuda, engine, umem, desc, X.MODE_AUTO, X.F_INPLACE)
    assert np.array_equal(got, np.where(v4, exp_v4, 0))
    assert engine.take_errors() == int(mal.sum())
    for i in np.nonzero(~v4)[0]:
        a = int(desc["addr"][i])
        assert np.array_equal(after[a:a + 64], umem[a:a + 64])
    got, _ = run(torch_cuda, engine, umem, desc, X.MODE_AUTO, X.F_VERIFY)
    assert np.array_equal(got[mal], np.full(mal.sum(), 0xffff, np.uint16))
    # V4 modes do not read h_proto: only the length rule
    engine.take_errors()
    got, _ = run(torch_cuda, engine, umem, desc, X.MODE_V4_RFC)
    lenok = np.array([c[0] >= 42 and c[0] - 34 <= 65535 for c in cases])
    assert np.array_equal(got, np.where(lenok, exp_v4, 0))
    assert engine.take_errors() == int((~lenok).sum())


@pytest.mark.parametrize("n", [1, 2, 255, 256, 257, 1023, 1025, 4097])
def test_batch_edges_and_orders(torch_cuda, engine, n):
    """Grid tails at every frames-per-thread, and forced visiting orders on a
    sparse (xudp slots) layout: identical results."""
    rng = np.random.default_rng(n)
    desc, nbytes = X.gen_layout(n, 4, 0, 1472, seed=n, stride=4096, offset=342)
    umem = np.zeros(nbytes + 64, np.uint8)
    X.gen_fill_host(umem, desc, 4, seed=n)
    exp = hdr_np(umem, desc["addr"])
    for order in ((-1, 0), (0, 0), (3, 4), (5, 4), (7, 0), (2, 1)):
        engine.set_order(*order)
        try:
            got, after = run(torch_cuda, engine, umem, desc, flags=X.F_INPLACE)
        finally:
            engine.set_order(-1, 0)
        assert np.array_equal(got, exp), order
        for i in rng.choice(n, min(n, 16), replace=False):
            a = int(desc["addr"][i])
            assert int(after[a + 24:a + 26].view("<u2")[0]) == exp[i]
            assert after[a + 40] == 0 and after[a + 41] == 0


def test_rejects(torch_cuda, engine):
    dev = torch_cuda.device("cuda:0")
    d = torch_cuda.zeros(64, dtype=torch_cuda.uint8, device=dev)
    o = torch_cuda.zeros(4, dtype=torch_cuda.int16, device=dev)
    with pytest.raises(X.XcsumError) as e:
        engine.batch_device(d, d, 1, o, X.MODE_V6, X.F_IPHDR_ONLY)
    assert e.value.rc == -X.ERR_INVAL
    umem, desc = X.gen_frames_host(4, 6, 10)
    out = np.zeros(4, np.uint16)
    with pytest.raises(X.XcsumError) as e:
        engine.batch_host(umem, desc, out, X.MODE_V6, X.F_IPHDR_ONLY)
    assert e.value.rc == -X.ERR_INVAL


def host_call(eng, umem, desc, mode, flags, buf=None):
    """xcsum_batch_host with XCSUM_F_IPHDR_ONLY on a copy of umem (or in
    buf, a registered UMEM): (out, frames after)"""
    if buf is None:
        buf = umem.copy()
    else:
        buf[:len(umem)] = umem
    out = np.full(len(desc), 0x5a5a, np.uint16)
    eng.batch_host(buf, desc, out, mode, X.F_IPHDR_ONLY | flags)
    return out, buf[:len(umem)].copy()


@pytest.mark.parametrize("n", [100, 20000, 70000])
@pytest.mark.parametrize("transport", ["pageable", "registered", "zerocopy", "resident"])
def test_host_batch_matches_device(torch_cuda, engine, transport, n):
    """libxudp's IPv4 call on host-resident frames (xcsum_batch_host,
    XCSUM_F_IPHDR_ONLY): the frames' first 42 bytes gathered into the pinned
    stage (pageable memory; 100 frames go by the direct path, 70000 span two
    chunks), or read in place over PCIe from a registered, GPU-mapped UMEM;
    a context with resident workgroups launches it.  Results and frames
    after the in-place call are identical to the device call's."""
    rng = np.random.default_rng(n)
    umem, desc = random_frames(rng, n, lmax=1000)
    got_d, after_d = run(torch_cuda, engine, umem, desc, flags=X.F_INPLACE)
    assert np.array_equal(got_d, hdr_np(umem, desc["addr"]))
    eng, buf, flags = engine, None, 0
    if transport == "resident":
        eng = X.Engine(0)
        eng.set_resident(8)
    if transport in ("registered", "zerocopy"):
        buf = X.umem_buffer(len(umem))
        engine.register_umem(buf)
        assert engine.umem_mapped(buf) == 1
        flags = X.F_ZEROCOPY if transport == "zerocopy" else 0
    try:
        for mode in (X.MODE_V4_LEGACY, X.MODE_AUTO):
            got, after = host_call(eng, umem, desc, mode, X.F_INPLACE | flags, buf)
            assert np.array_equal(got, got_d), mode
            assert np.array_equal(after, after_d), mode
        got, after = host_call(eng, umem, desc, X.MODE_V4_RFC, flags, buf)  # result only
        assert np.array_equal(got, got_d) and np.array_equal(after, umem)
        assert eng.take_errors() == 0
    finally:
        if buf is not None:
            engine.unregister_umem(buf)
        if eng is not engine:
            eng.close()


@pytest.mark.parametrize("register", [False, True])
def test_host_batch_slots(torch_cuda, engine, register):
    """xudp's own layout (one frame per 4096-byte chunk, eth at F+342, xudp's
    headers from the generator): the host call writes iph->check only, the
    value orc_ip_checksum_half (packet.c:43-66) gives."""
    n = 3000
    desc, nbytes = X.gen_layout(n, 4, 0, 1472, seed=9, stride=4096, offset=342)
    umem = np.zeros(nbytes + 64, np.uint8)
    X.gen_fill_host(umem, desc, 4, seed=9)
    for a in desc["addr"]:
        umem[int(a) + 24:int(a) + 26] = 0
    buf = None
    if register:
        buf = X.umem_buffer(len(umem))
        engine.register_umem(buf)
    try:
        got, after = host_call(engine, umem, desc, X.MODE_V4_LEGACY, X.F_INPLACE, buf)
    finally:
        if buf is not None:
            engine.unregister_umem(buf)
    P = oracle.port()
    for i in range(0, n, 11):
        a = int(desc["addr"][i])
        ip = np.ascontiguousarray(umem[a + 14:a + 34])
        assert got[i] == P.orc_ip_checksum_half(ip.ctypes.data)
    assert np.array_equal(got, hdr_np(umem, desc["addr"]))
    exp = umem.copy()
    for a, c in zip(desc["addr"], got):
        exp[int(a) + 24:int(a) + 26] = np.array([c], "<u2").view(np.uint8)
    assert np.array_equal(after, exp)


def test_host_batch_malformed_verify(torch_cuda, engine):
    """The host call's rules are the device call's: malformed frames (short,
    UDP length past 16 bits, another h_proto under AUTO) are counted and left
    alone, IPv6 frames under AUTO are left alone and not counted, and VERIFY
    (which never writes) flags exactly the corrupted headers."""
    rng = np.random.default_rng(8)
    umem = rng.integers(0, 256, 300000, dtype=np.uint8)
    lens = [0, 13, 41, 42, 65569, 65570, 100, 61, 100, 100, 1500]
    protos = [0x0800] * 6 + [0x86DD, 0x86DD, 0x0806, 0x0000, 0x0800]
    desc = np.zeros(len(lens), X.DESC_DTYPE)
    addr = 5
    for i, (ln, proto) in enumerate(zip(lens, protos)):
        desc["addr"][i], desc["len"][i] = addr, ln
        umem[addr + 12:addr + 14] = (proto >> 8, proto & 0xff)
        umem[addr + 24:addr + 26] = 0
        addr += max(ln, 64) + 3
    for mode in (X.MODE_AUTO, X.MODE_V4_LEGACY):
        for flags in (X.F_INPLACE, X.F_VERIFY, X.F_VERIFY | X.F_INPLACE):
            engine.take_errors()
            got_d, after_d = run(torch_cuda, engine, umem, desc, mode, flags)
            err_d = engine.take_errors()
            got, after = host_call(engine, umem, desc, mode, flags)
            assert np.array_equal(got, got_d), (mode, flags)
            assert np.array_equal(after, after_d), (mode, flags)
            assert engine.take_errors() == err_d > 0


@pytest.mark.slow
@pytest.mark.parametrize("layout", ["packed", "umem"])
def test_fullsize_vs_udp_kernel(torch_cuda, engine, layout):
    """BASELINE config 2 at full size (1M MTU frames, packed and in xudp's
    slots), generated on the device: the header-only call in place writes
    the same iph->check as the UDP kernel's XCSUM_F_INPLACE | XCSUM_F_IPHDR
    pass (itself pinned to the reference), leaves udp->check 0 and changes
    no other byte."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    n = 1 << 20
    if layout == "umem":
        desc, nbytes = X.gen_layout(n, 4, 1472, 1472, seed=2, stride=4096, offset=342)
    else:
        desc, nbytes = X.gen_layout(n, 4, 1472, 1472, seed=2)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    base = torch.zeros(nbytes + 64, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    engine.gen_fill_device(base, d_desc, n, 4, 2, 0, stream=s)
    a_buf, b_buf = base.clone(), base.clone()
    engine.batch_device(a_buf, d_desc, n, None, X.MODE_V4_LEGACY, X.F_INPLACE | X.F_IPHDR, 1514,
                        stream=s)
    out = torch.zeros(n, dtype=torch.int16, device=dev)
    engine.batch_device(b_buf, d_desc, n, out, X.MODE_V4_LEGACY, X.F_INPLACE | X.F_IPHDR_ONLY,
                        1514, stream=s)
    torch.cuda.synchronize(dev)
    addr = torch.from_numpy(desc["addr"].astype(np.int64)).to(dev)
    ip = torch.stack([addr + 24, addr + 25], 1).reshape(-1)
    ud = torch.stack([addr + 40, addr + 41], 1).reshape(-1)
    assert torch.equal(b_buf[ip], a_buf[ip])
    assert not bool(b_buf[ud].any())
    assert torch.equal(out.view(torch.uint8), b_buf[ip])
    b_buf[ip] = base[ip]
    assert torch.equal(b_buf, base)
