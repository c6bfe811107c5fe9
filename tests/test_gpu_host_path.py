"""GPU: host-resident batches (frames in a UMEM-like host buffer) and the
packet.c-level mirror, through the C ABI, against the reference fixtures and
the oracle."""
import os
import socket

import numpy as np
import pytest

import libxudp_amd as X
import oracle
from conftest import golden_desc
from test_gpu_parity import run_device
from test_oracle import KAT3, KAT4

pytestmark = pytest.mark.gpu


def host_batch(engine, umem, desc, mode, flags=0):
    out = np.full(len(desc), 0x5a5a, dtype=np.uint16)
    engine.batch_host(umem, desc, out, mode, flags)
    return out


@pytest.mark.parametrize("mode,col,fam", [(X.MODE_V4_LEGACY, "exp_legacy", 4),
                                          (X.MODE_V4_RFC, "exp_rfc", 4),
                                          (X.MODE_V6, "exp_v6", 6)])
def test_host_batch_golden(engine, golden, mode, col, fam):
    sel = np.nonzero(golden["family"] == fam)[0]
    got = host_batch(engine, golden["umem"], golden_desc(golden, sel), mode)
    assert np.array_equal(got, golden[col][sel])


def check_inplace(golden, after, desc):
    fam = golden["family"]
    for i, d in enumerate(desc):
        a = int(d["addr"])
        f = after[a:a + int(d["len"])]
        if fam[i] == 6:
            assert int(f[60:62].view("<u2")[0]) == golden["exp_v6"][i]
        else:
            assert int(f[40:42].view("<u2")[0]) == golden["exp_legacy"][i]
            assert int(f[24:26].view("<u2")[0]) == golden["exp_iphdr"][i]


@pytest.mark.parametrize("how", ["pageable", "registered", "zerocopy"])
def test_host_batch_inplace(engine, golden, how):
    umem = golden["umem"].copy()
    desc = golden_desc(golden)
    flags = X.F_INPLACE | X.F_IPHDR
    if how != "pageable":
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        engine.register_umem(umem)
    if how == "zerocopy":
        flags |= X.F_ZEROCOPY
    try:
        got = host_batch(engine, umem, desc, X.MODE_AUTO, flags)
    finally:
        if how != "pageable":
            engine.unregister_umem(umem)
    fam = golden["family"]
    assert np.array_equal(got, np.where(fam == 6, golden["exp_v6"], golden["exp_legacy"]))
    check_inplace(golden, umem, desc)


def test_zerocopy_needs_registration(engine, golden):
    with pytest.raises(X.XcsumError) as e:
        host_batch(engine, golden["umem"], golden_desc(golden), X.MODE_AUTO, X.F_ZEROCOPY)
    assert e.value.rc == -X.ERR_NOT_REGISTERED


@pytest.mark.parametrize("shuffle", [False, True])
def test_host_batch_many_chunks(engine, shuffle):
    """> 65536 frames and > 32 MiB of UMEM: several double-buffered chunks."""
    umem, desc = X.gen_frames_host(150000, 4, 0, 1472, seed=21, align=8)
    if shuffle:
        desc = desc[np.random.default_rng(0).permutation(len(desc))]
    exp = oracle.batch(umem, desc, X.MODE_V4_LEGACY)
    assert np.array_equal(host_batch(engine, umem, desc, X.MODE_V4_LEGACY), exp)
    umem = X.as_umem(umem)   # libxudp's UMEM mapping
    engine.register_umem(umem)
    try:
        assert np.array_equal(host_batch(engine, umem, desc, X.MODE_V4_LEGACY), exp)
        assert np.array_equal(host_batch(engine, umem, desc, X.MODE_V4_LEGACY, X.F_ZEROCOPY),
                              exp)
    finally:
        engine.unregister_umem(umem)


def test_host_batch_umem_mirror_layout(engine):
    """xudp's own TX layout: 4096-byte chunks, eth at F+342 (IPv4)."""
    umem, desc = X.gen_frames_host(5000, 4, 0, 1458, seed=8, stride=4096, offset=342)
    got = host_batch(engine, umem, desc, X.MODE_V4_LEGACY)
    assert np.array_equal(got, oracle.batch(umem, desc, X.MODE_V4_LEGACY))


@pytest.mark.parametrize("register", [False, True])
@pytest.mark.parametrize("n", [100, 5000, 70000])
@pytest.mark.parametrize("fam", [4, 6])
def test_host_batch_small_frames_in_slots(engine, n, fam, register):
    """Small frames one per 4096-byte chunk: in a pageable UMEM gathered frame
    by frame (xcsum_batch_host, gather_pays; copy-free up to 256 KiB, staged
    copies above, two chunks at 70,000 frames), in a registered one read in
    place without XCSUM_F_ZEROCOPY (zerocopy_pays); plain and in place."""
    umem, desc = X.gen_frames_host(n, fam, 0, 100, seed=31 + n, stride=4096,
                                   offset=322 if fam == 6 else 342)
    mode = X.MODE_V6 if fam == 6 else X.MODE_V4_RFC
    exp = oracle.batch(umem, desc, mode)
    flags = X.F_INPLACE | (X.F_IPHDR if fam == 4 else 0)
    before = umem.copy()
    if register:
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        engine.register_umem(umem)
    try:
        assert np.array_equal(host_batch(engine, umem, desc, mode), exp)
        assert np.array_equal(umem, before)
        assert np.array_equal(host_batch(engine, umem, desc, mode, flags), exp)
    finally:
        if register:
            engine.unregister_umem(umem)
    a = desc["addr"].astype(np.int64)
    chk = 60 if fam == 6 else 40
    got = umem[a[:, None] + np.array([chk, chk + 1])].copy().view("<u2").ravel()
    assert np.array_equal(got, exp)
    if fam == 4:
        iph = np.array([oracle.ip_header_rfc(umem[int(x):int(x) + 34]) for x in a[:200]])
        assert np.array_equal(umem[a[:200, None] + np.array([24, 25])].copy().view("<u2").ravel(),
                              iph)
    # nothing but the check fields changed
    mask = np.ones(len(umem), dtype=bool)
    for o in (chk, chk + 1) + ((24, 25) if fam == 4 else ()):
        mask[a + o] = False
    assert np.array_equal(umem[mask], before[mask])


@pytest.mark.parametrize("fam", [4, 6])
def test_host_batch_mtu_frames_in_slots_gathered(engine, monkeypatch, fam):
    """MTU frames one per 4096-byte chunk of a pageable UMEM fill ~1/3 of
    the range: gathered frame by frame since round 5 (gather_pays), the
    copies and the in-place stores split over threads (>= 16384 frames),
    several chunks.  The same results with the range copy
    (XCSUM_TUNE_GATHER_RATIO 8, the rule before) and through the receive path."""
    n = 40000
    umem, desc = X.gen_frames_host(n, fam, 1000, 1472 if fam == 4 else 1452, seed=77 + fam,
                                   stride=4096, offset=322 if fam == 6 else 342)
    mode = X.MODE_V6 if fam == 6 else X.MODE_V4_RFC
    exp = oracle.batch(umem, desc, mode)
    before = umem.copy()
    try:
        for ratio in (8, 0):
            engine.set_tuning(X.TUNE_GATHER_RATIO, ratio)     # 0: the default, 2
            assert np.array_equal(host_batch(engine, umem, desc, mode), exp), ratio
            assert np.array_equal(umem, before)
    finally:
        engine.set_tuning(X.TUNE_GATHER_RATIO, 0)
    flags = X.F_INPLACE | (X.F_IPHDR if fam == 4 else 0)
    assert np.array_equal(host_batch(engine, umem, desc, mode, flags), exp)
    a = desc["addr"].astype(np.int64)
    chk = 60 if fam == 6 else 40
    assert np.array_equal(umem[a[:, None] + np.array([chk, chk + 1])].copy().view("<u2").ravel(),
                          exp)
    mask = np.ones(len(umem), dtype=bool)
    for o in (chk, chk + 1) + ((24, 25) if fam == 4 else ()):
        mask[a + o] = False
    assert np.array_equal(umem[mask], before[mask])
    # receive side: every frame now verifies; one flipped payload byte fails it
    umem[a[n // 3] + 100] ^= 0x10
    msgs = np.zeros(n, dtype=X.RX_MSG_DTYPE)
    rx_flags = X.F_VERIFY | (X.F_IPHDR if fam == 4 else 0)
    assert engine.rx_host(umem, desc, msgs, rx_flags) == n - 1
    assert msgs["status"][n // 3] == X.RX_CSUM
    assert np.array_equal(msgs.view(np.uint8), oracle.rx_batch(umem, desc, rx_flags).view(np.uint8))


# ---- packet.c mirror --------------------------------------------------------

MAC1, MAC2 = bytes.fromhex("020000000001"), bytes.fromhex("020000000002")
A6 = lambda s: socket.inet_pton(socket.AF_INET6, s)


def kat_args():
    v6 = X.PacketArgs(6, b"abcdef", MAC1, MAC2, A6("1000:2000:3000:4000::2"), 3487,
                      A6("1000:2000:3000:4000::1"), 40000)
    v4 = X.PacketArgs(4, b"abcdef", MAC1, MAC2, socket.inet_aton("10.0.35.2"), 3486,
                      socket.inet_aton("10.0.35.1"), 40000)
    return v6, v4


def test_packet_udp_payload_kat3_kat4(torch_cuda):
    """xudp_packet_udp_payload (packet.c:196) frame bytes == Appendix A, checksums
    from the kernel."""
    v6, v4 = kat_args()
    X.packet_udp_payload(v6)
    X.packet_udp_payload(v4)
    assert v6.frame().tobytes().hex() == KAT3
    assert v4.frame().tobytes().hex() == KAT4


def test_packet_udp_single(torch_cuda):
    v6, v4 = kat_args()
    for pa in (v6, v4):
        pa.buf[64:70] = np.frombuffer(b"abcdef", dtype=np.uint8)
        X.packet_udp(pa)
    assert v6.frame().tobytes().hex() == KAT3
    assert v4.frame().tobytes().hex() == KAT4


@pytest.mark.parametrize("register", [False, True])
def test_packet_udp_batch_random(engine, register):
    """Many frames in one UMEM-like buffer, mixed families, one batch."""
    rng = np.random.default_rng(5)
    umem = np.zeros(4096 * 300, dtype=np.uint8)
    pas = []
    for i in range(300):
        fam = 6 if i % 3 == 0 else 4
        L = int(rng.integers(0, 1439))
        alen = 16 if fam == 6 else 4
        pa = X.PacketArgs(fam, rng.integers(0, 256, L, dtype=np.uint8).tobytes(),
                          rng.integers(0, 256, 6, dtype=np.uint8).tobytes(),
                          rng.integers(0, 256, 6, dtype=np.uint8).tobytes(),
                          rng.integers(0, 256, alen, dtype=np.uint8).tobytes(),
                          int(rng.integers(0, 65536)),
                          rng.integers(0, 256, alen, dtype=np.uint8).tobytes(),
                          int(rng.integers(0, 65536)), buf=umem, offset=4096 * i + 320)
        umem[4096 * i + 320 + 64:4096 * i + 320 + 64 + L] = pa.payload[:L]
        pas.append(pa)
    if register:
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        engine.register_umem(umem)
    try:
        X.packet_udp_batch(engine, pas)
    finally:
        if register:
            engine.unregister_umem(umem)
    for pa in pas:
        f = pa.frame()
        z = f.copy()
        desc = np.zeros(1, dtype=X.DESC_DTYPE)
        desc["len"] = len(f)
        if pa.family == 6:
            z[60:62] = 0
            assert int(f[60:62].view("<u2")[0]) == oracle.batch(z, desc, X.MODE_V6)[0]
        else:
            assert f[40:42].tobytes() == b"\0\0"          # packet.c:125, udp->check = 0
            assert int(f[24:26].view("<u2")[0]) == oracle.ip_header_rfc(f)
    # opt-in RFC UDP checksum for IPv4
    X.packet_udp_batch(engine, pas[1:3], X.F_V4_RFC)
    for pa in pas[1:3]:
        f = pa.frame()
        z = f.copy()
        z[40:42] = 0
        desc = np.zeros(1, dtype=X.DESC_DTYPE)
        desc["len"] = len(f)
        assert int(f[40:42].view("<u2")[0]) == oracle.batch(z, desc, X.MODE_V4_RFC)[0]


@pytest.mark.parametrize("how", ["pageable", "registered", "resident"])
def test_packet_udp_batch_ipv4_large(engine, how):
    """An all-IPv4 batch of 70,000 frames through the hook: libxudp's IPv4
    call (XCSUM_F_IPHDR_ONLY: 42-byte gathers from pageable memory over two
    chunks, in-place header reads from a registered UMEM); on a context with
    resident workgroups the checksum kernel on 42-byte headers.  Every
    iph->check is xudp_checksum_half's value, every udp->check 0, nothing
    else written but the headers."""
    from test_gpu_iphdr import hdr_np
    n, slot = 70000, 2048
    rng = np.random.default_rng(9)
    umem = np.zeros(n * slot, dtype=np.uint8)
    eng = engine
    if how == "registered":
        umem = X.umem_buffer(n * slot)
        engine.register_umem(umem)
        assert engine.umem_mapped(umem) == 1
    elif how == "resident":
        eng = X.Engine(0)
        eng.set_resident(8)
    pay = rng.integers(0, 256, (n, 1400), dtype=np.uint8)
    lens = rng.integers(0, 1401, n)
    pas = []
    for i in range(n):
        off = slot * i + 320
        umem[off + 64:off + 64 + lens[i]] = pay[i, :lens[i]]
        pas.append(X.PacketArgs(4, b"", b"\x02\0\0\0\0\x01", b"\x02\0\0\0\0\x02",
                                bytes([10, 0, 35, i & 255]), 3486 + (i & 1023),
                                bytes([10, 1, (i >> 8) & 255, 1]), 40000, buf=umem, offset=off))
        pas[-1].info.payload = umem.ctypes.data + off + 64     # payload already in place
        pas[-1].info.payload_size = int(lens[i])
    before = umem.copy()
    try:
        X.packet_udp_batch(eng, pas)
    finally:
        if how == "registered":
            engine.unregister_umem(umem)
        if eng is not engine:
            eng.close()
    eth = np.array([p.info.packet - umem.ctypes.data for p in pas], np.int64)
    assert np.array_equal(np.array([p.info.len for p in pas]), lens + 42)
    got = umem[eth[:, None] + np.array([24, 25])].copy().view("<u2").ravel()
    assert np.array_equal(got, hdr_np(umem, eth))
    assert not umem[eth[:, None] + np.array([40, 41])].any()      # packet.c:125
    mask = np.ones(len(umem), dtype=bool)
    for k in range(42):
        mask[eth + k] = False
    assert np.array_equal(umem[mask], before[mask])


def _guarded_pages(npages=3, hole=1):
    """An anonymous mapping of `npages` pages whose page `hole` is PROT_NONE:
    reading the address range across it faults."""
    import ctypes
    import mmap
    pg = mmap.PAGESIZE
    mm = mmap.mmap(-1, npages * pg, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS,
                   prot=mmap.PROT_READ | mmap.PROT_WRITE)
    buf = np.frombuffer(mm, dtype=np.uint8)
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mprotect.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert libc.mprotect(buf.ctypes.data + hole * pg, pg, 0) == 0
    return mm, buf, pg


@pytest.mark.parametrize("rfc", [False, True])
def test_packet_udp_batch_frames_around_unmapped_page(engine, rfc):
    """Frames in the caller's buffers with an unmapped page between them: the
    staged path copies frame by frame (the address range they span is not
    readable), and IPv4 without V4_RFC ships headers only."""
    mm, buf, pg = _guarded_pages()
    rng = np.random.default_rng(9)
    pas = []
    for fam, off, L in ((4, 100, 1000), (6, 2 * pg + 40, 900), (4, 2 * pg + 2000, 77)):
        alen = 16 if fam == 6 else 4
        pa = X.PacketArgs(fam, rng.integers(0, 256, L, dtype=np.uint8).tobytes(), MAC1, MAC2,
                          rng.integers(0, 256, alen, dtype=np.uint8).tobytes(), 1000 + L,
                          rng.integers(0, 256, alen, dtype=np.uint8).tobytes(), 2000 + L,
                          buf=buf, offset=off)
        buf[off + 64:off + 64 + L] = pa.payload[:L]
        pas.append(pa)
    X.packet_udp_batch(engine, pas, X.F_V4_RFC if rfc else 0)
    for pa in pas:
        f = pa.frame()
        z = f.copy()
        desc = np.zeros(1, dtype=X.DESC_DTYPE)
        desc["len"] = len(f)
        if pa.family == 6:
            z[60:62] = 0
            assert int(f[60:62].view("<u2")[0]) == oracle.batch(z, desc, X.MODE_V6)[0]
        else:
            assert int(f[24:26].view("<u2")[0]) == oracle.ip_header_rfc(f)
            if rfc:
                z[40:42] = 0
                assert int(f[40:42].view("<u2")[0]) == oracle.batch(z, desc, X.MODE_V4_RFC)[0]
            else:
                assert f[40:42].tobytes() == b"\0\0"
    del pas, buf   # the mapping goes with its last view


@pytest.mark.parametrize("how", ["device", "pageable", "registered", "zerocopy"])
def test_inplace_skips_truncated_frame(torch_cuda, engine, how):
    """INPLACE never writes for a frame the kernel rejects as malformed: a
    20-byte runt packed right before a valid frame would otherwise get its
    'udp->check' (runt + 40) stored into the next frame's bytes."""
    umem, desc = X.gen_frames_host(2, 4, 50, 50, seed=3, align=1)
    runt = np.zeros(1, dtype=X.DESC_DTYPE)
    big = np.zeros(len(umem) + 20, dtype=np.uint8)
    big[20:] = umem
    big[:20] = 0x33
    d = np.concatenate([runt, desc])
    d["addr"][1:] += 20
    d["len"][0] = 20
    exp = oracle.batch(big, d, X.MODE_V4_RFC)
    before = big.copy()
    engine.take_errors()   # clear what earlier tests left
    if how == "device":
        got, after = run_device(torch_cuda, engine, big, d, X.MODE_V4_RFC, X.F_INPLACE)
    else:
        flags = X.F_INPLACE
        if how != "pageable":
            big = X.as_umem(big)   # libxudp's UMEM mapping
            engine.register_umem(big)
        after = big
        if how == "zerocopy":
            flags |= X.F_ZEROCOPY
        try:
            got = host_batch(engine, big, d, X.MODE_V4_RFC, flags)
        finally:
            if how != "pageable":
                engine.unregister_umem(big)
    assert np.array_equal(got, exp) and got[0] == 0
    assert engine.take_errors() == 1
    changed = set(np.nonzero(after != before)[0].tolist())
    own = {int(a) + k for a in d["addr"][1:] for k in (40, 41)}
    assert changed <= own            # only the valid frames' own udp->check fields


def _thp_staging_expected():
    """xcsum_register_umem stages THP-eligible memory unless THP is off for
    the system ([never]) or for this process (XCSUM_TEST_NO_THP)."""
    if os.environ.get("XCSUM_TEST_NO_THP"):
        return False
    try:
        return "[never]" not in open("/sys/kernel/mm/transparent_hugepage/enabled").read()
    except OSError:
        return True


def test_thp_eligible_memory_is_staged(engine):
    """every registered-memory GPU fault was on memory eligible
    for transparent huge pages.  A numpy array of >= 4 MiB (numpy marks it
    MADV_HUGEPAGE) is registered for bookkeeping only (xcsum_umem_mapped
    0) and staged -- with XCSUM_F_ZEROCOPY too -- while the same frames in a
    libxudp-style mapping (umem_buffer) are GPU-mapped; every transport gives
    the oracle's results and in-place bytes."""
    umem, desc = X.gen_frames_host(4000, 4, 1472, seed=81, align=8)
    assert umem.nbytes >= 4 << 20
    exp = oracle.batch(umem, desc, X.MODE_V4_RFC)
    for buf, mapped in ((umem.copy(), 0 if _thp_staging_expected() else 1),
                        (X.as_umem(umem), 1)):
        engine.register_umem(buf)
        try:
            assert engine.umem_mapped(buf) == mapped
            a = desc["addr"].astype(np.int64)
            for flags in (0, X.F_ZEROCOPY, X.F_INPLACE | X.F_IPHDR,
                          X.F_ZEROCOPY | X.F_INPLACE | X.F_IPHDR):
                buf[a[:, None] + np.array([24, 25, 40, 41])] = 0   # as packet.c leaves them
                got = host_batch(engine, buf, desc, X.MODE_V4_RFC, flags)
                assert np.array_equal(got, exp), (mapped, flags)
            check_inplace_frames(buf, desc, exp)
        finally:
            engine.unregister_umem(buf)
    with pytest.raises(X.XcsumError):
        engine.umem_mapped(umem)


def check_inplace_frames(buf, desc, exp):
    a = desc["addr"].astype(np.int64)
    assert np.array_equal(buf[a[:, None] + np.array([40, 41])].copy().view("<u2").ravel(), exp)
    for i in range(0, len(desc), 397):
        f = buf[int(a[i]):int(a[i]) + int(desc["len"][i])].copy()
        ip = int(f[24:26].view("<u2")[0])
        f[24:26] = 0
        assert ip == oracle.ip_header_rfc(f)
