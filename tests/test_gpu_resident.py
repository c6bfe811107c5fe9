"""GPU: host batches served by resident workgroups (xcsum_ctx_set_resident,
csrc/xcsum_resident.hip) against the reference fixtures and the oracle.  The
resident path must give the same bytes as the launched one in every mode,
flag and transport (registered or pageable UMEM: the frames are gathered into
the library's pinned stage),
stay correct when the same UMEM changes between calls (no stale cache
lines), and serve every frame exactly once when its workgroups leave and
come back between calls (an in-place frame served twice would sum its own
check field)."""
import time

import numpy as np
import pytest

import libxudp_amd as X
import oracle
from conftest import golden_desc, h2d, d2h
from test_gpu_host_path import check_inplace, host_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def res_engine():
    e = X.Engine(0)
    e.set_resident(8)
    yield e
    e.close()


@pytest.mark.parametrize("mode,col,fam", [(X.MODE_V4_LEGACY, "exp_legacy", 4),
                                          (X.MODE_V4_RFC, "exp_rfc", 4),
                                          (X.MODE_V6, "exp_v6", 6)])
@pytest.mark.parametrize("register", [False, True])
def test_resident_golden(res_engine, golden, mode, col, fam, register):
    sel = np.nonzero(golden["family"] == fam)[0]
    umem = golden["umem"].copy()
    if register:
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        res_engine.register_umem(umem)
    try:
        for lo in range(0, len(sel), 300):       # batches the resident path takes
            s = sel[lo:lo + 300]
            got = host_batch(res_engine, umem, golden_desc(golden, s), mode)
            assert np.array_equal(got, golden[col][s])
    finally:
        if register:
            res_engine.unregister_umem(umem)


@pytest.mark.parametrize("how", ["pageable", "registered", "zerocopy"])
def test_resident_inplace(res_engine, golden, how):
    umem = golden["umem"].copy()
    desc = golden_desc(golden)
    flags = X.F_INPLACE | X.F_IPHDR
    if how != "pageable":
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        res_engine.register_umem(umem)
    if how == "zerocopy":
        flags |= X.F_ZEROCOPY
    try:
        got = host_batch(res_engine, umem, desc, X.MODE_AUTO, flags)
    finally:
        if how != "pageable":
            res_engine.unregister_umem(umem)
    fam = golden["family"]
    assert np.array_equal(got, np.where(fam == 6, golden["exp_v6"], golden["exp_legacy"]))
    check_inplace(golden, umem, desc)


def test_resident_verify(res_engine, golden):
    """VERIFY through the resident workgroups: frames with their reference
    checksum in place verify (0); a corrupted payload byte does not."""
    sel = np.nonzero(golden["family"] == 6)[0][:200]
    desc = golden_desc(golden, sel)
    umem = golden["umem"].copy()
    for i, d in zip(sel, desc):
        a = int(d["addr"])
        umem[a + 60:a + 62] = np.array([golden["exp_v6"][i]], dtype="<u2").view(np.uint8)
    assert not host_batch(res_engine, umem, desc, X.MODE_V6, X.F_VERIFY).any()
    a = int(desc["addr"][7])
    umem[a + int(desc["len"][7]) - 1] ^= 0x40
    got = host_batch(res_engine, umem, desc, X.MODE_V6, X.F_VERIFY)
    assert got[7] != 0 and np.count_nonzero(got) == 1


@pytest.mark.parametrize("fam", [4, 6])
@pytest.mark.parametrize("register", [False, True])
def test_resident_slots(res_engine, fam, register):
    """xudp's TX layout (one frame per 4096-byte chunk), pageable and
    registered UMEM (gathered either way); in place + IP header."""
    umem, desc = X.gen_frames_host(100, fam, 0, 1458, seed=77 + fam, stride=4096,
                                   offset=322 if fam == 6 else 342)
    mode = X.MODE_V6 if fam == 6 else X.MODE_V4_RFC
    exp = oracle.batch(umem, desc, mode)
    if register:
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        res_engine.register_umem(umem)
    try:
        assert np.array_equal(host_batch(res_engine, umem, desc, mode), exp)
        got = host_batch(res_engine, umem, desc, mode,
                         X.F_INPLACE | (X.F_IPHDR if fam == 4 else 0))
        assert np.array_equal(got, exp)
    finally:
        if register:
            res_engine.unregister_umem(umem)
    a = desc["addr"].astype(np.int64)
    chk = 60 if fam == 6 else 40
    assert np.array_equal(umem[a[:, None] + np.array([chk, chk + 1])].copy().view("<u2").ravel(),
                          exp)


@pytest.mark.parametrize("n", [1, 2, 99, 100, 1024, 4096, 4097, 20000])
def test_resident_sizes(res_engine, n):
    """Batch sizes around the resident limit (4096 frames): larger batches
    and staged ranges over 256 KiB take the launched path; same results."""
    umem, desc = X.gen_frames_host(n, 4, 0, 1472, seed=n, align=8)
    exp = oracle.batch(umem, desc, X.MODE_V4_LEGACY)
    assert np.array_equal(host_batch(res_engine, umem, desc, X.MODE_V4_LEGACY), exp)
    umem = X.as_umem(umem)   # libxudp's UMEM mapping
    res_engine.register_umem(umem)
    try:
        assert np.array_equal(host_batch(res_engine, umem, desc, X.MODE_V4_LEGACY), exp)
    finally:
        res_engine.unregister_umem(umem)
    assert res_engine.pending() == 0


def test_resident_fresh_bytes_every_call(res_engine):
    """The same registered UMEM rewritten between calls: every call must read
    the new bytes (the workgroups' acquire drops cached lines)."""
    umem, desc = X.gen_frames_host(100, 6, 0, 1400, seed=5, stride=4096, offset=322)
    umem = X.as_umem(umem)   # libxudp's UMEM mapping
    res_engine.register_umem(umem)
    rng = np.random.default_rng(1)
    a = desc["addr"].astype(np.int64)
    try:
        for it in range(200):
            k = int(rng.integers(0, 100))
            pos = a[k] + 62 + int(rng.integers(0, int(desc["len"][k]) - 62))
            umem[pos] = rng.integers(0, 256)
            got = host_batch(res_engine, umem, desc, X.MODE_V6)
            assert np.array_equal(got, oracle.batch(umem, desc, X.MODE_V6)), it
    finally:
        res_engine.unregister_umem(umem)


def test_resident_fresh_descriptors_every_call(res_engine):
    """A different batch every call (size, frames, order) from one registered
    UMEM: the descriptors the host wrote into the doorbell are the ones read."""
    umem, desc = X.gen_frames_host(2000, 4, 0, 1472, seed=12, stride=2048, offset=64)
    umem = X.as_umem(umem)   # libxudp's UMEM mapping
    res_engine.register_umem(umem)
    rng = np.random.default_rng(3)
    try:
        for it in range(300):
            n = int(rng.integers(1, 400))
            d = desc[rng.choice(len(desc), n, replace=False)]
            got = host_batch(res_engine, umem, d, X.MODE_V4_RFC)
            assert np.array_equal(got, oracle.batch(umem, d, X.MODE_V4_RFC)), it
    finally:
        res_engine.unregister_umem(umem)


def test_resident_fresh_staged_bytes_every_call(res_engine):
    """Small frames in a pageable UMEM (gathered into the pinned stage): one
    payload byte changes before every call, and every call must checksum the
    new bytes."""
    umem, desc = X.gen_frames_host(100, 6, 0, 300, seed=15, stride=2048, offset=64)
    rng = np.random.default_rng(5)
    a = desc["addr"].astype(np.int64)
    for it in range(300):
        k = int(rng.integers(0, 100))
        pos = a[k] + 62 + int(rng.integers(0, max(1, int(desc["len"][k]) - 62)))
        umem[pos] = rng.integers(0, 256)
        got = host_batch(res_engine, umem, desc, X.MODE_V6)
        assert np.array_equal(got, oracle.batch(umem, desc, X.MODE_V6)), it


def test_resident_large_descriptor_batches(res_engine):
    """4096-frame batches (the doorbell's capacity), a different selection
    and order every call, from a registered UMEM: all 64 KiB
    of descriptors must be the ones just written."""
    umem, desc = X.gen_frames_host(6000, 4, 0, 200, seed=16, stride=512, offset=0)
    exp_all = oracle.batch(umem, desc, X.MODE_V4_RFC)
    umem = X.as_umem(umem)   # libxudp's UMEM mapping
    res_engine.register_umem(umem)
    rng = np.random.default_rng(6)
    try:
        for it in range(60):
            n = 4096 if it % 2 == 0 else int(rng.integers(1000, 4097))
            sel = rng.choice(len(desc), n, replace=False)
            got = host_batch(res_engine, umem, desc[sel], X.MODE_V4_RFC)
            assert np.array_equal(got, exp_all[sel]), it
    finally:
        res_engine.unregister_umem(umem)


@pytest.mark.parametrize("idle_us", [1, 3, 30, 1000])
def test_resident_leave_and_return(idle_us):
    """Workgroups that leave after idle_us come back with the next batch; with
    a 1-30 us idle time they leave between (and during) calls, so relaunches
    after a partial service happen too.  In place on a registered UMEM: a
    frame served twice would sum its own, already written check field."""
    e = X.Engine(0)
    e.set_resident(16, idle_us)
    umem, desc = X.gen_frames_host(300, 6, 0, 1400, seed=9, stride=4096, offset=322)
    a = desc["addr"].astype(np.int64)
    chk = a[:, None] + np.array([60, 61])
    exp = oracle.batch(umem, desc, X.MODE_V6)
    umem = X.as_umem(umem)   # libxudp's UMEM mapping
    e.register_umem(umem)
    try:
        for it in range(300):
            umem[chk] = 0
            got = host_batch(e, umem, desc, X.MODE_V6, X.F_INPLACE)
            assert np.array_equal(got, exp), it
            assert np.array_equal(umem[chk].copy().view("<u2").ravel(), exp), it
            if it % 50 == 49:
                time.sleep(0.002)
    finally:
        e.unregister_umem(umem)
        e.close()


def test_resident_errors_and_switch(res_engine, golden):
    """Malformed frames are counted with resident workgroups live
    (take_errors stops them first); set_resident(0) falls back to launches,
    a new count takes effect on the next batch."""
    umem, desc = X.gen_frames_host(50, 4, 10, 200, seed=2, align=8)
    d = desc.copy()
    d["len"][3] = 20            # too short for the headers
    exp = oracle.batch(umem, d, X.MODE_V4_RFC)
    res_engine.take_errors()
    assert np.array_equal(host_batch(res_engine, umem, d, X.MODE_V4_RFC), exp)
    assert res_engine.take_errors() == 1
    for w in (0, 1, 64, 3):
        res_engine.set_resident(w)
        assert np.array_equal(host_batch(res_engine, umem, d, X.MODE_V4_RFC), exp)
    with pytest.raises(X.XcsumError):
        res_engine.set_resident(65)


def test_resident_packet_mirror(res_engine):
    """xudp_packet_udp_batch (the packet.c mirror) through a resident
    context: headers on the host, checksums from the resident workgroups."""
    from test_gpu_host_path import MAC1, MAC2
    rng = np.random.default_rng(4)
    umem = np.zeros(4096 * 100, dtype=np.uint8)
    pas = []
    for i in range(100):
        fam = 6 if i % 2 else 4
        L = int(rng.integers(0, 1439))
        alen = 16 if fam == 6 else 4
        pa = X.PacketArgs(fam, rng.integers(0, 256, L, dtype=np.uint8).tobytes(), MAC1, MAC2,
                          rng.integers(0, 256, alen, dtype=np.uint8).tobytes(), 1000 + i,
                          rng.integers(0, 256, alen, dtype=np.uint8).tobytes(), 2000 + i,
                          buf=umem, offset=4096 * i + 320)
        umem[4096 * i + 320 + 64:4096 * i + 320 + 64 + L] = pa.payload[:L]
        pas.append(pa)
    X.packet_udp_batch(res_engine, pas, X.F_V4_RFC)
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
            z[40:42] = 0
            assert int(f[40:42].view("<u2")[0]) == oracle.batch(z, desc, X.MODE_V4_RFC)[0]


@pytest.mark.parametrize("how", ["pageable", "registered"])
def test_resident_inplace_skips_truncated_frame(res_engine, how):
    """As test_gpu_host_path::test_inplace_skips_truncated_frame, through the
    resident workgroups: a 20-byte runt before a valid frame is counted as
    malformed and nothing outside the valid frames' check fields changes."""
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
    res_engine.take_errors()
    if how == "registered":
        big = X.as_umem(big)   # libxudp's UMEM mapping
        res_engine.register_umem(big)
    try:
        got = host_batch(res_engine, big, d, X.MODE_V4_RFC, X.F_INPLACE)
    finally:
        if how == "registered":
            res_engine.unregister_umem(big)
    assert np.array_equal(got, exp) and got[0] == 0
    assert res_engine.take_errors() == 1
    changed = set(np.nonzero(big != before)[0].tolist())
    assert changed <= {int(a) + k for a in d["addr"][1:] for k in (40, 41)}


def test_resident_auto_mixed_families_verify_iphdr(res_engine, golden):
    """AUTO mode over mixed IPv4/IPv6 fixtures with V4_RFC, then VERIFY +
    IPHDR on the frames the first call completed in place."""
    umem = golden["umem"].copy()
    desc = golden_desc(golden)
    fam = golden["family"]
    umem = X.as_umem(umem)   # libxudp's UMEM mapping
    res_engine.register_umem(umem)
    try:
        for lo in range(0, len(desc), 400):
            d = desc[lo:lo + 400]
            got = host_batch(res_engine, umem, d, X.MODE_AUTO,
                             X.F_V4_RFC | X.F_INPLACE | X.F_IPHDR)
            f = fam[lo:lo + 400]
            assert np.array_equal(got, np.where(f == 6, golden["exp_v6"][lo:lo + 400],
                                                golden["exp_rfc"][lo:lo + 400]))
            assert not host_batch(res_engine, umem, d, X.MODE_AUTO,
                                  X.F_VERIFY | X.F_IPHDR).any()
    finally:
        res_engine.unregister_umem(umem)


def test_resident_descriptor_check(monkeypatch, capfd):
    """The workgroups check every descriptor against the request's bounds
    inside the checksum loop, before any load of its frame: with the limit cut
    one byte short (test hook XCSUM_TUNE_RESIDENT_LIMIT_CUT) the last staged frame
    is refused, the call fails with XCSUM_ERR_INVAL and names it; the same
    context then serves the frames that fit.  Under the bounds-checked build
    the refused frame leaves no load outside its extent either."""
    e = X.Engine(0)
    e.set_tuning(X.TUNE_RESIDENT_LIMIT_CUT, 1)
    try:
        e.set_resident(8)
        umem, desc = X.gen_frames_host(100, 4, 0, 1400, seed=13, align=8)
        with pytest.raises(X.XcsumError) as ex:
            host_batch(e, umem, desc, X.MODE_V4_RFC)
        assert ex.value.rc == -X.ERR_INVAL
        assert "descriptor 99 " in capfd.readouterr().err
        exp = oracle.batch(umem, desc[:1], X.MODE_V4_RFC)
        # one frame: its limit is its own length, one byte short again
        with pytest.raises(X.XcsumError):
            host_batch(e, umem, desc[:1], X.MODE_V4_RFC)
        assert "descriptor 0 " in capfd.readouterr().err
    finally:
        e.close()
    e = X.Engine(0)
    try:
        e.set_resident(8)
        assert np.array_equal(host_batch(e, umem, desc[:1], X.MODE_V4_RFC), exp)
    finally:
        e.close()


def test_resident_inline_descriptors(res_engine):
    """Batches of 1-6 frames carry their descriptors in the polled doorbell
    lines (RB_INLINE): a different selection, order and count every call,
    alternating with larger batches that use the descriptor array, so a stale
    inline line would show as a wrong result."""
    umem, desc = X.gen_frames_host(500, 6, 0, 1400, seed=21, stride=2048, offset=64)
    umem = X.as_umem(umem)   # libxudp's UMEM mapping
    res_engine.register_umem(umem)
    rng = np.random.default_rng(8)
    try:
        for it in range(400):
            n = int(rng.integers(1, 7)) if it % 3 else int(rng.integers(7, 40))
            d = desc[rng.choice(len(desc), n, replace=False)]
            got = host_batch(res_engine, umem, d, X.MODE_V6)
            assert np.array_equal(got, oracle.batch(umem, d, X.MODE_V6)), (it, n)
    finally:
        res_engine.unregister_umem(umem)


def _busy_resident_loop(eng, stop, errors, calls):
    """Context `eng` keeps sending 100-frame batches (libxudp's tx_batch_num)
    through its resident workgroups until `stop` is set."""
    umem, desc = X.gen_frames_host(100, 4, 0, 1400, seed=61, align=8)
    exp = oracle.batch(umem, desc, X.MODE_V4_RFC)
    try:
        while not stop.is_set():
            if not np.array_equal(host_batch(eng, umem, desc, X.MODE_V4_RFC), exp):
                errors.append("mismatch")
                return
            calls[0] += 1
    except Exception as ex:   # surfaces in the main thread's assert
        errors.append(repr(ex))


def test_resident_peer_busy_teardown_bounded():
    """one context's take_errors, unregister_umem and destroy wait
    for that context's own work only -- never for a peer context whose
    resident workgroups stay busy (a device-wide wait would last as long as
    the peer keeps sending)."""
    import threading
    a = X.Engine(0)
    a.set_resident(8)
    stop, errors, calls = threading.Event(), [], [0]
    t = threading.Thread(target=_busy_resident_loop, args=(a, stop, errors, calls))
    t.start()
    try:
        time.sleep(0.05)
        b = X.Engine(0)
        b.set_resident(8)
        umem, desc = X.gen_frames_host(50, 6, 0, 600, seed=62, align=8)
        t0 = time.perf_counter()
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        b.register_umem(umem)
        assert np.array_equal(host_batch(b, umem, desc, X.MODE_V6),
                              oracle.batch(umem, desc, X.MODE_V6))
        b.take_errors()
        b.unregister_umem(umem)
        b.close()
        dt = time.perf_counter() - t0
        n_during = calls[0]
    finally:
        stop.set()
        t.join(60)
        a.close()
    assert not errors, errors
    assert n_during > 0
    assert dt < 2.0, f"teardown beside a busy peer took {dt:.3f} s"


@pytest.mark.parametrize("life_us", [None, 20000])
def test_resident_queue_sharing(torch_cuda, monkeypatch, capsys, life_us):
    """ADVICE r3 / VERDICT r5 #7: streams beyond GPU_MAX_HW_QUEUES share
    hardware queues, and work behind a live resident grid on a shared queue
    waits until the grid leaves.  A busy resident context in one thread,
    small device batches on eight fresh streams in this one; the slowest
    batch's wait is bounded by the resident life the context was given
    (xcsum_ctx_set_resident_life: the default 2 ms, and 20 ms) + 0.5 ms, and
    printed; results are always right."""
    import threading
    torch = torch_cuda
    dev = torch.device("cuda:0")
    a = X.Engine(0)
    a.set_resident(8)
    a.set_resident_life(life_us or 0)
    b = X.Engine(0)
    umem, desc = X.gen_frames_host(2000, 4, 0, 1472, seed=63, align=8)
    exp = oracle.batch(umem, desc, X.MODE_V4_LEGACY)
    d_umem = h2d(torch, umem, dev)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    streams = [torch.cuda.Stream(dev) for _ in range(8)]
    outs = [torch.zeros(len(desc), dtype=torch.int16, device=dev) for _ in streams]
    stop, errors, calls = threading.Event(), [], [0]
    t = threading.Thread(target=_busy_resident_loop, args=(a, stop, errors, calls))
    t.start()
    worst = 0.0
    try:
        time.sleep(0.05)
        for _ in range(5):
            for s, o in zip(streams, outs):
                t0 = time.perf_counter()
                b.batch_device(d_umem, d_desc, len(desc), o, X.MODE_V4_LEGACY, 0, 1500,
                               stream=s.cuda_stream)
                s.synchronize()
                worst = max(worst, time.perf_counter() - t0)
    finally:
        stop.set()
        t.join(60)
        a.close()
        b.close()
    assert not errors, errors
    for o in outs:
        assert np.array_equal(d2h(o).view(np.uint16), exp)
    with capsys.disabled():
        print(f"\n[queue sharing] resident life {life_us or 'default 2000'} us: slowest of 40 "
              f"device batches on 8 streams beside a busy resident context: "
              f"{worst * 1e3:.2f} ms ({calls[0]} resident calls meanwhile)")
    life_ms = (life_us or 2000) / 1e3
    assert worst * 1e3 <= life_ms + 0.5, f"a device batch waited {worst * 1e3:.2f} ms " \
                                         f"(resident life {life_ms} ms)"
