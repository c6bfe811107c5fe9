"""CPU: pin the oracle restatement (oracle/xcsum_oracle.c) to the reference.

Three anchors, strongest first:
  1. oracle/_ref -- the reference's own packet.c + checksum.h compiled in place
     (only where /root/reference exists; skipped elsewhere);
  2. tests/golden -- fixtures and digests generated from (1) by
     tests/golden/make_golden.py (travel everywhere);
  3. the known-answer vectors of SURVEY.md Appendix A.
"""
import hashlib
import socket
import struct

import numpy as np
import pytest

import libxudp_amd as X
import oracle
from conftest import golden_desc

needs_ref = pytest.mark.skipif(not oracle.have_ref(), reason="oracle/_ref not built here")


def a4(s):
    return struct.unpack("<I", socket.inet_aton(s))[0]  # network-order bytes as a u32


# ---- Appendix A known-answer tests ---------------------------------------

def test_kat1_udp_checksum():
    u = np.frombuffer(bytes.fromhex("0d9e1f90000e0000") + b"abcdef", dtype=np.uint8).copy()
    assert oracle.port().orc_udp_checksum(u.ctypes.data, a4("10.0.35.1"), a4("10.0.35.2"),
                                          14) == 0x4E74


def test_kat2_single_fold_quirk():
    """udp_checksum() drops the end-around carry: 0xfffe where RFC gives 0xfffd."""
    u = np.frombuffer(bytes.fromhex("ffffffff00100000fff6fff0fff4fff3"), dtype=np.uint8).copy()
    assert oracle.port().orc_udp_checksum(u.ctypes.data, 0xffffffff, 0xffffffff, 16) == 0xFFFE
    # the same bytes through the RFC path (mode V4_RFC) give 0xfffd (host order)
    frame = np.zeros(34 + 16, dtype=np.uint8)
    frame[12:14] = [0x08, 0x00]
    frame[26:34] = 0xff
    frame[34:] = u
    desc = np.zeros(1, dtype=X.DESC_DTYPE)
    desc["len"] = len(frame)
    assert oracle.batch(frame, desc, oracle.MODE_V4_RFC)[0] == 0xFDFF   # htons(0xfffd)
    assert oracle.batch(frame, desc, oracle.MODE_V4_LEGACY)[0] == 0xFEFF  # htons(0xfffe)


KAT3 = ("02000000000202000000000186dd60039f0d000e114010002000300040000000000000000002100020003"
        "000400000000000000000010d9f9c40000eebc1616263646566")
KAT4 = ("020000000002020000000001080045000022000040004011e0c80a0023020a0023010d9e9c40000e0000"
        "616263646566")


def test_kat3_ipv6_frame():
    f = np.frombuffer(bytes.fromhex(KAT3), dtype=np.uint8).copy()
    exp = int(f[60:62].view("<u2")[0])  # 'eb c1' as stored by udp_csum6
    assert f[60:62].tobytes() == b"\xeb\xc1"
    f[60:62] = 0
    desc = np.zeros(1, dtype=X.DESC_DTYPE)
    desc["len"] = len(f)
    assert oracle.batch(f, desc, oracle.MODE_V6)[0] == exp


def test_kat4_ipv4_frame():
    f = np.frombuffer(bytes.fromhex(KAT4), dtype=np.uint8).copy()
    assert f[24:26].tobytes() == b"\xe0\xc8" and f[40:42].tobytes() == b"\x00\x00"
    ip = f[14:34].copy()
    ip[10:12] = 0
    assert oracle.port().orc_ip_checksum_half(ip.ctypes.data) == 0xC8E0
    assert oracle.ip_header_rfc(np.concatenate([np.zeros(14, np.uint8), ip])) == 0xC8E0
    desc = np.zeros(1, dtype=X.DESC_DTYPE)
    desc["len"] = len(f)
    assert oracle.batch(f, desc, oracle.MODE_V4_LEGACY)[0] == 0xC3D1  # wire bytes d1 c3


@needs_ref
def test_kats_against_compiled_reference():
    R = oracle.ref()
    u = np.frombuffer(bytes.fromhex("0d9e1f90000e0000") + b"abcdef", dtype=np.uint8).copy()
    assert R.ref_udp_checksum(u.ctypes.data, a4("10.0.35.1"), a4("10.0.35.2"), 14) == 0x4E74
    u = np.frombuffer(bytes.fromhex("ffffffff00100000fff6fff0fff4fff3"), dtype=np.uint8).copy()
    assert R.ref_udp_checksum(u.ctypes.data, 0xffffffff, 0xffffffff, 16) == 0xFFFE
    a6 = lambda s: socket.inet_pton(socket.AF_INET6, s)
    f = oracle.build_frame_ref(b"abcdef", 6, bytes.fromhex("020000000001"),
                               bytes.fromhex("020000000002"), a6("1000:2000:3000:4000::2"), 3487,
                               a6("1000:2000:3000:4000::1"), 40000)
    assert f.tobytes().hex() == KAT3
    f = oracle.build_frame_ref(b"abcdef", 4, bytes.fromhex("020000000001"),
                               bytes.fromhex("020000000002"), socket.inet_aton("10.0.35.2"), 3486,
                               socket.inet_aton("10.0.35.1"), 40000)
    assert f.tobytes().hex() == KAT4


# ---- golden fixtures --------------------------------------------------------

def test_golden_fixture_shape(golden):
    fam = golden["family"]
    assert len(fam) > 900 and golden["umem"].nbytes < (1 << 20)
    lens = golden["len"]
    assert lens.min() == 42 and lens.max() >= 9000 + 42
    assert (golden["addr"] % 2 == 1).any()          # odd span starts covered
    q = (fam == 4) & (golden["exp_legacy"] != golden["exp_rfc"])
    assert q.sum() >= 100                          # quirk-triggering frames
    assert ((fam == 6) & (golden["exp_v6"] == 0xffff)).sum() >= 4  # CSUM_MANGLED_0 cases
    assert ((fam == 4) & (golden["exp_legacy"] == 0)).sum() >= 1


@pytest.mark.parametrize("col,mode,fam", [("exp_legacy", oracle.MODE_V4_LEGACY, 4),
                                          ("exp_rfc", oracle.MODE_V4_RFC, 4),
                                          ("exp_v6", oracle.MODE_V6, 6)])
def test_oracle_matches_golden(golden, col, mode, fam):
    sel = np.nonzero(golden["family"] == fam)[0]
    got = oracle.batch(golden["umem"], golden_desc(golden, sel), mode)
    assert np.array_equal(got, golden[col][sel])


def test_oracle_auto_mode_matches_golden(golden):
    fam = golden["family"]
    got = oracle.batch(golden["umem"], golden_desc(golden), oracle.MODE_AUTO)
    assert np.array_equal(got, np.where(fam == 6, golden["exp_v6"], golden["exp_legacy"]))
    got = oracle.batch(golden["umem"], golden_desc(golden), oracle.MODE_AUTO, 0x4)
    assert np.array_equal(got, np.where(fam == 6, golden["exp_v6"], golden["exp_rfc"]))


def test_oracle_ip_header_matches_golden(golden):
    P = oracle.port()
    for i in np.nonzero(golden["family"] == 4)[0]:
        a = int(golden["addr"][i])
        ip = np.ascontiguousarray(golden["umem"][a + 14:a + 34])
        assert P.orc_ip_checksum_half(ip.ctypes.data) == golden["exp_iphdr"][i]
        assert P.orc_ip_header_rfc(ip.ctypes.data) == golden["exp_iphdr"][i]


# ---- against the compiled reference on generated frames --------------------

@needs_ref
@pytest.mark.parametrize("family", [4, 6])
@pytest.mark.parametrize("align", [1, 8])
def test_oracle_vs_reference_random(family, align):
    umem, desc = X.gen_frames_host(4000, family, 0, 9000, seed=100 + family + align, align=align)
    mode = oracle.MODE_V6 if family == 6 else oracle.MODE_V4_LEGACY
    assert np.array_equal(oracle.batch(umem, desc, mode), oracle.ref_batch(umem, desc, mode))


@needs_ref
def test_oracle_rfc_vs_reference_primitives():
    R = oracle.ref()
    umem, desc = X.gen_frames_host(2000, 4, 0, 3000, seed=9, align=1)
    got = oracle.batch(umem, desc, oracle.MODE_V4_RFC)
    for i, d in enumerate(desc):
        a = int(d["addr"])
        f = umem[a:a + int(d["len"])]
        udp = np.ascontiguousarray(f[34:])
        sa, da = np.ascontiguousarray(f[26:30]), np.ascontiguousarray(f[30:34])
        assert got[i] == R.ref_udp_csum4_rfc(udp.ctypes.data, len(udp), sa.ctypes.data,
                                             da.ctypes.data)


def test_quirk_rate_matches_survey():
    """legacy != RFC on ~0.556 % of random 1472-byte payloads."""
    umem, desc = X.gen_frames_host(50000, 4, 1472, 1472, seed=1)
    leg = oracle.batch(umem, desc, oracle.MODE_V4_LEGACY)
    rfc = oracle.batch(umem, desc, oracle.MODE_V4_RFC)
    rate = float((leg != rfc).mean())
    assert 0.004 < rate < 0.0075, rate


def test_malformed_frames_give_zero():
    umem, desc = X.gen_frames_host(6, 4, 10, 10, seed=3)
    desc = desc.copy()
    desc["len"][0] = 41
    desc["len"][1] = 0
    desc["len"][2] = 34 + 65536
    umem = np.concatenate([umem, np.zeros(70000, np.uint8)])
    out = oracle.batch(umem, desc, oracle.MODE_V4_LEGACY)
    assert list(out[:3]) == [0, 0, 0]
    umem[int(desc["addr"][3]) + 12] = 0x42
    out = oracle.batch(umem, desc, oracle.MODE_AUTO)
    assert out[3] == 0


# ---- BASELINE config 1 (4096 x 64 B IPv4 on the host CPU) ------------------

def test_config1_digest(digests):
    d = digests["config1"]
    umem, desc = X.gen_frames_host(d["n"], d["family"], d["pmin"], d["pmax"], seed=d["seed"])
    h = hashlib.sha256()
    for dd in desc:
        h.update(umem[dd["addr"]:dd["addr"] + dd["len"]].tobytes())
    assert h.hexdigest() == d["sha256_frames"]
    out = oracle.batch(umem, desc, oracle.MODE_V4_LEGACY)
    assert hashlib.sha256(out.astype("<u2").tobytes()).hexdigest() == d["sha256_out"]
    rfc = oracle.batch(umem, desc, oracle.MODE_V4_RFC)
    assert hashlib.sha256(rfc.astype("<u2").tobytes()).hexdigest() == d["sha256_out_v4_rfc"]
    if oracle.have_ref():
        ref = oracle.ref_batch(umem, desc, 0)
        assert np.array_equal(ref, out)


def test_digest_file_covers_baseline_configs(digests):
    for c, (n, fam) in {1: (4096, 4), 2: (1 << 20, 4), 3: (1 << 20, 4), 4: (1 << 20, 6),
                        5: (8 << 20, 4)}.items():
        d = digests[f"config{c}"]
        assert d["n"] == n and d["family"] == fam and len(d["sha256_out"]) == 64
        assert d["seed"] == 0x78756470 ^ c


@pytest.mark.parametrize("cid", [2, 4])
def test_oracle_reproduces_fullsize_digest_prefix(digests, cid):
    """The first 64K frames of configs 2/4 through the oracle: the digest of the
    whole 1M-frame output is checked on the GPU; here, consistency of the
    generator + oracle with the reference on a prefix (reference recomputed
    only where it exists)."""
    d = digests[f"config{cid}"]
    umem, desc = X.gen_frames_host(1 << 16, d["family"], d["pmin"], d["pmax"], seed=d["seed"])
    mode = oracle.MODE_V6 if d["family"] == 6 else oracle.MODE_V4_LEGACY
    out = oracle.batch(umem, desc, mode)
    if oracle.have_ref():
        assert np.array_equal(out, oracle.ref_batch(umem, desc, mode))
    assert out.dtype == np.uint16 and len(out) == 1 << 16


# ---- XCSUM_F_IPHDR_ONLY: libxudp's IPv4 TX call (xudp_checksum_half alone) --

IPHDR_ONLY = 0x80


def test_iphdr_only_matches_golden(golden):
    """The oracle's header-only batch equals the reference's exp_iphdr on
    every IPv4 fixture frame; AUTO gives IPv6 frames 0."""
    fam = golden["family"]
    desc = golden_desc(golden)
    out = oracle.batch(golden["umem"], desc, oracle.MODE_V4_LEGACY, IPHDR_ONLY)
    assert np.array_equal(out[fam == 4], golden["exp_iphdr"][fam == 4])
    out = oracle.batch(golden["umem"], desc, oracle.MODE_AUTO, IPHDR_ONLY)
    assert np.array_equal(out, np.where(fam == 6, 0, golden["exp_iphdr"]))


@pytest.mark.parametrize("cid", [1, 2, 3, 5])
def test_iphdr_only_digests(digests, cid):
    """digests.json sha256_iphdr: the reference's xudp_checksum_half over
    every frame of the IPv4 configs (make_golden.py --only-iphdr).  Config
    1 in full through the oracle; the others on a 64K-frame prefix against
    the compiled reference where it exists."""
    d = digests[f"config{cid}"]
    assert len(d["sha256_iphdr"]) == 64
    m = d["n"] if cid == 1 else 1 << 16
    umem, desc = X.gen_frames_host(m, 4, d["pmin"], d["pmax"], seed=d["seed"])
    out = oracle.batch(umem, desc, oracle.MODE_V4_LEGACY, IPHDR_ONLY)
    if cid == 1:
        assert hashlib.sha256(out.astype("<u2").tobytes()).hexdigest() == d["sha256_iphdr"]
    if oracle.have_ref():
        ref = np.zeros(m, np.uint16)
        oracle.ref().ref_batch(umem.ctypes.data, desc.ctypes.data, m, ref.ctypes.data, 4)
        assert np.array_equal(out, ref)


def test_iphdr_only_rules():
    """Malformed frames and VERIFY in the oracle's header-only mode (the rules
    include/xcsum.h states for XCSUM_F_IPHDR_ONLY)."""
    umem, desc = X.gen_frames_host(64, 4, 0, 200, seed=4)
    good = oracle.batch(umem, desc, oracle.MODE_V4_LEGACY, IPHDR_ONLY)
    filled = umem.copy()
    for d, c in zip(desc, good):
        filled[int(d["addr"]) + 24:int(d["addr"]) + 26] = np.array([c], "<u2").view(np.uint8)
    assert not oracle.batch(filled, desc, oracle.MODE_V4_LEGACY, IPHDR_ONLY | VERIFY).any()
    bad = desc.copy()
    bad["len"][:4] = [0, 41, 65570, 70000]
    out = oracle.batch(filled, bad, oracle.MODE_V4_LEGACY, IPHDR_ONLY)
    assert list(out[:4]) == [0, 0, 0, 0] and np.array_equal(out[4:], good[4:])
    out = oracle.batch(filled, bad, oracle.MODE_V4_LEGACY, IPHDR_ONLY | VERIFY)
    assert list(out[:4]) == [0xffff] * 4 and not out[4:].any()


# ---- receive-side verify (the reference never verifies) --

def filled_golden(golden, v4_col="exp_rfc"):
    """Golden frames with their expected checksums written into the frames."""
    umem = golden["umem"].copy()
    for i, fam in enumerate(golden["family"]):
        a = int(golden["addr"][i])
        if fam == 6:
            umem[a + 60:a + 62] = np.array([golden["exp_v6"][i]], "<u2").view(np.uint8)
        else:
            umem[a + 40:a + 42] = np.array([golden[v4_col][i]], "<u2").view(np.uint8)
            umem[a + 24:a + 26] = np.array([golden["exp_iphdr"][i]], "<u2").view(np.uint8)
    return umem


VERIFY, IPHDR = 0x10, 0x2


def test_verify_accepts_reference_checksums(golden):
    umem = filled_golden(golden)
    out = oracle.batch(umem, golden_desc(golden), oracle.MODE_AUTO, VERIFY | IPHDR)
    assert (out == 0).all()


def test_verify_rejects_udp_checksum_quirk_values(golden):
    """checksum.h's udp_checksum() (single fold) writes values an RFC 768
    receiver rejects -- exactly on the frames where legacy != RFC."""
    umem = filled_golden(golden, "exp_legacy")
    out = oracle.batch(umem, golden_desc(golden), oracle.MODE_AUTO, VERIFY)
    fam = golden["family"]
    quirk = (fam == 4) & (golden["exp_legacy"] != golden["exp_rfc"])
    # a legacy value of 0 means "no checksum" to a receiver: accepted
    quirk &= golden["exp_legacy"] != 0
    assert (out[quirk] != 0).all() and (out[~quirk] == 0).all()


def test_verify_zero_check_and_corruption(golden):
    umem = filled_golden(golden)
    desc = golden_desc(golden)
    fam = golden["family"]
    z = umem.copy()
    for i, d in enumerate(desc):
        a = int(d["addr"])
        z[a + (60 if fam[i] == 6 else 40):a + (62 if fam[i] == 6 else 42)] = 0
    out = oracle.batch(z, desc, oracle.MODE_AUTO, VERIFY)
    assert (out[fam == 4] == 0).all() and (out[fam == 6] != 0).all()
    rng = np.random.default_rng(1)
    c = umem.copy()
    for i, d in enumerate(desc):       # flip one bit somewhere in each span
        a, ln = int(d["addr"]), int(d["len"])
        lo = a + (22 if fam[i] == 6 else 26)
        c[int(rng.integers(lo, a + ln))] ^= 1 << int(rng.integers(0, 8))
    out = oracle.batch(c, desc, oracle.MODE_AUTO, VERIFY)
    assert (out != 0).all()
    bad_ip = umem.copy()
    for i in np.nonzero(fam == 4)[0]:
        bad_ip[int(desc["addr"][i]) + 22] ^= 0x01          # TTL byte
    assert (oracle.batch(bad_ip, desc, oracle.MODE_AUTO, VERIFY | IPHDR)[fam == 4] != 0).all()
    assert (oracle.batch(bad_ip, desc, oracle.MODE_AUTO, VERIFY)[fam == 4] == 0).all()


def test_oracle_verify_uses_udp_length():
    """RFC 768 verify on received frames: the datagram ends at udp +
    ntohs(udp->len); Ethernet padding (zeros or junk) is not summed, and a
    UDP length below 8 or past the frame never verifies."""
    import rx_frames
    rng = np.random.default_rng(3)
    good, bad = [], []
    for plen in (0, 1, 5, 10, 17):
        good.append(rx_frames.pad60(rx_frames.v4_frame(rng, plen)))
        good.append(rx_frames.pad60(rx_frames.v4_frame(rng, plen), rx_frames.rand_bytes(rng, 60)))
    for plen in (64, 1472):
        good.append(rx_frames.v4_frame(rng, plen) + b"\x01" * 9)
        good.append(rx_frames.v6_frame(rng, plen) + b"\x80" * 3)
    for ulen in (0, 7, 200):
        f = bytearray(rx_frames.v4_frame(rng, 50))
        f[38:40] = ulen.to_bytes(2, "big")
        bad.append(bytes(f))
    for frames, ok in ((good, True), (bad, False)):
        umem, addr, ln = rx_frames.layout(frames, rng)
        desc = np.zeros(len(frames), dtype=X.DESC_DTYPE)
        desc["addr"] = addr
        desc["len"] = ln
        got = oracle.batch(umem, desc, oracle.MODE_AUTO, 0x10 | 0x2)
        assert ((got == 0) == ok).all(), got
