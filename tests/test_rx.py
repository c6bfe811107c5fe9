"""Receive path on the CPU: the oracle's packet_parse() restatement against the
reference's own (include/packet_parse.h compiled in place, and its results
frozen in tests/golden/rx_fixtures.npz), and the receive records against the
way each fixture frame was constructed (tests/golden/rx_frames.py)."""
import os
import sys

import numpy as np
import pytest

import libxudp_amd as X
import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
import rx_frames  # noqa: E402


@pytest.fixture(scope="module")
def rx():
    z = np.load(os.path.join(GOLDEN, "rx_fixtures.npz"))
    d = {k: z[k] for k in z.files}
    d["desc"] = d["desc"].view(X.DESC_DTYPE)
    for k in ("rec_plain", "rec_verify", "rec_iphdr"):
        d[k] = d[k].view(X.RX_MSG_DTYPE)
    return d


def frames_of(rx):
    u = rx["umem"]
    return [u[int(a):int(a) + int(n)].tobytes() for a, n in zip(rx["desc"]["addr"],
                                                                 rx["desc"]["len"])]


def test_fixture_corpus_covers_every_branch(rx):
    exp = list(rx["expect"])
    for kind in ("ok", "csum", "parse", "stats", "iphdr", "quirk"):
        assert exp.count(kind) >= 5, kind
    st = rx["rec_verify"]["status"]
    for s in (X.RX_OK, X.RX_PARSE, X.RX_STATS, X.RX_CSUM):
        assert (st == s).sum() >= 5


def test_parse_matches_reference_fixtures(rx):
    got = np.array([oracle.packet_parse(f) for f in frames_of(rx)])
    assert np.array_equal(got, rx["refparse"])


@pytest.mark.skipif(not oracle.have_ref(), reason="needs oracle/_ref (build container)")
def test_parse_matches_reference_fuzz():
    """20k mutated frames: oracle packet_parse == the reference's, live."""
    rng = np.random.default_rng(11)
    base = [f for f, _ in rx_frames.corpus(seed=5)]
    for _ in range(20000):
        f = bytearray(base[int(rng.integers(0, len(base)))])
        for _ in range(int(rng.integers(0, 4))):
            if f:
                f[int(rng.integers(0, len(f)))] = int(rng.integers(0, 256))
        if f and rng.integers(0, 4) == 0:
            f = f[:int(rng.integers(0, len(f) + 1))]
        f = bytes(f)
        assert oracle.packet_parse(f) == oracle.ref_packet_parse(f), f.hex()


def test_records_match_construction(rx):
    """Status from how each frame was built, not from the oracle's arithmetic."""
    exp = rx["expect"]
    want = {"ok": (X.RX_OK, X.RX_OK, X.RX_OK), "csum": (X.RX_OK, X.RX_CSUM, X.RX_CSUM),
            "parse": (X.RX_PARSE,) * 3, "stats": (X.RX_STATS,) * 3,
            "iphdr": (X.RX_OK, X.RX_OK, X.RX_CSUM)}
    for i, e in enumerate(exp):
        if e not in want:
            continue
        got = (rx["rec_plain"]["status"][i], rx["rec_verify"]["status"][i],
               rx["rec_iphdr"]["status"][i])
        assert got == want[e], (i, e, got)


def test_fill_msg_fields(rx):
    """xudp_fill_msg() fields (channel.c:69-128) for well-formed frames."""
    for i, f in enumerate(frames_of(rx)):
        r = rx["rec_verify"][i]
        addr = int(rx["desc"]["addr"][i])
        assert int(r["frame"]) == addr
        if rx["expect"][i] not in ("ok", "iphdr", "stats"):
            continue
        v6 = f[12:14] == b"\x86\xdd"
        l4 = 54 if v6 else 14 + 4 * (f[14] & 0xf)
        assert r["family"] == (6 if v6 else 4) and r["l4_off"] == l4
        assert int(r["body"]) == addr + l4 + 8
        assert int(r["size"]) == int.from_bytes(f[l4 + 4:l4 + 6], "big") - 8
        assert int(r["sport_be"]).to_bytes(2, "little") == f[l4:l4 + 2]
        assert int(r["dport_be"]).to_bytes(2, "little") == f[l4 + 2:l4 + 4]
        na, so = (16, 22) if v6 else (4, 26)
        assert bytes(r["saddr"][:na]) == f[so:so + na]
        assert bytes(r["daddr"][:na]) == f[so + na:so + 2 * na]
        assert not r["saddr"][na:].any() and not r["daddr"][na:].any()


def test_parse_failures_are_zero_records(rx):
    r = rx["rec_verify"]
    bad = r["status"] == X.RX_PARSE
    assert bad.sum() > 0
    assert not r["body"][bad].any() and not r["size"][bad].any()
    assert not r["family"][bad].any() and not r["saddr"][bad].any()


def test_oracle_reproduces_stored_records(rx):
    for name, fl in (("plain", 0), ("verify", X.F_VERIFY), ("iphdr", X.F_VERIFY | X.F_IPHDR)):
        got = oracle.rx_batch(rx["umem"], rx["desc"], fl)
        assert np.array_equal(got.view(np.uint8), rx[f"rec_{name}"].view(np.uint8)), name
