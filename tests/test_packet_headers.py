"""CPU: the host half of the packet.c mirror -- xudp_packet_build_headers()
writes the same eth/IP/UDP header bytes as the reference's xudp_packet_udp()
(checksum fields left 0 for the kernel).  Pinned by Appendix A KAT3/KAT4 and,
where oracle/_ref exists, against the reference builder on random frames."""
import socket

import numpy as np
import pytest

import libxudp_amd as X
import oracle

from test_oracle import KAT3, KAT4

MAC1, MAC2 = bytes.fromhex("020000000001"), bytes.fromhex("020000000002")


def build(family, payload, saddr, sport, daddr, dport, smac=MAC1, dmac=MAC2):
    pa = X.PacketArgs(family, payload, smac, dmac, saddr, sport, daddr, dport)
    pa.buf[64:64 + len(payload)] = np.frombuffer(payload, dtype=np.uint8) if payload else 0
    X.packet_build_headers(pa)
    return pa


def test_kat3_header_bytes():
    a6 = lambda s: socket.inet_pton(socket.AF_INET6, s)
    pa = build(6, b"abcdef", a6("1000:2000:3000:4000::2"), 3487, a6("1000:2000:3000:4000::1"),
               40000)
    exp = np.frombuffer(bytes.fromhex(KAT3), dtype=np.uint8).copy()
    exp[60:62] = 0
    assert pa.info.len == 68 and pa.info.packet == pa.info.head + 2
    assert np.array_equal(pa.frame(), exp)


def test_kat4_header_bytes():
    pa = build(4, b"abcdef", socket.inet_aton("10.0.35.2"), 3486, socket.inet_aton("10.0.35.1"),
               40000)
    exp = np.frombuffer(bytes.fromhex(KAT4), dtype=np.uint8).copy()
    exp[24:26] = 0
    assert pa.info.len == 48 and pa.info.packet == pa.info.head + 22
    assert np.array_equal(pa.frame(), exp)


@pytest.mark.skipif(not oracle.have_ref(), reason="oracle/_ref not built here")
@pytest.mark.parametrize("family", [4, 6])
def test_random_headers_equal_reference_builder(family):
    rng = np.random.default_rng(family)
    alen = 16 if family == 6 else 4
    for L in list(range(0, 40)) + [1471, 1472]:
        pl = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        sa, da = rng.integers(0, 256, alen, dtype=np.uint8).tobytes(), \
            rng.integers(0, 256, alen, dtype=np.uint8).tobytes()
        sp, dp = int(rng.integers(0, 65536)), int(rng.integers(0, 65536))
        sm, dm = rng.integers(0, 256, 6, dtype=np.uint8).tobytes(), \
            rng.integers(0, 256, 6, dtype=np.uint8).tobytes()
        pa = build(family, pl, sa, sp, da, dp, sm, dm)
        r = oracle.build_frame_ref(pl, family, sm, dm, sa, sp, da, dp)
        if family == 4:
            r[24:26] = 0
        else:
            r[60:62] = 0
        assert np.array_equal(pa.frame(), r)
