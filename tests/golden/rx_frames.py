"""Received-frame builders for the receive-path tests (tests/test_rx.py,
tests/test_gpu_rx.py) and fixtures (make_golden.py --only-rx).

Plain byte assembly of Ethernet + IPv4 (any ihl, options) / IPv6 (any chain
of extension headers) + UDP frames, with RFC 768/791/2460 checksums computed
here from first principles, plus the malformed shapes packet_parse()
(include/packet_parse.h:101-165) has to sort out.  Each builder returns
(frame bytes, expect) where expect is "ok", "csum", "parse" or "stats" as the
frame was constructed -- an expectation independent of the oracle.
"""
import numpy as np

NEXT_UDP, NEXT_TCP = 17, 6
EXT_OPT = (0, 43, 47, 50, 60, 135)      # HOP, ROUTING, GRE, ESP, DEST, MOBILITY
EXT_FRAG, EXT_AUTH = 44, 51


def ones_sum(b):
    """RFC 1071 one's-complement sum of big-endian words (odd tail padded)"""
    b = bytes(b)
    if len(b) % 2:
        b += b"\0"
    s = int(np.frombuffer(b, dtype=">u2").astype(np.int64).sum())
    while s >> 16:
        s = (s & 0xffff) + (s >> 16)
    return s


def csum(b):
    return (~ones_sum(b)) & 0xffff


def udp_datagram(payload, sport, dport, pseudo, zero_check=False):
    ulen = 8 + len(payload)
    hdr = sport.to_bytes(2, "big") + dport.to_bytes(2, "big") + ulen.to_bytes(2, "big")
    if zero_check:
        return hdr + b"\0\0" + payload
    c = csum(pseudo + hdr + b"\0\0" + payload)
    c = c or 0xffff
    return hdr + c.to_bytes(2, "big") + payload


def eth(h_proto, dmac=b"\x02\0\0\0\0\x02", smac=b"\x02\0\0\0\0\x01"):
    return dmac + smac + h_proto.to_bytes(2, "big")


def ipv4(payload, saddr, daddr, proto=NEXT_UDP, options=b"", ihl=None, good_check=True):
    ihl = 5 + len(options) // 4 if ihl is None else ihl
    tot = 4 * max(ihl, 5) + len(payload) if ihl >= 5 else 20 + len(payload)
    h = bytes([0x40 | (ihl & 0xf), 0]) + tot.to_bytes(2, "big") + b"\0\0\x40\0" + \
        bytes([64, proto]) + b"\0\0" + saddr + daddr + options
    c = csum(h)
    if not good_check:
        c ^= 0x1234
    return h[:10] + c.to_bytes(2, "big") + h[12:] + payload


def ipv6(payload, saddr, daddr, nexthdr=NEXT_UDP, ext=b""):
    plen = len(ext) + len(payload)
    return bytes([0x60, 0x03, 0x0d, 0x9f]) + plen.to_bytes(2, "big") + bytes([nexthdr, 64]) + \
        saddr + daddr + ext + payload


def ext_chain(kinds, rng, last=NEXT_UDP):
    """IPv6 extension headers of the given kinds, each pointing at the next"""
    out = b""
    for i, k in enumerate(kinds):
        nxt = kinds[i + 1] if i + 1 < len(kinds) else last
        if k == EXT_FRAG:
            out += bytes([nxt, 0]) + bytes(rng.integers(0, 256, 6, dtype=np.uint8))
        elif k == EXT_AUTH:
            hl = int(rng.integers(0, 3))
            n = (hl + 2) << 2
            out += bytes([nxt, hl]) + bytes(rng.integers(0, 256, n - 2, dtype=np.uint8))
        else:
            hl = int(rng.integers(0, 2))
            n = (hl + 1) << 3
            out += bytes([nxt, hl]) + bytes(rng.integers(0, 256, n - 2, dtype=np.uint8))
    return out


def rand_bytes(rng, n):
    return bytes(rng.integers(0, 256, n, dtype=np.uint8))


def v4_frame(rng, plen, options=b"", zero_check=False, same_addr=False):
    sa = rand_bytes(rng, 4)
    da = sa if same_addr else rand_bytes(rng, 4)
    pay = rand_bytes(rng, plen)
    ulen = 8 + plen
    pseudo = sa + da + bytes([0, 17]) + ulen.to_bytes(2, "big")
    u = udp_datagram(pay, int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), pseudo,
                     zero_check)
    return eth(0x0800) + ipv4(u, sa, da, options=options)


def v6_frame(rng, plen, zero_check=False, quirk_stats=False):
    sa = bytearray(rand_bytes(rng, 16))
    if quirk_stats:
        sa[8:12] = sa[4:8]   # iphdr saddr/daddr offsets 12/16 of the IPv6 header
    sa = bytes(sa)
    da = rand_bytes(rng, 16)
    pay = rand_bytes(rng, plen)
    ulen = 8 + plen
    pseudo = sa + da + ulen.to_bytes(4, "big") + b"\0\0\0\x11"
    u = udp_datagram(pay, int(rng.integers(1, 65536)), int(rng.integers(1, 65536)), pseudo,
                     zero_check)
    return eth(0x86DD) + ipv6(u, sa, da)


def pad60(frame, junk=None):
    """Ethernet minimum frame: pad to 60 bytes (zeros, or given junk)"""
    if len(frame) >= 60:
        return frame
    n = 60 - len(frame)
    return frame + (junk[:n] if junk is not None else b"\0" * n)


def corpus(seed=7):
    """[(frame, expect)] covering packet_parse()'s branches and the verify rules"""
    rng = np.random.default_rng(seed)
    out = []
    add = out.append
    sizes = [0, 1, 2, 3, 7, 17, 18, 63, 64, 65, 200, 511, 1023, 1472]
    for plen in sizes:
        add((v4_frame(rng, plen), "ok"))
        add((v4_frame(rng, plen, zero_check=True), "ok"))    # IPv4: no checksum
        add((v6_frame(rng, plen), "ok"))
        add((v6_frame(rng, plen, zero_check=True), "csum"))  # IPv6: zero invalid
    for plen in (0, 1, 5, 10, 17):                           # Ethernet padding
        add((pad60(v4_frame(rng, plen)), "ok"))
        add((pad60(v4_frame(rng, plen), rand_bytes(rng, 60)), "ok"))
    for ihl in range(6, 16):                                 # IPv4 options
        add((v4_frame(rng, int(rng.integers(0, 300)), options=rand_bytes(rng, 4 * (ihl - 5))),
             "ok"))
    for ihl in range(0, 5):                                  # ihl < 5: parse quirk
        f = bytearray(v4_frame(rng, 40))
        f[14] = 0x40 | ihl
        add((bytes(f), "csum"))
    for plen in (0, 30, 700):                                # stats requests
        add((v4_frame(rng, plen, same_addr=True), "stats"))
        add((v6_frame(rng, plen, quirk_stats=True), "stats"))
    for _ in range(12):                                      # corrupted bytes
        f = bytearray(v4_frame(rng, int(rng.integers(1, 600))))
        f[int(rng.integers(34, len(f)))] ^= 1 << int(rng.integers(0, 8))
        add((bytes(f), "csum"))
        f = bytearray(v6_frame(rng, int(rng.integers(1, 600))))
        f[int(rng.integers(22, len(f)))] ^= 1 << int(rng.integers(0, 8))
        add((bytes(f), "csum"))
    for _ in range(6):                                       # bad IPv4 header checksum
        f = bytearray(v4_frame(rng, int(rng.integers(0, 100))))
        f[24] ^= 0x40
        add((bytes(f), "iphdr"))
    for delta in (-9, -1, 1, 100):                           # udp->len inconsistent
        f = bytearray(v4_frame(rng, 50))
        ulen = 58 + delta
        f[38:40] = ulen.to_bytes(2, "big", signed=False) if ulen >= 0 else b"\0\0"
        add((bytes(f), "csum"))
    # IPv6 extension headers: the reference takes UDP at iph6 + 1 anyway
    for kinds in ([0], [60], [43], [EXT_FRAG], [EXT_AUTH], [0, 60, 43], [135, 47, 50],
                  [0] * 7, [0] * 8, [60] * 9):
        pay = rand_bytes(rng, 40)
        sa, da = rand_bytes(rng, 16), rand_bytes(rng, 16)
        u = udp_datagram(pay, 1234, 5678, sa + da + (48).to_bytes(4, "big") + b"\0\0\0\x11")
        f = eth(0x86DD) + ipv6(ext_chain(kinds, rng) + u, sa, da, nexthdr=kinds[0])
        add((f, "quirk"))
    for nh in (NEXT_TCP, 58, 59, 41, 132, 99):               # not UDP
        add((eth(0x86DD) + ipv6(rand_bytes(rng, 40), rand_bytes(rng, 16), rand_bytes(rng, 16),
                                nexthdr=nh), "parse"))
        add((eth(0x0800) + ipv4(rand_bytes(rng, 40), rand_bytes(rng, 4), rand_bytes(rng, 4),
                                proto=nh), "parse"))
    for proto in (0x0806, 0x8100, 0x0800, 0x1200, 0x86DD, 0x86DE, 0x88DD, 0x0000):
        f = bytearray(v4_frame(rng, 30))                     # h_proto quirks
        f[12:14] = proto.to_bytes(2, "big")
        add((bytes(f), "quirk"))
    for n in (0, 1, 13, 14, 20, 33, 34, 41, 42, 53, 54, 61, 62):   # truncated
        src = v4_frame(rng, 40) if n < 45 else v6_frame(rng, 40)
        # a UDP header that fits parses; its length then does not
        add((src[:n], "parse" if n < (42 if n < 45 else 62) else "csum"))
    for _ in range(40):                                      # random junk after eth
        f = bytearray(rand_bytes(rng, int(rng.integers(14, 200))))
        f[12:14] = [(0x08, 0x00), (0x86, 0xDD), (0x08, 0x06), (0x81, 0x00)][
            int(rng.integers(0, 4))]
        if len(f) > 23 and rng.integers(0, 2):
            f[23] = 17
        add((bytes(f), "quirk"))
    return out


def layout(frames, rng, align_max=7):
    """frames at irregular byte offsets in one buffer -> (umem, desc fields)"""
    offs, pos = [], 64
    for f in frames:
        pos += int(rng.integers(0, align_max + 1))
        offs.append(pos)
        pos += len(f)
    umem = np.zeros(pos + 64, dtype=np.uint8)
    for o, f in zip(offs, frames):
        umem[o:o + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return umem, np.array(offs, dtype=np.uint64), np.array([len(f) for f in frames],
                                                           dtype=np.uint32)
