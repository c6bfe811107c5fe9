"""GPU: BASELINE config 1 -- 4096 x 64-byte UDP/IPv4 frames in host memory --
through the plumbing the config names: xcsum_batch_host (staged, registered,
zero-copy) and the packet.c mirror xudp_packet_udp_batch, with the SHA-256
digests the REFERENCE produced over the same frames (tests/golden/digests.json:
udp_checksum() output, the RFC variant, and the frame bytes)."""
import hashlib

import numpy as np
import pytest

import libxudp_amd as X
import oracle

pytestmark = pytest.mark.gpu


def sha16(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u2").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def config1(digests):
    d = digests["config1"]
    umem, desc = X.gen_frames_host(d["n"], d["family"], d["pmin"], d["pmax"], seed=d["seed"])
    return d, umem, desc


@pytest.mark.parametrize("how", ["staged", "registered", "zerocopy"])
def test_config1_batch_host_digest(engine, config1, how):
    d, umem, desc = config1
    umem = umem.copy()
    flags = X.F_ZEROCOPY if how == "zerocopy" else 0
    if how != "staged":
        umem = X.as_umem(umem)   # libxudp's UMEM mapping
        engine.register_umem(umem)
    try:
        for mode, key in ((X.MODE_V4_LEGACY, "sha256_out"), (X.MODE_V4_RFC, "sha256_out_v4_rfc")):
            out = np.zeros(len(desc), dtype=np.uint16)
            engine.batch_host(umem, desc, out, mode, flags)
            assert sha16(out) == d[key], (how, mode)
    finally:
        if how != "staged":
            engine.unregister_umem(umem)


def packet_args(umem, desc, slots=None):
    """packet_info for every generated frame: its MACs, addresses, ports and
    payload, built into xudp TX slots (one UMEM, 4096-byte chunks, data at
    F + 384) or, slots=None, each into its own buffer."""
    pas = []
    for i, dd in enumerate(desc):
        f = umem[int(dd["addr"]):int(dd["addr"]) + int(dd["len"])]
        sport = int(f[34]) << 8 | int(f[35])
        dport = int(f[36]) << 8 | int(f[37])
        kw = dict(buf=slots, offset=4096 * i + 320) if slots is not None else {}
        pa = X.PacketArgs(4, f[42:].tobytes(), f[6:12].tobytes(), f[0:6].tobytes(),
                          f[26:30].tobytes(), sport, f[30:34].tobytes(), dport, **kw)
        buf_off = (4096 * i + 320) if slots is not None else 0
        pa.buf[buf_off + 64:buf_off + 64 + len(f) - 42] = f[42:]
        pas.append(pa)
    return pas


@pytest.mark.parametrize("where", ["own_buffers", "umem_slots", "umem_registered"])
def test_config1_packet_udp_batch_digest(engine, config1, where):
    d, umem, desc = config1
    slots = np.zeros(4096 * len(desc), dtype=np.uint8) if where != "own_buffers" else None
    if where == "umem_registered":
        slots = X.as_umem(slots)   # libxudp's UMEM mapping
        engine.register_umem(slots)
    try:
        # packet.c semantics: udp->check = 0 (packet.c:125), iph->check computed
        pas = packet_args(umem, desc, slots)
        X.packet_udp_batch(engine, pas)
        frames = [pa.frame() for pa in pas]
        ip = np.array([int(f[24:26].view("<u2")[0]) for f in frames], dtype=np.uint16)
        assert all(f[40:42].tobytes() == b"\0\0" for f in frames)
        assert all(int(ip[k]) == oracle.ip_header_rfc(f) for k, f in enumerate(frames))
        h = hashlib.sha256()
        for f in frames:
            g = f.copy()
            g[24:26] = 0
            h.update(g.tobytes())
        assert h.hexdigest() == d["sha256_frames"]
        # opt-in RFC UDP checksum: the reference's RFC digest of the same frames
        pas = packet_args(umem, desc, slots)
        X.packet_udp_batch(engine, pas, X.F_V4_RFC)
        rfc = np.array([int(pa.frame()[40:42].view("<u2")[0]) for pa in pas], dtype=np.uint16)
        assert sha16(rfc) == d["sha256_out_v4_rfc"]
    finally:
        if where == "umem_registered":
            engine.unregister_umem(slots)
