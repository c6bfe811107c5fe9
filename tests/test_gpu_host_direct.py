"""GPU: the copy-free small-batch host path (csrc/xcsum_api.hip,
XCSUM_DIRECT_MAX = 256 KiB of gathered bytes).  Gathered batches at or below
the threshold are read and answered by the kernel in the pinned stage itself;
larger ones go through the staged copies.  Every call reuses the same two
stage slots, so these tests rewrite the frames between calls and check each
call against the oracle: a slot must never serve bytes of an earlier call."""
import numpy as np
import pytest

import libxudp_amd as X
import oracle

pytestmark = pytest.mark.gpu

MAC1, MAC2 = bytes.fromhex("020000000001"), bytes.fromhex("020000000002")


def make_batch(umem, n, fam, rng, size):
    """n frames, one per 4096-byte UMEM chunk (data at F + 384)."""
    pas = []
    alen = 16 if fam == 6 else 4
    for i in range(n):
        L = size if size is not None else int(rng.integers(0, 1439))
        pa = X.PacketArgs(fam, rng.integers(0, 256, L, dtype=np.uint8).tobytes(), MAC1, MAC2,
                          rng.integers(0, 256, alen, dtype=np.uint8).tobytes(),
                          int(rng.integers(0, 65536)),
                          rng.integers(0, 256, alen, dtype=np.uint8).tobytes(),
                          int(rng.integers(0, 65536)), buf=umem, offset=4096 * i + 320)
        umem[4096 * i + 384:4096 * i + 384 + L] = pa.payload[:L]
        pas.append(pa)
    return pas


def check(pas, rfc):
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


# (family, RFC flag, frames, payload): gathered bytes per call below and above
# 256 KiB -- IPv4 without RFC ships 42 header bytes per frame, the others
# whole frames (IPv6 MTU frames: 1534 B, 170 of them ~ 261 KB)
CASES = [(4, False, 1, None), (4, False, 100, None), (4, False, 1024, 1472),
         (6, False, 16, None), (6, False, 160, 1452), (6, False, 180, 1452),
         (4, True, 100, None), (4, True, 200, 1472)]


@pytest.mark.parametrize("fam,rfc,n,size", CASES)
def test_repeated_calls_reuse_slots(engine, fam, rfc, n, size):
    rng = np.random.default_rng(1000 * fam + n + (7 if rfc else 0))
    umem = np.zeros(4096 * n + 4096, dtype=np.uint8)
    for _ in range(6):   # 3 uses of each stage slot, new bytes every call
        pas = make_batch(umem, n, fam, rng, size)
        X.packet_udp_batch(engine, pas, X.F_V4_RFC if rfc else 0)
        check(pas, rfc)


def test_single_frame_calls_alternate_families(engine):
    """xudp_packet_udp one frame at a time (the per-packet drop-in), IPv4 and
    IPv6 alternating, through the default per-thread context."""
    rng = np.random.default_rng(77)
    umem = np.zeros(4096 * 2, dtype=np.uint8)
    for k in range(40):
        fam = 6 if k % 2 else 4
        pa = make_batch(umem, 1, fam, rng, None)[0]
        X.packet_udp(pa)
        check([pa], False)
