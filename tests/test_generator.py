"""CPU: the synthetic-frame generator (product host code, shared with the
device kernel) writes exactly what the reference's xudp_packet_udp() writes,
is shard-consistent, and the byte-balanced sharding is a partition."""
import numpy as np
import pytest

import libxudp_amd as X
import oracle


def fields(f, fam):
    hdr = X.HDR6 if fam == 6 else X.HDR4
    o = 54 if fam == 6 else 34
    sa, da = (f[22:38], f[38:54]) if fam == 6 else (f[26:30], f[30:34])
    return dict(payload=f[hdr:].tobytes(), family=fam, smac=f[6:12].tobytes(),
                dmac=f[0:6].tobytes(), saddr=sa.tobytes(), sport=int(f[o]) << 8 | int(f[o + 1]),
                daddr=da.tobytes(), dport=int(f[o + 2]) << 8 | int(f[o + 3]))


@pytest.mark.skipif(not oracle.have_ref(), reason="oracle/_ref not built here")
@pytest.mark.parametrize("family", [4, 6])
def test_frames_equal_reference_builder(family):
    umem, desc = X.gen_frames_host(300, family, 0, 1500, seed=7, align=1)
    for d in desc:
        f = umem[d["addr"]:d["addr"] + d["len"]]
        a = fields(f, family)
        r = oracle.build_frame_ref(a["payload"], family, a["smac"], a["dmac"], a["saddr"],
                                   a["sport"], a["daddr"], a["dport"])
        if family == 4:
            r[24:26] = 0   # the reference has already filled iph->check
        else:
            r[60:62] = 0   # ... and udp->check
        assert np.array_equal(r, f)


@pytest.mark.parametrize("family", [4, 6])
def test_layout_packed_and_strided(family):
    hdr = X.HDR6 if family == 6 else X.HDR4
    desc, nbytes = X.gen_layout(1000, family, 0, 2000, seed=3, align=8)
    assert (desc["addr"] % 8 == 0).all()
    assert (desc["len"] >= hdr).all() and (desc["len"] <= hdr + 2000).all()
    ends = desc["addr"] + desc["len"]
    assert (desc["addr"][1:] >= ends[:-1]).all() and nbytes >= ends[-1]
    desc2, nbytes2 = X.gen_layout(1000, family, 0, 2000, seed=3, stride=4096, offset=342)
    assert np.array_equal(desc2["len"], desc["len"])
    assert np.array_equal(desc2["addr"], np.arange(1000) * 4096 + 342) and nbytes2 == 4096000


def test_fixed_size_and_uniform_range():
    desc, _ = X.gen_layout(5000, 4, 1472, 1472, seed=1)
    assert (desc["len"] == 1472 + 42).all()
    desc, _ = X.gen_layout(20000, 4, 64, 9000, seed=2)
    p = desc["len"] - 42
    assert p.min() >= 64 and p.max() <= 9000 and 4000 < p.mean() < 5100


def test_shard_consistency():
    """Frames [a, b) generated with first_index=a equal that slice of the whole."""
    u_all, d_all = X.gen_frames_host(900, 6, 0, 600, seed=5)
    u_part, d_part = X.gen_frames_host(300, 6, 0, 600, seed=5, first_index=300)
    for i in range(300):
        a, b = d_all[300 + i], d_part[i]
        assert a["len"] == b["len"]
        assert np.array_equal(u_all[a["addr"]:a["addr"] + a["len"]],
                              u_part[b["addr"]:b["addr"] + b["len"]])


@pytest.mark.parametrize("nshards", [1, 2, 3, 4, 8])
def test_shard_by_bytes_is_a_balanced_partition(nshards):
    desc, _ = X.gen_layout(50000, 4, 64, 9000, seed=11)
    ranges = [X.shard_by_bytes(desc, nshards, k) for k in range(nshards)]
    nxt = 0
    for first, count in ranges:
        assert first == nxt
        nxt = first + count
    assert nxt == len(desc)
    total = int(desc["len"].sum())
    for first, count in ranges:
        part = int(desc["len"][first:first + count].sum())
        assert abs(part - total / nshards) <= 9100


def test_shard_by_bytes_edges():
    desc, _ = X.gen_layout(3, 4, 10, 10)
    assert [X.shard_by_bytes(desc, 8, k)[1] for k in range(8)].count(0) >= 5
    assert sum(X.shard_by_bytes(desc, 8, k)[1] for k in range(8)) == 3
    empty = np.zeros(0, dtype=X.DESC_DTYPE)
    assert X.shard_by_bytes(empty, 4, 3) == (0, 0)
