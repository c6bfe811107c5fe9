"""GPU: the segmented-stream checksum kernel (csrc/variants/xcsum_seg.hip, an
A/B kernel outside libxcsum.so: runs only when XCSUM_LIB loads a variants
build; geometries
X.SEG_GEOMETRIES) against the oracle on the batch shapes it treats
differently: mixed sizes U[0, 9000] packed at byte and 8-byte alignment,
ragged unit counts, units whose descriptors are out of UMEM order or
overlap (walked), a unit whose region is over the 8 MiB cap (walked), a
sparse batch (the frame-group fallback), and every flag set.  The config-5
full-size digest with these geometries is in test_gpu_fullsize.py."""
import numpy as np
import pytest

import libxudp_amd as X
import oracle
from test_gpu_parity import geometry, run_device

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not X.variants_built(),
                                 reason="segmented stream: variants build only (XCSUM_LIB)")]

MODES = {4: X.MODE_V4_LEGACY, 6: X.MODE_V6}


def mixed(n, family, seed, align=8):
    return X.gen_frames_host(n, family, 0, 9000, seed=seed, align=align)


@pytest.mark.parametrize("geom", X.SEG_GEOMETRIES + X.SEG_ATOM_GEOMETRIES)
@pytest.mark.parametrize("family", [4, 6])
@pytest.mark.parametrize("align", [1, 8])
def test_seg_mixed_vs_oracle(torch_cuda, engine, geom, family, align):
    umem, desc = mixed(1000 + 37, family, seed=40 + family + align, align=align)
    mode = MODES[family]
    with geometry(engine, geom):
        for m in (mode, X.MODE_AUTO) + ((X.MODE_V4_RFC,) if family == 4 else ()):
            got, _ = run_device(torch_cuda, engine, umem, desc, m)
            assert np.array_equal(got, oracle.batch(umem, desc, m)), m


@pytest.mark.parametrize("geom", X.SEG_GEOMETRIES + X.SEG_ATOM_GEOMETRIES)
def test_seg_flags_vs_oracle(torch_cuda, engine, geom):
    """INPLACE | IPHDR writes the same bytes as the default kernel; VERIFY
    after it passes; one flipped byte per frame fails."""
    umem, desc = mixed(700, 4, seed=7)
    with geometry(engine, geom):
        got, after = run_device(torch_cuda, engine, umem, desc, X.MODE_V4_RFC,
                                X.F_INPLACE | X.F_IPHDR)
    exp, exp_after = run_device(torch_cuda, engine, umem, desc, X.MODE_V4_RFC,
                                X.F_INPLACE | X.F_IPHDR)
    assert np.array_equal(got, exp)
    assert np.array_equal(after, exp_after)
    with geometry(engine, geom):
        ok, _ = run_device(torch_cuda, engine, after, desc, X.MODE_V4_RFC,
                           X.F_VERIFY | X.F_IPHDR)
        assert (ok == 0).all()
        bad = after.copy()
        rng = np.random.default_rng(3)
        for d in desc:
            a, ln = int(d["addr"]), int(d["len"])
            bad[int(rng.integers(a + 26, a + ln))] ^= 0x40
        got, _ = run_device(torch_cuda, engine, bad, desc, X.MODE_V4_RFC, X.F_VERIFY)
        assert np.array_equal(got, oracle.batch(bad, desc, X.MODE_V4_RFC, X.F_VERIFY))
        assert (got != 0).all()


@pytest.mark.parametrize("geom", X.SEG_GEOMETRIES + X.SEG_ATOM_GEOMETRIES)
def test_seg_unsorted_and_overlapping_units(torch_cuda, engine, geom):
    """Units whose spans are out of order or overlap are walked: same output."""
    umem, desc = mixed(64 * 6 + 5, 4, seed=9)
    desc = desc.copy()
    rng = np.random.default_rng(1)
    u1 = np.arange(64, 128)
    desc[u1] = desc[rng.permutation(u1)]          # unit 1 shuffled
    desc[200] = desc[199]                         # unit 3: a duplicate frame
    desc[64 * 4 + 10], desc[64 * 4 + 11] = desc[64 * 4 + 11].copy(), desc[64 * 4 + 10].copy()
    with geometry(engine, geom):
        for mode in (X.MODE_V4_LEGACY, X.MODE_AUTO):
            got, _ = run_device(torch_cuda, engine, umem, desc, mode)
            assert np.array_equal(got, oracle.batch(umem, desc, mode)), mode
        got, _ = run_device(torch_cuda, engine, umem, desc, X.MODE_V4_RFC, X.F_VERIFY)
        assert np.array_equal(got, oracle.batch(umem, desc, X.MODE_V4_RFC, X.F_VERIFY))


@pytest.mark.parametrize("geom", X.SEG_GEOMETRIES + X.SEG_ATOM_GEOMETRIES)
def test_seg_region_over_cap_and_malformed(torch_cuda, engine, geom):
    """A 9 MiB hole inside one unit (its region is over the cap: walked), and
    malformed frames (too short, UDP length over 65535) in streamed units."""
    umem, desc = mixed(64 * 5, 4, seed=13)
    desc = desc.copy()
    hole = 9 << 20
    desc["addr"][64 * 2 + 30:] += hole
    big = np.zeros(len(umem) + hole, dtype=np.uint8)
    cut = int(desc["addr"][64 * 2 + 30]) - hole
    big[:cut] = umem[:cut]
    big[cut + hole:] = umem[cut:]
    desc["len"][5] = 41                              # shorter than eth+ip+udp
    desc["len"][64 * 3 + 7] = 20                     # shorter than the addresses
    with geometry(engine, geom):
        engine.take_errors()
        got, _ = run_device(torch_cuda, engine, big, desc, X.MODE_V4_LEGACY)
        assert np.array_equal(got, oracle.batch(big, desc, X.MODE_V4_LEGACY))
        assert engine.take_errors() == 2


@pytest.mark.parametrize("geom", X.SEG_GEOMETRIES + X.SEG_ATOM_GEOMETRIES)
def test_seg_sparse_batch_fallback(torch_cuda, engine, geom):
    """xudp's 4096-byte chunks (sparse): the frame-group fallback, frames up
    to 3 KB (over its 2 KiB preload: its walk)."""
    umem, desc = X.gen_frames_host(2000 + 3, 4, 0, 3000, seed=17, stride=4096, offset=342)
    with geometry(engine, geom):
        got, _ = run_device(torch_cuda, engine, umem, desc, X.MODE_V4_LEGACY)
    assert np.array_equal(got, oracle.batch(umem, desc, X.MODE_V4_LEGACY))


@pytest.mark.parametrize("geom", X.SEG_GEOMETRIES + X.SEG_ATOM_GEOMETRIES)
@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 130])
def test_seg_small_batches(torch_cuda, engine, geom, n):
    umem, desc = mixed(n, 6, seed=n)
    with geometry(engine, geom):
        got, _ = run_device(torch_cuda, engine, umem, desc, X.MODE_V6)
    assert np.array_equal(got, oracle.batch(umem, desc, X.MODE_V6))
