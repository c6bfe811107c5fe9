"""GPU: randomized parity.  Seeded random batches -- several families, payload
size ranges, alignments and layouts concatenated in one UMEM, descriptors
partly shuffled, random mode, flags, geometry and length hint -- through
xcsum_batch_device, against the oracle; and random receive corpora through
xcsum_rx_device for every receive geometry.  Each case prints its seed when
it fails, so it can be replayed alone (pytest -k 'fuzz and <seed>')."""
import numpy as np
import pytest

import libxudp_amd as X
import oracle
import rx_frames  # tests/golden (conftest puts it on sys.path)
from test_gpu_parity import run_device
from test_gpu_rx import GEOMETRIES as RX_GEOMETRIES, run_rx

pytestmark = pytest.mark.gpu

MODES = [X.MODE_V4_LEGACY, X.MODE_V4_RFC, X.MODE_V6, X.MODE_AUTO]
SIZE_RANGES = [(0, 64), (0, 300), (1000, 1500), (1400, 1472), (0, 9000), (8000, 9000)]


def random_batch(rng):
    """(umem, desc): 1-4 segments of generated frames (random family, size
    range, alignment or xudp chunk layout), descriptors partly shuffled."""
    parts, descs, base = [], [], 0
    for _ in range(int(rng.integers(1, 5))):
        fam = int(rng.choice([4, 6]))
        lo, hi = SIZE_RANGES[int(rng.integers(len(SIZE_RANGES)))]
        n = int(rng.integers(1, 1200))
        seed = int(rng.integers(1 << 30))
        if rng.random() < 0.2 and hi <= 3000:
            umem, desc = X.gen_frames_host(n, fam, lo, hi, seed=seed, stride=4096,
                                           offset=342 if fam == 4 else 322)
        else:
            umem, desc = X.gen_frames_host(n, fam, lo, hi, seed=seed,
                                           align=int(rng.choice([1, 2, 4, 8, 16])))
        pad = int(rng.integers(0, 64))
        d = desc.copy()
        d["addr"] += base
        descs.append(d)
        parts.append(umem)
        parts.append(np.zeros(pad, np.uint8))
        base += len(umem) + pad
    umem = np.concatenate(parts + [np.zeros(64, np.uint8)])
    desc = np.concatenate(descs)
    if rng.random() < 0.3:                    # a shuffled window
        a = int(rng.integers(0, len(desc)))
        b = min(len(desc), a + int(rng.integers(2, 300)))
        desc[a:b] = desc[a:b][rng.permutation(b - a)]
    if rng.random() < 0.2:                    # a few malformed lengths
        for i in rng.integers(0, len(desc), 3):
            desc["len"][i] = int(rng.choice([0, 13, 41, 61]))
    return umem, desc


@pytest.mark.parametrize("seed", range(160))
def test_fuzz_checksum_vs_oracle(torch_cuda, engine, seed):
    rng = np.random.default_rng(1000 + seed)
    umem, desc = random_batch(rng)
    geoms = [None] + X.GEOMETRIES
    geom = geoms[int(rng.integers(len(geoms)))]
    mode = MODES[int(rng.integers(len(MODES)))]
    hint = int(rng.choice([0, 64, 100, 600, 1500, 4500, 9000]))
    verify = rng.random() < 0.4
    if geom is not None:
        engine.set_geometry(*geom)
    try:
        if verify:
            # checks written first (RFC rules), then some frames corrupted
            wmode = X.MODE_AUTO if mode == X.MODE_AUTO else (
                X.MODE_V6 if mode == X.MODE_V6 else X.MODE_V4_RFC)
            _, umem = run_device(torch_cuda, engine, umem, desc, wmode,
                                 X.F_INPLACE | X.F_IPHDR | X.F_V4_RFC)
            for i in rng.integers(0, len(desc), max(1, len(desc) // 10)):
                a, ln = int(desc["addr"][i]), int(desc["len"][i])
                if ln > 30:
                    umem[a + int(rng.integers(14, ln))] ^= 1 << int(rng.integers(8))
            flags = X.F_VERIFY | (X.F_IPHDR if rng.random() < 0.5 else 0)
        else:
            flags = (X.F_V4_RFC if rng.random() < 0.3 else 0)
        got, after = run_device(torch_cuda, engine, umem, desc, mode, flags, hint)
        exp = oracle.batch(umem, desc, mode, flags)
        bad = np.nonzero(got != exp)[0]
        assert len(bad) == 0, f"seed {seed}: geom {geom} mode {mode} flags {flags:#x} " \
                              f"hint {hint}: frames {bad[:8].tolist()}"
        assert np.array_equal(after, umem)
    finally:
        engine.set_geometry(0)


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_receive_vs_oracle(torch_cuda, engine, seed):
    rng = np.random.default_rng(2000 + seed)
    frames = [f for f, _ in rx_frames.corpus(seed=int(rng.integers(1 << 20)))]
    frames = [frames[i] for i in rng.integers(0, len(frames), int(rng.integers(50, 3000)))]
    if rng.random() < 0.5:
        umem, offs, lens = rx_frames.layout(frames, rng, align_max=int(rng.choice([0, 3, 7, 15])))
        desc = np.zeros(len(frames), dtype=X.DESC_DTYPE)
        desc["addr"], desc["len"] = offs, lens
    else:                                      # one frame per 4096-byte chunk
        n = len(frames)
        desc = np.zeros(n, dtype=X.DESC_DTYPE)
        desc["addr"] = np.arange(n, dtype=np.uint64) * 4096 + 256 + rng.integers(0, 8, n)
        desc["len"] = [len(f) for f in frames]
        umem = np.zeros(n * 4096 + 64, np.uint8)
        for d, f in zip(desc, frames):
            umem[int(d["addr"]):int(d["addr"]) + len(f)] = np.frombuffer(f, np.uint8)
    geometry = [None, *RX_GEOMETRIES][int(rng.integers(len(RX_GEOMETRIES) + 1))]
    flags = int(rng.choice([0, X.F_VERIFY, X.F_VERIFY | X.F_IPHDR]))
    hint = int(rng.choice([0, 100, 1500, 9000]))
    recs, count = run_rx(torch_cuda, engine, umem, desc, flags, hint, geometry)
    exp = oracle.rx_batch(umem, desc, flags)
    bad = np.nonzero((recs.view(np.uint8).reshape(-1, 64) != exp.view(np.uint8).reshape(-1, 64))
                     .any(axis=1))[0]
    assert len(bad) == 0, f"seed {seed}: geometry {geometry} flags {flags:#x} hint {hint}: " \
                          f"records {bad[:8].tolist()}"
    assert count == int((exp["status"] == X.RX_OK).sum())


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_host_path_vs_device(torch_cuda, engine, seed):
    """xcsum_batch_host (staged copies, or zero-copy from a registered UMEM)
    on random batches: the same results as the oracle, and with INPLACE the
    same frame bytes as the device path writes."""
    host_fuzz_case(torch_cuda, engine, seed)


def host_fuzz_case(torch_cuda, engine, seed):
    rng = np.random.default_rng(3000 + seed)
    umem, desc = random_batch(rng)
    mode = MODES[int(rng.integers(len(MODES)))]
    flags = int(rng.choice([0, X.F_INPLACE, X.F_INPLACE | X.F_IPHDR, X.F_VERIFY,
                            X.F_VERIFY | X.F_IPHDR]))
    zerocopy = rng.random() < 0.5
    exp = oracle.batch(umem, desc, mode, flags & ~X.F_INPLACE)
    _, exp_after = run_device(torch_cuda, engine, umem, desc, mode, flags)
    host = umem.copy()
    out = np.full(len(desc), 0x5a5a, dtype=np.uint16)
    if zerocopy:
        host = X.as_umem(host)   # libxudp's UMEM mapping
        engine.register_umem(host)
    try:
        engine.batch_host(host, desc, out, mode, flags | (X.F_ZEROCOPY if zerocopy else 0))
    finally:
        if zerocopy:
            engine.unregister_umem(host)
    bad = np.nonzero(out != exp)[0]
    assert len(bad) == 0, f"seed {seed}: mode {mode} flags {flags:#x} zerocopy {zerocopy}: " \
                          f"frames {bad[:8].tolist()}"
    if not np.array_equal(host, exp_after):
        diff = np.nonzero(host != exp_after)[0]
        starts = desc["addr"].astype(np.int64)
        where = []
        for o in diff[:6].tolist():
            k = int(np.searchsorted(np.sort(starts), o, side="right")) - 1
            a0 = int(np.sort(starts)[k]) if k >= 0 else -1
            where.append(f"byte {o} (frame at {a0} +{o - a0}): host {host[o]} device "
                         f"{exp_after[o]} original {umem[o]}")
        raise AssertionError(f"seed {seed}: {len(diff)} in-place bytes differ "
                             f"(zerocopy {zerocopy}, flags {flags:#x}): " + "; ".join(where))


@pytest.fixture
def fpt_reset(engine):
    """the header kernel's frames per thread back to the default after a test"""
    yield
    engine.set_tuning(X.TUNE_IPHDR_FPT, 4)


@pytest.mark.parametrize("seed", range(48))
def test_fuzz_iphdr_only(torch_cuda, engine, fpt_reset, seed):
    """XCSUM_F_IPHDR_ONLY (libxudp's IPv4 call) on random batches -- IPv6
    and malformed frames mixed in, random phases, layouts and frames per
    thread -- on the device against the oracle (orc_iphdr_only), and through
    xcsum_batch_host (gathered, or in place from a registered UMEM) against
    the device: results and frame bytes.  In place, only iph->check of the
    IPv4 frames the rules accept may change."""
    rng = np.random.default_rng(4000 + seed)
    umem, desc = random_batch(rng)
    mode = int(rng.choice([X.MODE_V4_LEGACY, X.MODE_V4_RFC, X.MODE_AUTO]))
    flags = X.F_IPHDR_ONLY | int(rng.choice([0, X.F_INPLACE, X.F_VERIFY, X.F_VERIFY | X.F_INPLACE]))
    engine.set_tuning(X.TUNE_IPHDR_FPT, int(rng.choice([1, 2, 4, 8])))
    exp = oracle.batch(umem, desc, mode, flags & ~X.F_INPLACE)
    got, after = run_device(torch_cuda, engine, umem, desc, mode, flags)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, f"seed {seed}: mode {mode} flags {flags:#x}: frames {bad[:8].tolist()}"
    changed = set(np.nonzero(after != umem)[0].tolist())
    fields = set()
    for a in desc["addr"].astype(np.int64):
        fields.update((int(a) + 24, int(a) + 25))
    assert changed <= fields
    if not (flags & X.F_INPLACE) or (flags & X.F_VERIFY):
        assert not changed
    zerocopy = rng.random() < 0.5
    host = umem.copy()
    if zerocopy:
        host = X.as_umem(host)   # libxudp's UMEM mapping
        engine.register_umem(host)
    out = np.full(len(desc), 0x5a5a, dtype=np.uint16)
    try:
        engine.batch_host(host, desc, out, mode, flags)
    finally:
        if zerocopy:
            engine.unregister_umem(host)
    assert np.array_equal(out, exp), f"seed {seed}: host path (zerocopy {zerocopy})"
    assert np.array_equal(host, after), f"seed {seed}: host in-place bytes (zerocopy {zerocopy})"
