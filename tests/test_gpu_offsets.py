"""GPU: frames at UMEM offsets across 2 GiB and 4 GiB (a 4.3 GB device
buffer).  The kernels carry UMEM offsets in 64 bits but move them between
lanes as 32-bit halves (v_readlane, ds_bpermute); a sign-extended low half
once broke every offset with bit 31 set (found by the config-5 digest, 37 GB
of UMEM).  Each kernel family sees packed batches straddling both
boundaries, checked against the oracle on the same frames at offset 0."""
import numpy as np
import pytest

import libxudp_amd as X
from conftest import h2d, d2h
import oracle

pytestmark = pytest.mark.gpu

OFFSETS = [(1 << 31) - 5000, (1 << 32) - 3000]
GEOMS = [None, (16, 2, 6), (64, 1, 9), (4, 1, 2)] + X.STREAM_GEOMETRIES[1:2] + (X.SEG_GEOMETRIES + X.SEG_ATOM_GEOMETRIES if X.variants_built() else [])


@pytest.fixture(scope="module")
def big(torch_cuda):
    buf = torch_cuda.zeros((1 << 32) + (64 << 20), dtype=torch_cuda.uint8, device="cuda:0")
    yield buf
    del buf
    torch_cuda.cuda.empty_cache()


def place(torch, big, umem, desc, off):
    big[off:off + len(umem)] = torch.from_numpy(umem).to(big.device)
    d = desc.copy()
    d["addr"] += off
    return torch.from_numpy(d.view(np.uint8)).to(big.device)


@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("sizes", [(0, 64), (1400, 1500), (0, 9000)])
def test_checksum_across_2g_and_4g(torch_cuda, engine, big, geom, sizes):
    umem, desc = X.gen_frames_host(700, 4, sizes[0], sizes[1], seed=sizes[1])
    exp = oracle.batch(umem, desc, X.MODE_V4_LEGACY)
    if geom is not None:
        engine.set_geometry(*geom)
    try:
        for off in OFFSETS:
            d_desc = place(torch_cuda, big, umem, desc, off)
            out = torch_cuda.zeros(len(desc), dtype=torch_cuda.int16, device="cuda:0")
            engine.batch_device(big, d_desc, len(desc), out, X.MODE_V4_LEGACY, 0,
                                int(desc["len"].mean()))
            torch_cuda.cuda.synchronize()
            assert np.array_equal(d2h(out).view(np.uint16), exp), (geom, off)
    finally:
        engine.set_geometry(0)


@pytest.mark.parametrize("geometry", [None, "4,2,1", "32,3,0", "64,9,0", "64,8,3"])
def test_receive_across_2g_and_4g(torch_cuda, engine, big, geometry, monkeypatch):
    umem, desc = X.gen_frames_host(700, 6, 0, 3000, seed=3)
    exp = oracle.rx_batch(umem, desc, X.F_VERIFY)
    if geometry:
        engine.set_tuning(X.TUNE_RX_GEOMETRY, *[int(v) for v in geometry.split(",")])
    try:
        for off in OFFSETS:
            d_desc = place(torch_cuda, big, umem, desc, off)
            msgs = torch_cuda.zeros(len(desc) * 64, dtype=torch_cuda.uint8, device="cuda:0")
            engine.rx_device(big, d_desc, len(desc), msgs, None, X.F_VERIFY, 1500)
            torch_cuda.cuda.synchronize()
            got = d2h(msgs).view(X.RX_MSG_DTYPE)
            # records hold UMEM offsets: compare with the expected ones moved by off
            e = exp.copy()
            e["frame"] += off
            e["body"][e["body"] != 0] += off
            assert np.array_equal(got.view(np.uint8), e.view(np.uint8)), (geometry, off)
    finally:
        engine.set_tuning(X.TUNE_RX_GEOMETRY, 0)


@pytest.mark.parametrize("inplace", [False, True])
def test_build_across_2g_and_4g(torch_cuda, engine, big, inplace):
    """xcsum_build_device into 4096-byte slots around 2 GiB and 4 GiB."""
    torch = torch_cuda
    FRAME, DATA_OFF = 4096, 384
    rng = np.random.default_rng(21)
    slots = np.concatenate([np.arange((1 << 19) - 12, (1 << 19) + 12),
                            np.arange((1 << 20) - 12, (1 << 20) + 12)]).astype(np.uint32)
    n = len(slots)
    r = dict(smac=bytes(range(6)), dmac=bytes(range(6, 12)), saddr=bytes([10, 0, 0, 1]),
             daddr=bytes([10, 0, 0, 2]), sport=1234, dport=5678)
    route = X.make_route(4, r["smac"], r["dmac"], r["saddr"], r["sport"], r["daddr"], r["dport"])
    pays = [rng.integers(0, 256, int(L), dtype=np.uint8) for L in rng.integers(0, 3000, n)]
    msgs = np.zeros(n, dtype=X.MSG_DTYPE)
    msgs["len"] = [len(p) for p in pays]
    msgs["slot"] = slots
    if inplace:
        for s, p in zip(slots, pays):
            o = int(s) * FRAME + DATA_OFF
            big[o:o + len(p)] = torch.from_numpy(p).to(big.device)
        d_src = torch.zeros(16, dtype=torch.uint8, device="cuda:0")
    else:
        src = np.concatenate(pays + [np.zeros(16, np.uint8)])
        msgs["src"] = np.concatenate([[0], np.cumsum([len(p) for p in pays])[:-1]])
        d_src = h2d(torch, src, "cuda:0")
    d_msgs = h2d(torch, msgs.view(np.uint8), "cuda:0")
    d_desc = torch.zeros(n * 16, dtype=torch.uint8, device="cuda:0")
    d_out = torch.zeros(n, dtype=torch.int16, device="cuda:0")
    engine.build_device(route, d_src, d_msgs, n, big, FRAME, DATA_OFF, d_desc, d_out,
                        X.F_BUILD_INPLACE if inplace else 0, 1500)
    torch.cuda.synchronize()
    desc = d2h(d_desc).view(X.DESC_DTYPE)
    for i, p in enumerate(pays):
        exp = oracle.build_frame(p.tobytes(), 4, r["smac"], r["dmac"], r["saddr"], r["sport"],
                                 r["daddr"], r["dport"], False)
        eth = int(slots[i]) * FRAME + DATA_OFF - 42
        assert int(desc["addr"][i]) == eth and int(desc["len"][i]) == len(exp)
        got = d2h(big[eth:eth + len(exp)])
        assert np.array_equal(got, exp), (i, int(slots[i]))
