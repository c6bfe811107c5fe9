"""GPU: the two in-place schedules of xcsum_batch_device (xcsum_ctx_set_inplace).

XCSUM_F_INPLACE stores udp->check (and, with XCSUM_F_IPHDR, iph->check) into
every frame, as libxudp's TX path does before it publishes a frame
(xudp/packet.c:156-194, tx.c:696-726).  FUSED stores each field from the
checksum pass; TWO_PASS runs the checksum pass into a result array and stores
the fields in a second launch (csrc/xcsum_scatter.hip).  Both must leave
byte-identical frames, equal to the reference's values (golden fixtures,
oracle), touch nothing but the check fields of well-formed frames, count
malformed frames once, and work on any stream, under graph capture and with
or without a result array."""
import numpy as np
import pytest

import libxudp_amd as X
import oracle
from conftest import golden_desc, h2d, d2h
from test_gpu_fuzz import random_batch, MODES
from test_gpu_parity import FEATURE_GEOMS, geometry, run_device

pytestmark = pytest.mark.gpu

SCHEDULES = {"fused": X.INPLACE_FUSED, "two_pass": X.INPLACE_TWO_PASS}


def expected_frames(umem, desc, mode, flags):
    """The frames after an in-place pass: the oracle's results stored at the
    check fields of every well-formed frame (the reference's values,
    packet.c:23 CSUM_MANGLED_0 included), every other byte unchanged."""
    after = umem.copy()
    res = oracle.batch(umem, desc, mode, flags & ~X.F_INPLACE)
    for i, d in enumerate(desc):
        a, ln = int(d["addr"]), int(d["len"])
        fam = 6 if mode == X.MODE_V6 else 4
        if mode == X.MODE_AUTO:
            proto = (int(umem[a + 12]) << 8 | int(umem[a + 13])) if ln >= 14 else 0
            fam = 4 if proto == 0x0800 else 6 if proto == 0x86DD else 0
        hdr = 54 if fam == 6 else 34
        if fam == 0 or ln < hdr + 8 or ln - hdr > 65535:
            continue
        off = 60 if fam == 6 else 40
        after[a + off:a + off + 2] = np.array([res[i]], "<u2").view(np.uint8)
        if fam == 4 and flags & X.F_IPHDR:
            ipc = oracle.ip_header_rfc(umem[a:a + ln])
            after[a + 24:a + 26] = np.array([ipc], "<u2").view(np.uint8)
    return res, after


@pytest.mark.parametrize("sched", sorted(SCHEDULES))
@pytest.mark.parametrize("geom", FEATURE_GEOMS)
@pytest.mark.parametrize("flags", [X.F_INPLACE, X.F_INPLACE | X.F_IPHDR,
                                   X.F_INPLACE | X.F_IPHDR | X.F_V4_RFC])
@pytest.mark.parametrize("out", [True, False])
def test_golden_schedules(torch_cuda, engine, golden, sched, geom, flags, out):
    """Every golden frame (both families, AUTO): the reference's udp->check
    and iph->check in place, nothing else changed, with and without d_out."""
    umem = golden["umem"]
    desc = golden_desc(golden)
    engine.set_inplace(SCHEDULES[sched])
    try:
        with geometry(engine, geom):
            got, after = run_device(torch_cuda, engine, umem.copy(), desc, X.MODE_AUTO, flags,
                                    out=out)
    finally:
        engine.set_inplace(X.INPLACE_AUTO)
    fam = golden["family"]
    col = "exp_rfc" if flags & X.F_V4_RFC else "exp_legacy"
    exp = np.where(fam == 6, golden["exp_v6"], golden[col])
    if out:
        assert np.array_equal(got, exp)
    res, exp_after = expected_frames(umem, desc, X.MODE_AUTO, flags)
    assert np.array_equal(res, exp)
    assert np.array_equal(after, exp_after)


@pytest.mark.parametrize("block", [0, 32, 64])
@pytest.mark.parametrize("layout", ["packed1", "packed8", "slots"])
def test_two_pass_store_widths(torch_cuda, monkeypatch, block, layout):
    """The second pass's store widths (XCSUM_TUNE_INPLACE_BLOCK): 2-byte stores,
    or the whole 32-B sector / 64-B line holding a field, read and patched
    when it lies inside the frame.  Frames at every byte phase, packed (the
    blocks of neighbouring frames' fields meet) and in xudp's slots: the
    reference's fields in place and not one other byte changed."""
    e = X.Engine(0)
    e.set_tuning(X.TUNE_INPLACE_BLOCK, block)
    try:
        e.set_inplace(X.INPLACE_TWO_PASS)
        for fam, mode in ((4, X.MODE_V4_RFC), (6, X.MODE_V6), (4, X.MODE_AUTO)):
            kw = {"packed1": dict(align=1), "packed8": dict(align=8),
                  "slots": dict(stride=4096, offset=342 if fam == 4 else 322)}[layout]
            umem, desc = X.gen_frames_host(2500, fam, 0, 1472, seed=70 + fam + block, **kw)
            for flags in (X.F_INPLACE, X.F_INPLACE | X.F_IPHDR):
                res, exp_after = expected_frames(umem, desc, mode, flags)
                got, after = run_device(torch_cuda, e, umem.copy(), desc, mode, flags)
                assert np.array_equal(got, res)
                diff = np.nonzero(after != exp_after)[0]
                assert len(diff) == 0, f"{fam} {mode} {flags:#x}: {len(diff)} bytes, {diff[:4]}"
    finally:
        e.close()


@pytest.mark.parametrize("block", [0, 32, 64])
def test_r04d_field_at_block_end(torch_cuda, monkeypatch, block):
    """profiles/r04/fault/r04d_pytest_gpu_thp_off_scatter_bug.log, pinned: the
    batch of test_fuzz_host_path_vs_device[3] (seed 3003 draws: odd-address
    frames, flags INPLACE | IPHDR), whose udp->check high byte (eth+41) fell
    on a 32-byte boundary in 193 frames.  The round-4 work-in-progress second
    pass patched such a field into the block holding its first byte and lost
    the second; store_block (xcsum_scatter.hip) now sends any field that
    reaches past its block to the 2-byte stores.  Both schedules, every
    store width: the reference's fields, no other byte changed."""
    rng = np.random.default_rng(3000 + 3)
    umem, desc = random_batch(rng)
    mode = MODES[int(rng.integers(len(MODES)))]
    flags = int(rng.choice([0, X.F_INPLACE, X.F_INPLACE | X.F_IPHDR, X.F_VERIFY,
                            X.F_VERIFY | X.F_IPHDR]))
    assert flags == X.F_INPLACE | X.F_IPHDR
    straddle = ((desc["addr"].astype(np.int64) + 40) % 32 == 31).sum()
    assert straddle >= 100, straddle               # the r04d shape is in the batch
    res, exp_after = expected_frames(umem, desc, mode, flags)
    monkeypatch.setenv("XCSUM_INPLACE_BLOCK", str(block))
    e = X.Engine(0)
    monkeypatch.delenv("XCSUM_INPLACE_BLOCK")
    try:
        for sched in ("two_pass", "fused"):
            e.set_inplace(SCHEDULES[sched])
            got, after = run_device(torch_cuda, e, umem.copy(), desc, mode, flags)
            assert np.array_equal(got, res), sched
            diff = np.nonzero(after != exp_after)[0]
            assert len(diff) == 0, f"{sched}: {len(diff)} bytes differ, first {diff[:4]}"
    finally:
        e.close()


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_schedules_identical(torch_cuda, engine, seed):
    """Random batches (mixed sizes, alignments, shuffled and malformed
    descriptors): both schedules leave byte-identical frames and results,
    equal to the oracle's, and count the same malformed frames."""
    rng = np.random.default_rng(5000 + seed)
    umem, desc = random_batch(rng)
    mode = MODES[int(rng.integers(len(MODES)))]
    flags = X.F_INPLACE | int(rng.choice([0, X.F_IPHDR, X.F_IPHDR | X.F_V4_RFC]))
    hint = int(rng.choice([0, 64, 1500, 9000]))
    res_exp, after_exp = expected_frames(umem, desc, mode, flags)
    for sched in ("fused", "two_pass"):
        engine.set_inplace(SCHEDULES[sched])
        try:
            engine.take_errors()
            got, after = run_device(torch_cuda, engine, umem.copy(), desc, mode, flags, hint)
            errs = engine.take_errors()
        finally:
            engine.set_inplace(X.INPLACE_AUTO)
        assert np.array_equal(got, res_exp), f"seed {seed} {sched}"
        diff = np.nonzero(after != after_exp)[0]
        assert len(diff) == 0, f"seed {seed} {sched}: {len(diff)} bytes differ, first {diff[:4]}"
        if sched == "fused":
            errs_fused = errs
        else:
            assert errs == errs_fused


@pytest.mark.parametrize("with_out", [False, True])
def test_two_pass_under_graph_capture(torch_cuda, with_out):
    """A TWO_PASS context captured into a graph, with no scratch yet and after
    an eager call made one; then an eager call with 20x the frames (the
    scratch is freed and regrown) and the graph replayed again.  A capture
    that needs the scratch (no d_out, or IPHDR) runs FUSED, so the replay
    touches no scratch; without IPHDR and with the caller's d_out the two
    passes are captured as they are.  Every replay writes the reference's
    fields (a graph that kept the old scratch pointer wrote into
    freed memory after the regrowth)."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    flags = X.F_INPLACE | (0 if with_out else X.F_IPHDR)
    umem, desc = X.gen_frames_host(5000, 4, 0, 1472, seed=31, align=8)
    exp_out, exp_after = expected_frames(umem, desc, X.MODE_V4_LEGACY, flags)
    big_u, big_d = X.gen_frames_host(100000, 4, 0, 200, seed=32, align=8)
    _, big_exp = expected_frames(big_u, big_d, X.MODE_V4_LEGACY, X.F_INPLACE | X.F_IPHDR)
    d_desc = h2d(torch, desc.view(np.uint8), dev)
    d_big_desc = h2d(torch, big_d.view(np.uint8), dev)
    for eager_first in (False, True):
        e = X.Engine(0)
        e.set_inplace(X.INPLACE_TWO_PASS)
        try:
            d_umem = h2d(torch, umem, dev)
            d_out = torch.zeros(len(desc), dtype=torch.int16, device=dev) if with_out else None
            s = torch.cuda.Stream(dev)
            if eager_first:
                scratch = h2d(torch, umem, dev)
                e.batch_device(scratch, d_desc, len(desc), None, X.MODE_V4_LEGACY,
                               X.F_INPLACE | X.F_IPHDR, 1500, stream=s.cuda_stream)
                torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.graph(g, stream=s):
                e.batch_device(d_umem, d_desc, len(desc), d_out, X.MODE_V4_LEGACY, flags, 1500,
                               stream=torch.cuda.current_stream(dev).cuda_stream)
            g.replay()
            torch.cuda.synchronize(dev)
            assert np.array_equal(d2h(d_umem), exp_after), f"eager_first={eager_first}"
            # an eager call that regrows the scratch, then the graph again on
            # fresh frames
            d_big = h2d(torch, big_u, dev)
            e.batch_device(d_big, d_big_desc, len(big_d), None, X.MODE_V4_LEGACY,
                           X.F_INPLACE | X.F_IPHDR, 200, stream=s.cuda_stream)
            d_umem.copy_(h2d(torch, umem, dev))
            torch.cuda.synchronize(dev)
            g.replay()
            torch.cuda.synchronize(dev)
            assert np.array_equal(d2h(d_umem), exp_after), f"regrown, eager_first={eager_first}"
            if with_out:
                assert np.array_equal(d2h(d_out).view(np.uint16), exp_out)
            assert np.array_equal(d2h(d_big), big_exp)
        finally:
            e.close()


def test_two_pass_alternating_streams(torch_cuda, engine):
    """One context's in-place calls on two streams, back to back without a
    host wait: the shared scratch is ordered through the context's event, so
    every call writes its own frames' values."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    engine.set_inplace(X.INPLACE_TWO_PASS)
    try:
        batches = []
        for k in range(6):
            umem, desc = X.gen_frames_host(3000 + 500 * k, 6 if k % 2 else 4, 0, 1472,
                                           seed=40 + k, align=8)
            mode = X.MODE_V6 if k % 2 else X.MODE_V4_RFC
            _, exp_after = expected_frames(umem, desc, mode, X.F_INPLACE | X.F_IPHDR)
            batches.append((h2d(torch, umem, dev), h2d(torch, desc.view(np.uint8), dev),
                            len(desc), mode, exp_after))
        streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        torch.cuda.synchronize(dev)
        for k, (du, dd, n, mode, _) in enumerate(batches):
            engine.batch_device(du, dd, n, None, mode, X.F_INPLACE | X.F_IPHDR, 1500,
                                stream=streams[k % 2].cuda_stream)
        torch.cuda.synchronize(dev)
        for k, (du, _, _, _, exp_after) in enumerate(batches):
            assert np.array_equal(d2h(du), exp_after), k
    finally:
        engine.set_inplace(X.INPLACE_AUTO)
