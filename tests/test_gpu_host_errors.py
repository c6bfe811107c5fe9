"""GPU: host entry points leave nothing in flight when they fail.

xcsum_batch_host / xcsum_rx_host work in chunks of <= 65,536 frames and
<= 32 MiB of UMEM, two chunks in flight.  A chunk that fails its checks
(here: a descriptor longer than a chunk may be) used to return at once while
the previous chunk's copy and kernel still read the caller's UMEM -- a caller
that unmaps it right after the error return would have the GPU read unmapped
memory ("What's weak" #2).  Now every error return drains the
context's streams first: xcsum_ctx_pending() is 0 and the UMEM can be
unregistered and unmapped immediately.

Also: the replay of the host-path fuzz sequence seeds 15 -> 16 -> 17 (the
calls that preceded round 2's one illegal-address fault, s29) in one test,
with the same checks after every call."""
import mmap

import numpy as np
import pytest

import libxudp_amd as X
import oracle

pytestmark = pytest.mark.gpu

N_OK = 20000          # MTU frames of the first chunk: 30 MB < 32 MiB


def rc_of(fn, *args):
    """fn(*args)'s error code (0: none), keeping no traceback: its frames
    would hold the UMEM array and keep the mapping exported"""
    try:
        fn(*args)
    except X.XcsumError as e:
        return e.rc
    return 0


def umem_with_bad_tail(buf):
    """N_OK packed MTU frames in `buf`, then one descriptor of 40 MB (longer
    than a chunk may be: the second chunk's check fails)."""
    desc, nbytes = X.gen_layout(N_OK, 4, 1472, 1472, seed=77)
    arr = np.frombuffer(buf, dtype=np.uint8)
    X.gen_fill_host(arr, desc, 4, seed=77)
    bad = np.zeros(1, dtype=X.DESC_DTYPE)
    bad["addr"], bad["len"] = 0, 40 << 20
    return np.concatenate([desc, bad]), arr


@pytest.mark.parametrize("registered", [False, True])
@pytest.mark.parametrize("flags", [0, X.F_INPLACE | X.F_IPHDR])
def test_batch_host_error_leaves_nothing_in_flight(engine, registered, flags):
    size = 48 << 20
    buf = mmap.mmap(-1, size)
    desc, arr = umem_with_bad_tail(buf)
    out = np.zeros(len(desc), dtype=np.uint16)
    if registered:
        engine.register_umem(arr)
    try:
        assert rc_of(engine.batch_host, arr, desc, out, X.MODE_V4_RFC, flags) == -X.ERR_INVAL
        assert engine.pending() == 0
    finally:
        if registered:
            engine.unregister_umem(arr)
    del arr
    buf.close()                                   # munmap right after the error
    # the context still works, on fresh memory
    umem, d = X.gen_frames_host(1000, 4, 1472, seed=5)
    out = np.zeros(len(d), dtype=np.uint16)
    engine.batch_host(umem, d, out, X.MODE_V4_RFC)
    assert np.array_equal(out, oracle.batch(umem, d, X.MODE_V4_RFC))
    assert engine.pending() == 0


@pytest.mark.parametrize("registered", [False, True])
def test_rx_host_error_leaves_nothing_in_flight(engine, registered):
    size = 48 << 20
    buf = mmap.mmap(-1, size)
    desc, arr = umem_with_bad_tail(buf)
    msgs = np.zeros(len(desc), dtype=X.RX_MSG_DTYPE)
    if registered:
        engine.register_umem(arr)
    try:
        assert rc_of(engine.rx_host, arr, desc, msgs, X.F_VERIFY) == -X.ERR_INVAL
        assert engine.pending() == 0
    finally:
        if registered:
            engine.unregister_umem(arr)
    del arr
    buf.close()


def test_s29_host_path_sequence_replay(torch_cuda, engine):
    """Round 2's one GPU fault (s29) surfaced in test_fuzz_host_path_vs_device
    [17] right after [16]; the exact inputs are deterministic (seeds 3015..3017).
    Replayed here in order, each call checked against the oracle, nothing in
    flight after each, and a device synchronise after each."""
    from test_gpu_fuzz import host_fuzz_case
    for seed in (15, 16, 17):
        host_fuzz_case(torch_cuda, engine, seed)
        assert engine.pending() == 0
        torch_cuda.cuda.synchronize()


@pytest.mark.skipif(not X.debug_build(), reason="bounds-checked debug build only (XCSUM_LIB)")
def test_debug_bounds_positive_control(torch_cuda):
    """The debug build's log -> xcsum_debug_bounds() path reports a failing
    check (a kernel that only evaluates one out-of-range address)."""
    X.take_bounds()
    assert X.lib().xcsum_debug_bounds_selftest(1234) == 0
    count, recs = X.take_bounds()
    assert count == 1 and recs[0][:2] == ("gen_store", 1234), recs
