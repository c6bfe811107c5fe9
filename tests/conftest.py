import json
import os
import sys

if os.environ.get("XCSUM_TEST_NO_THP"):
    # diagnostic: no transparent huge pages in this process
    # (PR_SET_THP_DISABLE = 41), set before the heap grows
    import ctypes
    assert ctypes.CDLL(None, use_errno=True).prctl(41, 1, 0, 0, 0) == 0

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)   # rx_frames, the receive-corpus builder


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size parity (seconds to minutes)")


@pytest.fixture(scope="session")
def golden():
    g = np.load(os.path.join(GOLDEN, "fixtures.npz"))
    return {k: g[k] for k in g.files}


@pytest.fixture(scope="session")
def digests():
    return json.load(open(os.path.join(GOLDEN, "digests.json")))


def h2d(torch, arr, dev):
    """Host array -> device tensor through torch's pinned host memory (cached,
    never returned to the OS).  Test helpers never hand pageable buffers to
    the HIP runtime for DMA: it pins such buffers in place and can reuse that
    pinning for a later buffer at the same addresses after the first one was
    freed -- the likely cause of the two illegal-address faults seen at a
    >= 1 MB pageable device-to-host copy."""
    import numpy as _np
    return torch.from_numpy(_np.ascontiguousarray(arr)).pin_memory().to(dev)


def d2h(t):
    """Device tensor -> numpy array in pinned host memory (see h2d)."""
    import torch
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h.numpy()


def golden_desc(g, sel=None):
    import libxudp_amd as X
    idx = np.arange(len(g["len"])) if sel is None else sel
    d = np.zeros(len(idx), dtype=X.DESC_DTYPE)
    d["addr"] = g["addr"][idx]
    d["len"] = g["len"][idx]
    return d


@pytest.fixture(scope="session")
def engine():
    import libxudp_amd as X
    e = X.Engine(0)
    yield e
    e.close()


@pytest.fixture(autouse=True)
def reg_trace_marker(request):
    """With XCSUM_REG_TRACE=<file> (the library's registration trace,
    DESIGN.md 6), each test's node id goes into the same file before the
    test, so a registration line names the test that made it."""
    path = os.environ.get("XCSUM_REG_TRACE")
    if path:
        with open(path, "a") as f:
            f.write(f"test {request.node.nodeid}\n")
    yield


@pytest.fixture(autouse=True)
def bounds_checked(request):
    """Under the bounds-checked debug build (XCSUM_LIB=libxudp_amd/debug/
    libxcsum.so, make -C libxudp_amd debug) every GPU test ends by reading the
    kernels' violation logs: any load or store outside its frame, stream
    region or result array fails the test that made it."""
    yield
    if "gpu" not in request.keywords or not os.environ.get("XCSUM_LIB"):
        return
    import libxudp_amd as X
    if not X.debug_build():
        return
    count, recs = X.take_bounds()
    assert count == 0, f"{count} out-of-bounds accesses, first: " + "; ".join(
        f"{s}[{i}] addr {a:#x} allowed [{lo:#x}, {hi:#x})" for s, i, a, lo, hi in recs[:4])


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test on a host without a GPU"
    return torch
