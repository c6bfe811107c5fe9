#!/usr/bin/env python3
"""Diagnostic (round 3): does the HIP runtime pin pageable host
buffers in place for the copies the tests and the host path make?  Run under
AMD_LOG_LEVEL=4; the runtime's copy path logs 'HSA Copy Using Pinned resource'
when it pins the caller's pages instead of staging.  Prints one marker line
before each copy so the log can be split.  Touches only valid memory."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import libxudp_amd as X  # noqa: E402

dev = torch.device("cuda:0")
for mb in (0.25, 1.5, 4, 16):
    n = int(mb * (1 << 20))
    a = np.random.default_rng(1).integers(0, 255, n, dtype=np.uint8)
    print(f"=== MARK h2d pageable {mb} MB", file=sys.stderr, flush=True)
    d = torch.from_numpy(a).to(dev)
    torch.cuda.synchronize()
    print(f"=== MARK d2h pageable {mb} MB", file=sys.stderr, flush=True)
    b = d.cpu().numpy()
    assert np.array_equal(a, b)
    del d, b
eng = X.Engine(0)
umem, desc = X.gen_frames_host(6000, 4, 1472, seed=3)
out = np.zeros(len(desc), dtype=np.uint16)
print(f"=== MARK batch_host pageable {umem.nbytes / 2**20:.1f} MB", file=sys.stderr, flush=True)
eng.batch_host(umem, desc, out, X.MODE_V4_RFC)
print("=== MARK end", file=sys.stderr, flush=True)
eng.close()
print("diag ok")
