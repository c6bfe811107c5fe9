#!/usr/bin/env python3
"""Read+write ceiling for the build kernel's copy modes: a device-to-device
copy of the same byte count (1M x 1472 B payloads -> 1M x 1536 B of slot
writes, ~3.1 GB moved per pass) with torch's copy kernel, and a plain
streaming read of the same source for comparison.  Timing only."""
import json
import sys

import numpy as np
import torch


def main():
    dev = torch.device("cuda:0")
    n = 1 << 20
    src = torch.randint(0, 255, (n * 1472,), dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    s = torch.cuda.current_stream(dev)

    def timed(fn, reps=30):
        for _ in range(10):
            fn()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(reps)]
        for e0, e1 in evs:
            e0.record(s)
            fn()
            e1.record(s)
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in evs]))

    t = timed(lambda: dst.copy_(src))
    moved = 2 * src.numel()
    print(json.dumps({"what": "d2d copy", "bytes_moved": moved, "ms": round(t, 4),
                      "GBps": round(moved / t / 1e6, 1)}), flush=True)
    v = src.view(torch.int64)
    t = timed(lambda: v.sum())
    print(json.dumps({"what": "stream read (sum)", "bytes_moved": src.numel(), "ms": round(t, 4),
                      "GBps": round(src.numel() / t / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
