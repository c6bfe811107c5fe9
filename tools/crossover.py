#!/usr/bin/env python3
"""Host-core side of the small-batch crossover: ns per frame
of the reference's own xudp_packet_udp() (packet.c:156-194, compiled in place
by oracle/Makefile into oracle/_ref) on one thread, over 100-frame batches in
xudp's 4096-byte slots, for IPv4 (headers + xudp_checksum_half) and IPv6
(headers + udp_csum6 over the whole datagram) at several payload sizes.
CPU-only; prints one JSON line.  Test/measurement infrastructure: loads
oracle/_ref, never the product."""
import ctypes
import json
import os
import platform

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libxudpref.so"))
    fn = L.ref_packet_udp_timed
    fn.restype = ctypes.c_double
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    n = 100
    umem = np.random.default_rng(1).integers(0, 256, n * 4096, dtype=np.uint8)
    res = {}
    for fam in (4, 6):
        for pl in (0, 64, 512, 1472):
            reps = 20000 if fam == 4 else max(200, 2000000 // (pl + 64))
            fn(umem.ctypes.data, n, fam, pl, max(1, reps // 10))   # warm
            best = min(fn(umem.ctypes.data, n, fam, pl, reps) for _ in range(3))
            res[f"v{fam}_{pl}"] = round(best / (reps * n) * 1e9, 2)
    cpu = "?"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    print(json.dumps({"what": "ns per frame of the reference xudp_packet_udp() on one thread, "
                              "100-frame batches in 4096-B slots (min of 3 timed runs)",
                      "cpu": cpu, "host": platform.node(), "ns_per_frame": res}), flush=True)


if __name__ == "__main__":
    main()
