#!/usr/bin/env python3
"""Does xudp's UMEM slot layout (one ~1.5 KB frame at a fixed offset in each
4096-B chunk) cost HBM read rate by itself, independent of the
checksum kernel?  Reads only the spans, 1M slots, with (a) packed spans,
(b) the fixed xudp offset, (c) offsets rotated across the slot, (d) 2048-B
slots.  One JSON line per case.  Bounds checked on the host: every read ends
inside the buffer."""
import argparse
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true",
                    help="config 3's 80-B spans (64-B payloads) instead of config 2's")
    args = ap.parse_args()
    L = ctypes.CDLL(os.path.join(HERE, "libhbmprobe.so"))
    L.probe_slot_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                  ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_void_p]
    dev = torch.device("cuda:0")
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nslots = 1 << 20
    # a config-2 span (94 x 16 B) or a config-3 one: 80 B at eth+26 = F+368,
    # two 64-B lines per 4096-B slot
    span16 = 5 if args.small else 1488 // 16 + 1
    buf = torch.zeros((nslots * 4096 + 4096,), dtype=torch.uint8, device=dev)
    out = torch.empty(cus * 16 * 256, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    # (name, slot bytes, offset, rot16, nrot, perm_mul, perm_shift)
    cases = [("packed", span16 * 16, 0, 0, 0, 0, 0),
             ("xudp_4096_fixed_off_368", 4096, 368, 0, 0, 0, 0),
             ("4096_rotated_off", 4096, 0, 37, (4096 - span16 * 16) // 16, 0, 0),
             ("4096_fixed_scattered_slots", 4096, 368, 0, 0, 0x9E3779B1, 0),
             ("4096_fixed_scattered_groups16", 4096, 368, 0, 0, 0x9E3779B1, 4),
             ("4096_fixed_scattered_groups256", 4096, 368, 0, 0, 0x9E3779B1, 8),
             ("xudp_2048_fixed_off_368", 2048, 368, 0, 0, 0, 0)]
    if args.small:
        cases += [("4096_fixed_scattered_groups64", 4096, 368, 0, 0, 0x9E3779B1, 6),
                  ("1024_fixed_off_368", 1024, 368, 0, 0, 0, 0),
                  ("512_fixed_off_368", 512, 368, 0, 0, 0, 0)]
    else:
        cases += [  # 16-byte loads at 8/4/2-byte aligned addresses (packed 1520-B slots)
             ("packed1520_align16", 1520, 0, 0, 0, 0, 0),
             ("packed1520_align8", 1520, 8, 0, 0, 0, 0),
             ("packed1520_align4", 1520, 4, 0, 0, 0, 0),
             ("packed1520_align2", 1520, 2, 0, 0, 0, 0),
             ("2048_rotated_off", 2048, 0, 7, (2048 - span16 * 16) // 16, 0, 0)]
    for name, slot, off0, rot, nrot, pm, ps in cases:
        assert (nslots - 1) * slot + off0 + max(nrot - 1, 0) * 16 + span16 * 16 <= buf.numel()
        lines = span16 * 16 if slot == span16 * 16 else \
            64 * ((off0 % 64 + span16 * 16 + 63) // 64)
        for per_cu in ((4, 8, 16) if args.small else (4, 8)):
            ts = []
            for _ in range(12):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                assert L.probe_slot_read(buf.data_ptr(), nslots, slot, span16, off0, rot, nrot,
                                         pm, ps, out.data_ptr(), cus * per_cu, s.cuda_stream) == 0
                b.record(s)
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b))
            t = sorted(ts)[len(ts) // 2]
            print(json.dumps({"case": name, "slot_bytes": slot, "span_bytes": span16 * 16,
                              "blocks_per_cu": per_cu, "ms": round(t, 4),
                              "GBps": round(nslots * span16 * 16 / (t * 1e-3) / 1e9, 1),
                              # 64-byte lines the spans touch (= HBM bytes)
                              "line_GBps": round(nslots * lines / (t * 1e-3) / 1e9, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
