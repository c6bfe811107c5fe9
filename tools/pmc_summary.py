#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs for the checksum kernel into
profiles/pmc_config<C>.json (read by bench.py for roofline.traffic), keyed by
the SHA-256 prefix of that kernel's machine code in the profiled library
(bench.kernel_sha16): bench.py reports the counters only while the timed
kernel's code is the same.

HBM bytes per launch follow MI355X_MICROARCH.md 'HBM' / cdna_hip_programming.md
section 7: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts
exactly half the bytes of a wide coalesced streaming read, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
The two counters come from separate --pmc passes (they cannot share one).

Usage: python tools/pmc_summary.py --config 2 --fetch <csv> --write <csv>
           --alg-bytes <per launch> [--out profiles/pmc_config2.json]
"""
import argparse
import csv
import json
import os
import re
import statistics

# the checksum kernels: csum_kernel<G,U,K,FEAT>, csum_kernel_tl<...>,
# csum_stream_kernel<KC>, csum_seg_kernel<D>, iphdr_kernel<FPT> (XCSUM_F_IPHDR_ONLY)
KERNEL = re.compile(r"csum_(stream_|seg_)?kernel|iphdr_kernel")


names = set()


def counter_values(path, name):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if not KERNEL.search(row.get("Kernel_Name", "")):
                continue
            names.add(row["Kernel_Name"])
            if row.get("Counter_Name") != name:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--alg-bytes", type=float, required=True)
    ap.add_argument("--out", default="")
    ap.add_argument("--flags", type=lambda v: int(v, 0), default=0,
                    help="the bench's XCSUM_F_* flags (file name tag _f<hex>)")
    ap.add_argument("--layout", default="packed", help="bench --layout (file name tag _umem)")
    ap.add_argument("--lib-sha", default="",
                    help="SHA-256 prefix of the profiled libxcsum.so's device code "
                         "(bench.py lib_sha16: its .hip_fatbin section), for the record")
    args = ap.parse_args()
    fetch = counter_values(args.fetch, "FETCH_SIZE")
    write = counter_values(args.write, "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit("no csum_kernel counter rows found")
    f_kib = statistics.median(fetch)
    w_kib = statistics.median(write)
    hbm = (2 * f_kib + w_kib) * 1024
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench   # noqa: E402  (kernel_sha16: the counted kernel's machine code)
    kern = sorted(names)
    ksha = bench.kernel_sha16(kern[0]) if len(kern) == 1 else None
    rec = {"config": args.config, "kernel": kern, "dispatches": [len(fetch), len(write)],
           "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib,
           "hbm_bytes_per_launch": round(hbm), "alg_bytes_per_launch": args.alg_bytes,
           "traffic_over_alg": round(hbm / args.alg_bytes, 4),
           "flags": args.flags, "layout": args.layout, "lib_sha16": args.lib_sha or None,
           "kernel_sha16": ksha,
           "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024  (gfx950 FETCH_SIZE = half of "
                      "wide streaming read bytes, MI355X_MICROARCH.md HBM)"}
    out = args.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
        __file__))), "profiles", "r05",
        f"pmc_config{args.config}{'_umem' if args.layout == 'umem' else ''}"
        f"{'_f%x' % args.flags if args.flags else ''}.json")
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
