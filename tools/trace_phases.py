#!/usr/bin/env python3
"""Split a rocprofv3 --kernel-trace CSV of `bench.py --steps K --warmup W`
into its phases for one kernel: W eager warm-up launches, the first (warm)
graph replay of K launches, and the timed replay of K launches.  The timed
replay's average is the number to compare with bench.py's live HIP-event
kernel_ms (the --stats average also counts the warm-up and the first replay).

Usage: python tools/trace_phases.py <run_kernel_trace.csv> --steps K --warmup W
       [--kernel csum_kernel]"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--kernel", default="csum_kernel")
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if args.kernel in r["Kernel_Name"]]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    w, k = args.warmup, args.steps
    out = {"kernel": rows[0]["Kernel_Name"] if rows else None, "launches": len(d),
           "all_avg_us": round(statistics.mean(d), 2) if d else None,
           "warmup_avg_us": round(statistics.mean(d[:w]), 2) if d[:w] else None,
           "first_replay_avg_us": round(statistics.mean(d[w:w + k]), 2) if d[w:w + k] else None,
           "timed_replay_avg_us": round(statistics.mean(d[w + k:w + 2 * k]), 2)
           if d[w + k:w + 2 * k] else None,
           "timed_replay_min_us": round(min(d[w + k:w + 2 * k]), 2) if d[w + k:w + 2 * k] else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
