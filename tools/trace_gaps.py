#!/usr/bin/env python3
"""Per-dispatch analysis of a rocprofv3 --kernel-trace CSV (kernel_trace.csv): for each kernel,
duration quantiles by phase of the merge loop, and the idle gap in front of each kernel
(previous dispatch's end -> this dispatch's start).  Streams the file; prints a small table.

usage: trace_gaps.py <kernel_trace.csv> [bucket_rounds]
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"bpe::\(anonymous namespace\)::|bpe::", "", name)
    return re.sub(r"\(.*", "", name).replace("void ", "")


def main():
    path = sys.argv[1]
    bucket = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    rows = []
    with open(path) as f:
        r = csv.DictReader(f)
        for d in r:
            rows.append((int(d["Start_Timestamp"]), int(d["End_Timestamp"]), short(d["Kernel_Name"])))
    rows.sort()
    dur = defaultdict(lambda: defaultdict(list))
    gap = defaultdict(lambda: defaultdict(list))
    rnd = -1
    prev_end = None
    for s, e, k in rows:
        if k.startswith("k_merge"):
            rnd += 1
        b = rnd // bucket if rnd >= 0 else -1
        dur[k][b].append((e - s) / 1e3)
        if prev_end is not None:
            g = (s - prev_end) / 1e3
            if 0 <= g < 200:          # larger gaps are host work between batches
                gap[k][b].append(g)
        prev_end = e
    print(f"# {path}: {len(rows)} dispatches, {rnd + 1} k_merge rounds, bucket {bucket} rounds")
    print(f"{'kernel':18s} {'bucket':>6s} {'n':>7s} {'dur_med':>8s} {'dur_mean':>8s} {'dur_p90':>8s} "
          f"{'gap_med':>8s} {'gap_mean':>8s}")
    for k in ("k_merge<unsigned short>", "k_merge<unsigned int>", "k_apply", "k_apply_argmax", "k_argmax"):
        if k not in dur:
            continue
        for b in sorted(dur[k]):
            if b < 0:
                continue
            d = dur[k][b]
            g = gap[k].get(b, [0.0])
            q = statistics.quantiles(d, n=10) if len(d) >= 10 else [max(d)] * 9
            print(f"{k[:18]:18s} {b:6d} {len(d):7d} {statistics.median(d):8.2f} {statistics.fmean(d):8.2f} "
                  f"{q[8]:8.2f} {statistics.median(g):8.2f} {statistics.fmean(g):8.2f}")


if __name__ == "__main__":
    main()
