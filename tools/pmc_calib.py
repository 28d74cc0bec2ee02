#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE (KB) of tools/microbench/pmc_calib.hip's kernels over the bytes they
touch: streaming kernels against their buffer size, random ones against 64 B and 128 B per distinct
line.  usage: pmc_calib.py <fetch csv> <write csv>"""
import csv
import re
import sys
from collections import defaultdict

KB = 1024
BIG = 4 << 30
LINES = 16 << 20


def per_kernel(path, counter):
    tot = defaultdict(float)
    with open(path) as f:
        for d in csv.DictReader(f):
            if d.get("Counter_Name") == counter:
                k = re.sub(r"\(.*", "", d["Kernel_Name"]).replace("void ", "")
                tot[k] += float(d["Counter_Value"]) * KB
    return tot


def main():
    f, w = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    known = {"c_read16": BIG, "c_read4": BIG, "c_write16": BIG, "c_write4": BIG, "c_write2": BIG}
    lines = {"c_gather<unsigned short>": LINES, "c_gather<unsigned int>": LINES,
             "c_gather<unsigned long>": LINES, "c_gather64": LINES // 16, "c_scatter4": LINES,
             "c_atomic4": LINES}
    print(f"{'kernel':28s} {'FETCH_SIZE B':>14s} {'WRITE_SIZE B':>14s}  ratios")
    for k in sorted(set(f) | set(w)):
        fb, wb = f.get(k, 0.0), w.get(k, 0.0)
        if k in known:
            r = f"fetch/bytes {fb / known[k]:.3f}  write/bytes {wb / known[k]:.3f}"
        elif k in lines:
            n = lines[k]
            r = (f"fetch per line {fb / n:.1f} B  write per line {wb / n:.1f} B  (lines {n})")
        else:
            r = ""
        print(f"{k:28s} {fb:14.0f} {wb:14.0f}  {r}")


if __name__ == "__main__":
    main()
