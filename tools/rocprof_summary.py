#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats output (rocpd SQLite .db or kernel_stats.csv)
into a plain-text table: kernel, calls, total ms, average us, share."""
import csv
import pathlib
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"bpe::\(anonymous namespace\)::|bpe::", "", name)
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")


def rows_from(path: pathlib.Path):
    if path.suffix == ".db":
        c = sqlite3.connect(str(path))
        for name, calls, total, avg, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            # the rocpd top_kernels view reports microseconds
            yield short(name), int(calls), total / 1e3, avg, pct
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield (short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6,
                       float(r["AverageNs"]) / 1e3, float(r["Percentage"]))


def main():
    path = pathlib.Path(sys.argv[1])
    print(f"# rocprofv3 kernel summary of {path.name}")
    print(f"{'kernel':40s} {'calls':>8s} {'total_ms':>10s} {'avg_us':>10s} {'share%':>7s}")
    for name, calls, tot, avg, pct in rows_from(path):
        print(f"{name[:40]:40s} {calls:8d} {tot:10.3f} {avg:10.3f} {pct:7.2f}")


if __name__ == "__main__":
    main()
