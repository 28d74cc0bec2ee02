"""Per-trip kernel durations from a rocprofv3 --kernel-trace database (second training of a bench run)."""
import sqlite3, sys
import numpy as np
c = sqlite3.connect(sys.argv[1])
for kn in ["k_apply_batch", "k_merge_batch", "k_select"]:
    d = np.array([r[0] for r in c.execute(f"select duration from kernels where name like '%{kn}%' order by start")]) / 1e3
    d = d[len(d) // 2:]
    if not len(d):
        continue
    dec = np.array_split(d, 10)
    print(f"{kn:14s} n={len(d)} mean {d.mean():.1f} p50 {np.percentile(d, 50):.1f} p90 {np.percentile(d, 90):.1f} "
          f"p99 {np.percentile(d, 99):.1f} | deciles " + " ".join("%.1f" % x.mean() for x in dec))
