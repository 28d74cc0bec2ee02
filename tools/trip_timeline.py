#!/usr/bin/env python3
"""Per-trip timeline of the merge loop from a rocprofv3 --kernel-trace database (rocpd .db):
k_select -> k_merge_batch -> k_apply_batch, each kernel's duration and the idle gap in front of
it (previous dispatch's end -> this dispatch's start), mean by decile of the trips that ran, and
the whole loop.  Trips queued behind a halt (every kernel returns at once) are counted apart.
No probe build is needed: the stamps are the dispatches' own.

usage: trip_timeline.py run_results.db [training index, default: the last] [trip log]
  trip log: the library's BPE355_TRIP_LOG file of the same run (8 ints per trip: round, k, full
  scan, list entries, ntok, |C|, listed keys, fresh tokens): the kernels' durations by those.
"""
import sqlite3
import sys

import numpy as np


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = [(n, s, e) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    trips, cur, prev_end, trainings = [], None, None, [[]]
    for name, s, e in rows:
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = e
        if "k_select" in name:
            cur = {"sel": (e - s) / 1e3, "g_sel": gap, "t0": s}
        elif "k_merge_batch" in name and cur is not None and "merge" not in cur:
            cur["merge"], cur["g_merge"] = (e - s) / 1e3, gap
        elif "k_apply_batch" in name and cur is not None and "merge" in cur:
            cur["apply"], cur["g_apply"] = (e - s) / 1e3, gap
            cur["t1"] = e
            trainings[-1].append(cur)
            cur = None
        elif "k_init_pairs" in name or "k_hist_words" in name:
            if trainings[-1]:
                trainings.append([])
    trainings = [t for t in trainings if t]
    pick = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    log = None
    if len(sys.argv) > 3:
        raw = np.fromfile(sys.argv[3], dtype=np.int32).reshape(-1, 8)
        log = raw[raw[:, 1] > 0]
    T = trainings[pick]
    ran = [t for t in T if t["merge"] > 6.0 and t["apply"] > 6.0]   # a trip queued behind a halt: every kernel returns at once (~5-6 us each under the tracer)
    halted = len(T) - len(ran)
    keys = ["g_sel", "sel", "g_merge", "merge", "g_apply", "apply"]
    A = np.array([[t[k] for k in keys] for t in ran])
    # the next trip's select gap belongs to this trip's cost
    nxt = np.array([ran[i + 1]["g_sel"] if i + 1 < len(ran) else 0.0 for i in range(len(ran))])
    span = (T[-1]["t1"] - T[0]["t0"]) / 1e6
    print(f"# {sys.argv[1]}: {len(trainings)} trainings; training {pick}: {len(T)} trips "
          f"({halted} queued behind a halt), first select -> last apply {span:.2f} ms")
    print(f"{'decile':>6s} {'sel':>6s} {'g>mrg':>6s} {'merge':>6s} {'g>app':>6s} {'apply':>6s} {'g>sel':>6s} {'trip':>6s}")
    for d, idx in enumerate(np.array_split(np.arange(len(ran)), 10)):
        m = A[idx].mean(axis=0)
        g = nxt[idx].mean()
        print(f"{d:6d} {m[1]:6.1f} {m[2]:6.1f} {m[3]:6.1f} {m[4]:6.1f} {m[5]:6.1f} {g:6.1f} {m[1:].sum() + g:6.1f}")
    m = A.mean(axis=0)
    g = nxt.mean()
    print(f"{'all':>6s} {m[1]:6.1f} {m[2]:6.1f} {m[3]:6.1f} {m[4]:6.1f} {m[5]:6.1f} {g:6.1f} {m[1:].sum() + g:6.1f}")
    # the host's halts: from a trip's apply end to the next select's start, with the kernels between
    halts, seen = [], False
    tr_rows = [(n, s, e) for n, s, e in rows]
    i0 = None
    for idx, (n, s, e) in enumerate(tr_rows):
        if "k_apply_batch" in n:
            i0 = idx
        elif "k_select" in n and i0 is not None:
            between = tr_rows[i0 + 1:idx]
            if between and any("k_select" not in b[0] and "k_merge_batch" not in b[0] and "k_snapshot" not in b[0]
                               for b in between):
                kern = {}
                for b in between:
                    nm = b[0].split("(")[0].replace("void ", "")[:28]
                    kern[nm] = kern.get(nm, 0.0) + (b[2] - b[1]) / 1e3
                halts.append(((s - tr_rows[i0][2]) / 1e3, kern))
            i0 = None
    if halts:
        tot = sum(h[0] for h in halts)
        kt = {}
        for _, kern in halts:
            for k, v in kern.items():
                kt[k] = kt.get(k, 0.0) + v
        print(f"host halts: {len(halts)}, {tot / 1e3:.2f} ms from apply end to the next select "
              f"({sum(kt.values()) / 1e3:.2f} ms of it in kernels); per halt us: "
              + " ".join(f"{h[0]:.0f}" for h in halts))
        print("  kernels in halts (ms): " + ", ".join(f"{k} {v / 1e3:.2f}" for k, v in sorted(kt.items(), key=lambda x: -x[1])[:14]))
    if log is not None and len(log) == len(ran):
        ntok, k, full, lst, nC, ln = log[:, 4], log[:, 1], log[:, 2], log[:, 3], log[:, 5], log[:, 6]

        def table(title, key, edges, col):
            print(f"{title}:")
            for lo, hi in zip(edges, edges[1:]):
                sel = (key >= lo) & (key < hi)
                if sel.sum():
                    print(f"   [{lo:>7d},{hi:>7d}) n={sel.sum():5d} " + " ".join(
                        f"{nm} {A[sel, c].mean():6.1f}" for nm, c in col))
        cols = [("sel", 1), ("merge", 3), ("apply", 5)]
        table("by ntok", ntok, [0, 1000, 2000, 4000, 8000, 12000, 16000, 20000, 24000, 28000, 40000], cols)
        table("by k", k, [1, 2, 4, 8, 12, 16, 17, 33], cols)
        table("by |C|", nC, [0, 2000, 4000, 6000, 8000, 12000, 16000, 32000, 1 << 30], cols)
        table("by list entries (list mode)", np.where(full > 0, -1, lst), [0, 1000, 10000, 50000, 100000, 300000, 1 << 30], cols)
        print(f"full scans: {int((full > 0).sum())} trips, merge {A[full > 0, 3].mean() if (full > 0).any() else 0:.1f} us")
    elif log is not None:
        print(f"trip log: {len(log)} trips, the trace {len(ran)}: not joined")
    print(f"sum over trips that ran: select {A[:, 1].sum() / 1e3:.1f} ms, merge {A[:, 3].sum() / 1e3:.1f} ms, "
          f"apply {A[:, 5].sum() / 1e3:.1f} ms, gaps {(A[:, 2].sum() + A[:, 4].sum() + nxt.sum()) / 1e3:.1f} ms")


if __name__ == "__main__":
    main()
