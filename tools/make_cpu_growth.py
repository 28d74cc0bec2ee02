#!/usr/bin/env python3
"""oracle/cpu_port_growth.json from a complete pure-Python run (tools/cpu_port_full.py output): the
cumulative merge-round time of the port against rounds done, which oracle/cpu_bench.py uses to
correct its flat-rate extrapolation of a capped run (the flat rate measured on
the first rounds under-estimated the complete 16 MB run by 86.5 %).

  python tools/make_cpu_growth.py profiles/r05/cpu_port_16MB_full.json oracle/cpu_port_growth.json
"""
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
d = json.load(open(src))
full, capped = d["full"], d["capped"]
off = full["t_count_s"] + full["t_build_s"]   # progress seconds count from the start of the call
pts = []
if capped["rounds_done"] > 0:   # the capped leg: the mean of its first rounds
    pts.append([capped["rounds_done"], round(capped["ms_per_round"] * capped["rounds_done"] / 1e3, 3)])
for r, t, _pairs in full["progress"]:
    pts.append([r, round(t - off, 3)])
total = full["wall_s"] - off
pts.append([full["rounds_total"], round(total, 3)])
out = {"_note": "cumulative merge-round seconds of oracle/cpu_ref.py against rounds done, one core, "
                "from " + src + " (" + d["sample"] + "); the full run's merges sha256 " + full["merges_sha256"],
       "rounds_total": full["rounds_total"], "points": pts,
       "flat_projection_error": d["extrapolation_error"]}
json.dump(out, open(dst, "w"), indent=1)
print(dst, len(pts), "points; mean ms/round over the run", round(total / full["rounds_total"] * 1e3, 1))
