#!/usr/bin/env python3
"""Checks bench.py's CPU-baseline extrapolation against a complete pure-Python run (VERDICT r04
next-round item 7).  Build container only: no GPU, no torch.

For a sample of the bench corpus (the first M bytes of bpe_synth_corpus_host seed 2, flavour 0,
which are the first M bytes of the 11.9 GB bench file: the generator is positional) it runs
oracle/cpu_ref.py twice on one core each:
  capped  exactly as oracle/cpu_bench.py does: the merge rounds stop after --cap-s seconds and the
          rest is extrapolated at the measured mean ms/round (flat rate);
  full    to completion, recording (rounds, seconds, live pairs) every 1000 rounds.
and writes both, plus the extrapolation's error, to --out.

  python tools/cpu_port_full.py --mb 16 --out profiles/r05/cpu_port_16MB_full.json
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import multiprocessing as mp
import pathlib
import struct
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "transformer-lm_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

EOT = "<|endoftext|>"
BLOCK = 4096


def sample_text(mb: float, seed: int, flavour: int) -> str:
    from bpe_amd import _lib
    m = int(mb * 1e6) // BLOCK * BLOCK
    buf = (ctypes.c_char * m)()
    assert _lib.lib().bpe_synth_corpus_host(ctypes.addressof(buf), m, seed, flavour, 0, 8) == 0
    text = bytes(buf).decode("utf-8")
    return text.replace("\r\n", "\n").replace("\r", "\n")   # the reference's text-mode read


def merges_sha(merges) -> str:
    return hashlib.sha256(b"".join(struct.pack("<I", len(a)) + a + struct.pack("<I", len(b)) + b
                                   for a, b in merges)).hexdigest()


class ProgressLog(list):
    """cpu_ref's progress list, also appended to a JSON-lines file as it grows (a long run can be
    read while it goes)"""
    def __init__(self, path):
        super().__init__()
        self.path = path

    def append(self, x):
        super().append(x)
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(x) + "\n")


def leg(args):
    mode, mb, vocab, cap_s, seed, flavour, plog = args
    from oracle import cpu_ref
    text = sample_text(mb, seed, flavour)
    nb = len(text.encode("utf-8"))
    prog: list = ProgressLog(plog if mode == "full" else None)
    t0 = time.perf_counter()
    _, merges, info = cpu_ref.train(text, vocab, [EOT], round_cap_s=cap_s if mode == "capped" else None,
                                    progress=prog)
    wall = time.perf_counter() - t0
    per_round = (info["t_merge_s"] - info["t_build_s"]) / max(1, info["rounds_done"])
    projected = info["t_count_s"] + info["t_build_s"] + per_round * info["rounds_total"]
    return {"mode": mode, "bytes": nb, "vocab": vocab, "wall_s": round(wall, 3),
            "t_count_s": round(info["t_count_s"], 3), "t_build_s": round(info["t_build_s"], 3),
            "rounds_done": info["rounds_done"], "rounds_total": info["rounds_total"],
            "complete": info["complete"], "ms_per_round": round(per_round * 1e3, 3),
            "projected_wall_s": round(projected, 3), "MBps_projected": round(nb / projected / 1e6, 5),
            "MBps_measured": round(nb / wall / 1e6, 5) if info["complete"] else None,
            "merges_sha256": merges_sha(merges), "progress": list(prog)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=16.0)
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--cap-s", type=float, default=20.0)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--flavour", type=int, default=0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--progress-file", default=None, help="JSON lines of the full leg's progress")
    a = ap.parse_args()
    legs = [(m, a.mb, a.vocab, a.cap_s, a.seed, a.flavour, a.progress_file) for m in ("capped", "full")]
    with mp.get_context("fork").Pool(2) as pool:
        capped, full = pool.map(leg, legs)
    err = capped["projected_wall_s"] / full["wall_s"] - 1.0
    out = {"sample": f"first {full['bytes'] / 1e6:.1f} MB of the bench corpus (seed {a.seed}, flavour "
                     f"{a.flavour}) at vocab {a.vocab}, oracle/cpu_ref.py on one core per leg",
           "capped": capped, "full": full,
           "extrapolation_error": round(err, 4),
           "note": "extrapolation_error = capped projected wall / full measured wall - 1 "
                   "(negative: the flat-rate model under-estimates the CPU's time, i.e. flatters it)"}
    pathlib.Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    pathlib.Path(a.out).write_text(json.dumps(out, indent=1))
    print(json.dumps({k: out[k] for k in ("sample", "extrapolation_error")}))


if __name__ == "__main__":
    main()
