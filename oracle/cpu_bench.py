"""ORACLE -- TEST INFRASTRUCTURE ONLY: the CPU baselines bench.py reports as `cpu_baseline`.

Run by bench.py as a child process (it never touches the GPU and never imports torch):

  python -m oracle.cpu_bench --corpus FILE --vocab 32000 --merges-json M.json --out R.json

Legs, all on this host's cores:
  c1        the reference's own test case in full: tests/fixtures corpus.en at vocab 500
            (tests/test_train_bpe.py:28-34), oracle/cpu_ref.py (pure-Python port of
            models/tokenizer/train.py, the reference's structure), one core.
  train     the first 16 MB and 64 MB of the bench corpus at the bench vocab, the same port, one
            core each (two processes): pre-tokenize + count measured in full, the merge rounds
            measured until a wall cap, the rest extrapolated (rounds_measured_frac says how much
            was measured).  The extrapolation follows the port's measured cost curve
            (cpu_port_growth.json: a complete 16 MB run, whose merges equal the C oracle's): a round
            costs ~10 x more at the end than over the first rounds (the argmax scans every live
            pair), so the flat mean of the first rounds under-estimated the complete run by 86.5 %
            (VERDICT r04 item 7).  MBps is the corrected rate; MBps_flat the old flat one.
  encode    Tokenizer.encode port (cpu_ref.Encoder, tokenizer.py:92-138) of the first 64 MB with
            the GPU-trained merges, in 1 M-character pieces each encoded on its own -- the
            reference's dataset encoder (encode.py:31-36) -- over a pool of processes (cores
            stated).  Piece 0's ids are returned for bench.py to compare with the GPU encoder.
  exact     the C oracle (oracle/bpe_oracle.c: exact incremental trainer) on the full bench corpus
            (C3: 11.9 GB OWT-like, vocab 32 000; BASELINE configs[2]; SURVEY.md §8d's "C++ exact
            CPU trainer on all host cores") with one counting thread per core of the host's share
            and its single-threaded merge loop; the result is checked against the train_C3 scale
            golden (train_C2 when the bench corpus is not C3).
"""
from __future__ import annotations

import argparse
import gzip
import hashlib
import json
import multiprocessing as mp
import os
import pathlib
import struct
import sys
import threading
import time

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parent
for p in (ROOT, ROOT / "transformer-lm_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

EOT = "<|endoftext|>"
BLOCK = 4096


def growth_factor(rounds_done: int, rounds_total: int, nbytes: int, vocab: int):
    """(mean ms per round over the whole run) / (mean over the first rounds_done rounds), from the
    complete run's cumulative cost curve (cpu_port_growth.json), and whether that curve was
    measured on this sample (same bytes and vocab: the correction is then validated; a larger
    sample has more live pairs and its cost grows along a curve nobody measured), or (None, False)"""
    f = HERE / "cpu_port_growth.json"
    if not f.exists() or rounds_done <= 0:
        return None, False
    g = json.loads(f.read_text())
    pts = g["points"]
    if rounds_total != g.get("rounds_total"):
        return None, False
    r = min(rounds_done, pts[-1][0])
    if r <= pts[0][0]:   # before the first point: its mean
        t = pts[0][1] * r / pts[0][0]
    else:
        t = pts[-1][1]
        for (r0, t0), (r1, t1) in zip(pts, pts[1:]):
            if r0 <= r <= r1:
                t = t0 + (t1 - t0) * (r - r0) / max(1, r1 - r0)
                break
    whole = pts[-1][1] / pts[-1][0]
    validated = nbytes == g.get("bytes") and vocab == g.get("vocab")
    return (whole / (t / r) if t > 0 else None), validated


def _train_leg(args):
    """one pure-Python training on `m` bytes of a file (m = None: the whole file)"""
    path, m, vocab, cap_s = args
    from oracle import cpu_ref
    with open(path, "rb") as f:
        text = (f.read(m) if m else f.read()).decode("utf-8")
    text = text.replace("\r\n", "\n").replace("\r", "\n")   # the reference's text-mode read
    t0 = time.perf_counter()
    _, merges, info = cpu_ref.train(text, vocab, [EOT], round_cap_s=cap_s)
    wall = time.perf_counter() - t0
    # the rounds' mean excludes the one-time build of the words, pair counts and index
    per_round = (info["t_merge_s"] - info["t_build_s"]) / max(1, info["rounds_done"])
    flat = info["t_count_s"] + info["t_build_s"] + per_round * info["rounds_total"]
    nb = len(text.encode("utf-8"))
    gf, gf_ok = (None, True) if info["complete"] else growth_factor(info["rounds_done"], info["rounds_total"], nb,
                                                                     vocab)
    projected = flat if gf is None else info["t_count_s"] + info["t_build_s"] + per_round * info["rounds_total"] * gf
    return {"bytes": nb, "vocab": vocab, "wall_s": round(wall, 3), "t_count_s": round(info["t_count_s"], 3),
            "t_build_s": round(info["t_build_s"], 3),
            "rounds_done": info["rounds_done"], "rounds_total": info["rounds_total"],
            "rounds_measured_frac": round(info["rounds_done"] / max(1, info["rounds_total"]), 4),
            "ms_per_round": round(per_round * 1e3, 3),
            "MBps": round(nb / projected / 1e6, 5) if projected > 0 else None,
            "MBps_flat": round(nb / flat / 1e6, 5) if flat > 0 else None,
            "growth_factor": round(gf, 3) if gf else None,
            "growth_validated": bool(gf_ok),
            "merges_per_s": round(info["rounds_total"] / max(1e-9, projected - info["t_count_s"] - info["t_build_s"]), 2)
                            if per_round > 0 else None,
            "complete": info["complete"],
            "merges_sha256": hashlib.sha256(b"".join(struct.pack("<I", len(a)) + a + struct.pack("<I", len(b)) + b
                                                     for a, b in merges)).hexdigest()}


_ENC = None


def _enc_init(vocab_items, merges):
    global _ENC
    from oracle import cpu_ref
    _ENC = cpu_ref.Encoder(dict(vocab_items), merges, [EOT])


def _enc_piece(piece: str):
    t = time.perf_counter()
    ids = _ENC.encode(piece)
    return len(ids), time.perf_counter() - t, ids


def _pieces(text: str, chars: int):
    return [text[i:i + chars] for i in range(0, len(text), chars)]


def encode_leg(path, m, merges_json, procs, chars=1024 * 1024):
    with open(merges_json) as f:
        mj = json.load(f)
    merges = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in mj["merges"]]
    vocab = {int(i): bytes.fromhex(h) for i, h in mj["vocab"]}
    with open(path, "rb") as f:
        text = f.read(m).decode("utf-8")
    pieces = _pieces(text, chars)
    ctx = mp.get_context("fork")   # this process never initialised a GPU
    t0 = time.perf_counter()
    with ctx.Pool(procs, initializer=_enc_init, initargs=(list(vocab.items()), merges)) as pool:
        res = pool.map(_enc_piece, pieces, chunksize=1)
    wall = time.perf_counter() - t0
    n_ids = sum(r[0] for r in res)
    busy = sum(r[1] for r in res)
    nb = len(text.encode("utf-8"))
    return {"bytes": nb, "pieces": len(pieces), "chars_per_piece": chars, "procs": procs,
            "wall_s": round(wall, 3), "MBps": round(nb / wall / 1e6, 4),
            "MBps_per_core": round(nb / busy / 1e6, 4), "n_ids": n_ids,
            "piece0_chars": len(pieces[0]) if pieces else 0}, (res[0][2] if res else [])


def host_threads():
    """threads for the CPU legs: the host's share of cores (OMP_NUM_THREADS where the job
    scheduler sets it -- 16 on the GPU box, whose os.cpu_count() shows every core of the machine
    -- else the cores this process may run on)"""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(int(env), aff) if env and env.isdigit() else aff)


def exact_leg(threads, corpus=None, golden="train_C2", piece=64 << 20):
    """The C oracle (exact incremental trainer, lazy max-heap argmax) on a full scale corpus:
    `corpus` = the bench's own corpus file (memory-mapped, page-cache warm), else the golden's
    corpus generated into host memory first (untimed).  Counted by `threads` threads (safe-split
    pieces, one oracle counter each), summed, trained, and checked against the golden."""
    import numpy as np
    from bpe_amd import _lib   # the corpus generator's host twin only (no device call)
    from oracle import oracle
    g = json.load(gzip.open(ROOT / "tests" / "golden" / "scale" / f"{golden}.json.gz", "rt"))
    n, seed, flavour = g["n"], g["seed"], g["flavour"]
    t_gen = 0.0
    if corpus is not None:
        assert os.path.getsize(corpus) == n, f"{corpus} is not the {golden} corpus"
        buf = np.memmap(corpus, dtype=np.uint8, mode="r")
    else:
        L = _lib.lib()
        buf = np.empty(n, dtype=np.uint8)
        tg = time.perf_counter()
        assert L.bpe_synth_corpus_host(buf.ctypes.data, n, seed, flavour, 0, threads) == 0
        t_gen = time.perf_counter() - tg
    base = buf.ctypes.data
    pieces = [(lo, min(piece, n - lo)) for lo in range(0, n, piece)]
    counters = [oracle.Counter([EOT]) for _ in range(threads)]
    t0 = time.perf_counter()

    def work(t):
        for i in range(t, len(pieces), threads):
            lo, m = pieces[i]
            counters[t].feed(base + lo, m)

    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for c in counters[1:]:
        counters[0].absorb(c)
        c.close()
    t_count = time.perf_counter() - t0
    print(f"[cpu_bench] exact leg: counted {n / 1e9:.2f} GB on {threads} threads in {t_count:.1f} s; training",
          file=sys.stderr, flush=True)
    # a heartbeat while the merge loop runs (one C call that prints nothing): a run that writes
    # nothing for minutes reads as hung
    done = threading.Event()

    def beat():
        while not done.wait(30.0):
            print(f"[cpu_bench] exact leg: training, {time.perf_counter() - t0 - t_count:.0f} s", file=sys.stderr,
                  flush=True)
    hb = threading.Thread(target=beat, daemon=True)
    hb.start()
    try:
        vocab, merges = counters[0].train(g["vocab"])
    finally:
        done.set()
        hb.join()
    wall = time.perf_counter() - t0
    counters[0].close()
    del buf
    h = hashlib.sha256()
    for i in range(len(vocab)):
        h.update(struct.pack("<I", len(vocab[i])) + vocab[i])
    want = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in g["merges"]]
    return {"config": golden, "bytes": n, "vocab": g["vocab"], "threads": threads,
            "source": "the bench's corpus file, memory-mapped" if corpus else "generated into host memory",
            "wall_s": round(wall, 3), "t_count_s": round(t_count, 3), "t_merge_s": round(wall - t_count, 3),
            "t_generate_s": round(t_gen, 3), "MBps": round(n / wall / 1e6, 2),
            "merges_per_s": round(len(merges) / max(1e-9, wall - t_count), 1),
            "exact": merges == want and h.hexdigest() == g["vocab_sha256"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--corpus", required=True)
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--samples-mb", default="16,64")
    ap.add_argument("--cap-s", type=float, default=20.0, help="wall cap of each sample's merge rounds")
    ap.add_argument("--merges-json", default=None)
    ap.add_argument("--encode-mb", type=float, default=64.0)
    ap.add_argument("--procs", type=int, default=0, help="cores for the encode pool and the exact leg (0: host_threads())")
    ap.add_argument("--no-exact", action="store_true")
    ap.add_argument("--exact-corpus", default=None, help="the corpus file of --exact-golden (else generated)")
    ap.add_argument("--exact-golden", default="train_C2", help="scale golden of the exact leg")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    a.procs = a.procs or host_threads()
    c1 = ROOT / "tests" / "golden" / "fixtures" / "corpus.en"
    legs = [(str(c1), None, 500, None)]
    for s in a.samples_mb.split(","):
        m = int(float(s) * 1e6) // BLOCK * BLOCK
        legs.append((a.corpus, m, a.vocab, a.cap_s))
    out = {"host_cpus": os.cpu_count(), "threads": host_threads()}
    t_all = time.perf_counter()

    def note(msg):   # progress on stderr (bench.py's log shows the run is alive)
        print(f"[cpu_bench {time.perf_counter() - t_all:6.1f}s] {msg}", file=sys.stderr, flush=True)
    note(f"legs: c1, training samples {a.samples_mb} MB, encode {a.encode_mb} MB; {a.procs} threads")
    ctx = mp.get_context("fork")
    with ctx.Pool(len(legs)) as pool:
        async_train = pool.map_async(_train_leg, legs)
        if a.merges_json:
            m = int(a.encode_mb * 1e6) // BLOCK * BLOCK
            out["encode"], piece0 = encode_leg(a.corpus, m, a.merges_json, max(1, a.procs - len(legs)))
            out["encode_piece0_ids_sha256"] = hashlib.sha256(struct.pack(f"<{len(piece0)}I", *piece0)).hexdigest()
        note("encode leg done")
        res = async_train.get()
    note("training legs done")
    out["c1"] = res[0]
    out["train"] = res[1:]
    if not a.no_exact:
        note(f"exact leg ({a.exact_golden})")
        out["exact"] = exact_leg(a.procs, a.exact_corpus, a.exact_golden)
        note(f"exact leg done: {out['exact']['wall_s']} s, exact {out['exact']['exact']}")
    with open(a.out, "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
