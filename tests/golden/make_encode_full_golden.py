"""Golden for BASELINE.json configs[4] at the full OWT size: Tokenizer.encode of the whole
11.9 GB C3 corpus with C3's 32k merges, from the C oracle (oracle/bpe_oracle.c, pinned to the
reference by the small goldens), on all host cores.

Two id streams are recorded, each as n_ids, the sha256 of the whole stream and the sha256 of
every slab of it (so a GPU test that disagrees says where):

  whole   encode(text) (reference models/tokenizer/tokenizer.py:111-138), ids as uint32 LE.
          The corpus is cut right after occurrences of <|endoftext|> near every 256 MiB: the
          special is the only split alternative and cannot overlap itself, so each occurrence
          is a re.split match and the segments after it are encoded independently of the text
          before it (tokenizer.py:63-90).  The slabs' ids, concatenated, are encode(text).
  pieces  encode.py:31-37: the text read 1024*1024 characters at a time (text mode; the corpus
          has no carriage return, checked), every piece encoded on its own, the ids saved as
          np.uint16.  Pieces are grouped ~256 per slab for the digests.

    python tests/golden/make_encode_full_golden.py [--threads 8]

writes tests/golden/scale/encode_C5_full.json.gz.
"""
from __future__ import annotations

import argparse
import gzip
import hashlib
import json
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import make_scale_golden as msg
from make_scale_golden import EOT, SCALE, load_train, oracle, _lib

SLAB = 256 << 20
CHARS_PER_PIECE = 1024 * 1024     # reference encode.py:33
PIECES_PER_GROUP = 256
SUB = 16 << 20                    # lead-byte counting block


def vocab_of(o, merges):
    vocab = {}
    for s in o["specials"]:
        vocab.setdefault(s.encode(), len(vocab))
    for b in range(256):
        vocab.setdefault(bytes([b]), len(vocab))
    for a, b in merges:
        vocab.setdefault(a + b, len(vocab))
    vocab = {i: b for b, i in vocab.items()}
    assert msg.vocab_digest(vocab) == o["vocab_sha256"]
    return vocab


def special_cuts(buf, n, step):
    """byte offsets right after the first <|endoftext|> at or past every multiple of `step`"""
    eot = EOT.encode()
    cuts = [0]
    for target in range(step, n, step):
        if target <= cuts[-1]:
            continue
        window = bytes(buf[target:min(n, target + (4 << 20))])
        i = window.find(eot)
        if i < 0:
            continue
        c = target + i + len(eot)
        if c < n:
            cuts.append(c)
    cuts.append(n)
    return cuts


def piece_starts(buf, n, threads):
    """byte offsets of characters K, 2K, ... (K = CHARS_PER_PIECE): where each f.read(K) begins"""
    blocks = [(lo, min(SUB, n - lo)) for lo in range(0, n, SUB)]

    def count(b):
        lo, m = b
        return int(np.count_nonzero((buf[lo:lo + m] & 0xC0) != 0x80))

    with ThreadPoolExecutor(threads) as ex:
        per = list(ex.map(count, blocks))
    before = np.concatenate([[0], np.cumsum(per)])

    def find(i):
        lo, m = blocks[i]
        c0, c1 = int(before[i]), int(before[i + 1])
        first = -(-c0 // CHARS_PER_PIECE) * CHARS_PER_PIECE
        if first == 0:
            first = CHARS_PER_PIECE
        if first >= c1:
            return []
        lead = np.flatnonzero((buf[lo:lo + m] & 0xC0) != 0x80)
        return [lo + int(x) for x in lead[first - c0:c1 - c0:CHARS_PER_PIECE]]

    with ThreadPoolExecutor(threads) as ex:
        out = [p for part in ex.map(find, range(len(blocks))) for p in part]
    return out, int(before[-1])


def run_ordered(jobs, fn, threads, consume):
    """fn(job) on a pool, results consumed in job order with at most 2 * threads outstanding"""
    with ThreadPoolExecutor(threads) as ex:
        futs = []
        nxt = 0
        for j in jobs:
            futs.append(ex.submit(fn, j))
            while len(futs) - nxt > 2 * threads:
                consume(jobs[nxt], futs[nxt].result())
                futs[nxt] = None
                nxt += 1
        for i in range(nxt, len(futs)):
            consume(jobs[i], futs[i].result())
            futs[i] = None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    o, merges = load_train("C3")
    vocab = vocab_of(o, merges)
    n = o["n"]
    L = _lib.lib()
    t0 = time.time()
    buf = np.empty(n, dtype=np.uint8)
    assert L.bpe_synth_corpus_host(buf.ctypes.data, n, o["seed"], o["flavour"], 0, a.threads) == 0
    piece = o["digest_piece"]
    with ThreadPoolExecutor(a.threads) as ex:
        dig = list(ex.map(lambda lo: hashlib.sha256(buf[lo:lo + piece]).hexdigest(), range(0, n, piece)))
    assert dig == o["piece_sha256"], "corpus differs from train_C3's"
    assert int(np.count_nonzero(buf == 13)) == 0, "corpus holds a carriage return"
    print(f"corpus {n} B generated and checked in {time.time() - t0:.0f}s", flush=True)
    enc = oracle.PieceEncoder(vocab, merges, o["specials"])
    out = {"case": "C5_full", "train": "C3", "n": n, "seed": o["seed"], "flavour": o["flavour"],
           "specials": o["specials"], "corpus_piece_sha256_of": "train_C3"}

    # ---- whole: encode(text)
    t1 = time.time()
    cuts = special_cuts(buf, n, SLAB)
    jobs = list(zip(cuts[:-1], cuts[1:]))
    h = hashlib.sha256()
    slabs = []
    head = []
    tail = [None]

    def enc_whole(job):
        lo, hi = job
        ids = enc.encode(buf.ctypes.data + lo, hi - lo)
        return ids, hashlib.sha256(ids.tobytes()).hexdigest()

    def take_whole(job, res):
        ids, d = res
        h.update(ids.tobytes())
        slabs.append([job[0], job[1], int(ids.size), d])
        if len(head) < 4096:
            head.extend(ids[:4096 - len(head)].tolist())
        tail[0] = ids[-4096:] if tail[0] is None or ids.size >= 4096 else np.concatenate([tail[0], ids])[-4096:]
        print(f"  whole slab {len(slabs)}/{len(jobs)}: {ids.size} ids", flush=True)

    run_ordered(jobs, enc_whole, a.threads, take_whole)
    n_ids = sum(s[2] for s in slabs)
    out["whole"] = {"n_ids": n_ids, "ids_sha256": h.hexdigest(), "dtype": "uint32",
                    "slabs": slabs, "ids_head": head, "ids_tail": tail[0].tolist(),
                    "oracle_seconds": round(time.time() - t1, 1)}
    print(f"whole: {n_ids} ids in {time.time() - t1:.0f}s", flush=True)

    # ---- pieces: encode.py
    t2 = time.time()
    starts, n_chars = piece_starts(buf, n, a.threads)
    bounds = [0] + starts + [n]
    groups = [(bounds[i], bounds[min(i + PIECES_PER_GROUP, len(bounds) - 1)], i)
              for i in range(0, len(bounds) - 1, PIECES_PER_GROUP)]
    hp = hashlib.sha256()
    gdig = []
    lock = threading.Lock()

    def enc_group(job):
        lo, hi, i0 = job
        inner = [b - lo for b in bounds[i0 + 1:i0 + PIECES_PER_GROUP] if lo < b < hi]
        ids = enc.encode(buf.ctypes.data + lo, hi - lo, inner)
        assert ids.size == 0 or int(ids.max()) <= 0xFFFF
        ids16 = ids.astype(np.uint16)
        return ids16, hashlib.sha256(ids16.tobytes()).hexdigest()

    def take_group(job, res):
        ids16, d = res
        hp.update(ids16.tobytes())
        with lock:
            gdig.append([job[0], job[1], int(ids16.size), d])
        print(f"  piece group {len(gdig)}/{len(groups)}: {ids16.size} ids", flush=True)

    run_ordered(groups, enc_group, a.threads, take_group)
    out["pieces"] = {"chars_per_piece": CHARS_PER_PIECE, "n_chars": n_chars, "n_pieces": len(bounds) - 1,
                     "piece_starts_sha256": hashlib.sha256(np.asarray(starts, dtype=np.uint64).tobytes()).hexdigest(),
                     "n_ids": sum(g[2] for g in gdig), "ids_u16_sha256": hp.hexdigest(), "dtype": "uint16",
                     "pieces_per_group": PIECES_PER_GROUP, "groups": gdig,
                     "oracle_seconds": round(time.time() - t2, 1)}
    print(f"pieces: {out['pieces']['n_pieces']} pieces, {out['pieces']['n_ids']} ids in {time.time() - t2:.0f}s",
          flush=True)
    SCALE.mkdir(exist_ok=True)
    with gzip.open(SCALE / "encode_C5_full.json.gz", "wt") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
