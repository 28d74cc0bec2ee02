"""`gloo` tests (world size 2 and 3) of the SHARDED training protocols, on CPU (no GPU needed).

libbpe355 shards the corpus into slabs cut at safe points (one per rank) and has two ways to
combine them (exchange.hip, train.hip):
  words  (default)  each rank counts its slab's unique words; ONE all-to-all sends every word to
                    the rank its hash names (its owner sums the ranks' counts); ONE all-gather of
                    the owners' tables (each word once); every rank trains on the union with no
                    further collective ("words-gather": the local tables gathered as they are,
                    counts summed by every rank; BPE355_EXCHANGE_OWNER=0);
  rounds            each rank keeps its unique words local and per merge round all-reduces one
                    fixed-layout int64 buffer of delta cells (L[x] for (x,a)-=c/(x,new)+=c and
                    R[y] for (b,y)-=c/(new,y)+=c); every rank applies the global deltas to a
                    replicated pair table and takes the same argmax.
These tests restate both protocols in plain Python over torch.distributed/gloo and check that
every rank produces exactly the merges of the unsharded reference semantics (the oracle, pinned
to the reference's goldens in test_oracle_golden.py).
"""
import multiprocessing as mp
import os
import socket

import pytest

import golden_cases as G
from oracle import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def safe_split(data: bytes, pos: int) -> int:
    """Largest p <= pos with data[p] == ' ' between two ASCII non-space bytes (see pretok.h)."""
    def nonspace(b):
        return b < 0x80 and b not in (0x20, 0x09, 0x0A, 0x0B, 0x0C, 0x0D)
    for p in range(min(pos, len(data) - 2), 0, -1):
        if data[p] == 0x20 and nonspace(data[p - 1]) and nonspace(data[p + 1]):
            return p
    return 0


def sharded_train(rank, world, slab: bytes, vocab_size, specials, mode="rounds"):
    import torch
    import torch.distributed as dist

    # local unique words (train.py:16-28 on this rank's slab; single bytes carry no pairs)
    text = oracle.decode_text(slab)
    counts = oracle.word_counts(text, specials)
    if mode == "words":
        # the all-to-all by owner: rank r's words for owner o are o's share of r's table (the
        # restatement ships every rank's per-owner tables and each keeps its column: gloo has no
        # object all-to-all); the owner sums the counts of its words over the ranks
        import zlib
        mine = [dict() for _ in range(world)]
        for w, c in counts.items():
            mine[zlib.crc32(w) % world][w] = c
        sent = [None] * world
        dist.all_gather_object(sent, mine)
        owned = {}
        for src in sent:
            for w, c in src[rank].items():
                owned[w] = owned.get(w, 0) + c
        # then one all-gather of the owners' tables: disjoint, so the union needs no sum
        gathered = [None] * world
        dist.all_gather_object(gathered, owned)
        counts = {}
        for table in gathered:
            for w, c in table.items():
                assert w not in counts, "a word with two owners"
                counts[w] = c
    elif mode == "words-gather":
        # gather every rank's table as it is, sum the counts word by word
        gathered = [None] * world
        dist.all_gather_object(gathered, counts)
        counts = {}
        for table in gathered:
            for w, c in table.items():
                counts[w] = counts.get(w, 0) + c
    words = [[bytes([c]) for c in w] for w in counts if len(w) >= 2]
    freq = [counts[w] for w in counts if len(w) >= 2]

    # vocab and token ids (by bytes) exactly as the device does: ids 0..255 = bytes
    base = []
    seen = set()
    for t in [s.encode() for s in specials] + [bytes([i]) for i in range(256)]:
        if t not in seen:
            seen.add(t)
            base.append(t)
    rounds = vocab_size - len(base)
    tok = [bytes([i]) for i in range(256)]
    tid = {t: i for i, t in enumerate(tok)}
    W = [[tid[c] for c in w] for w in words]

    def allreduce(vals):
        if mode != "rounds":   # the union is global already: no per-round exchange
            return vals
        t = torch.tensor(vals, dtype=torch.int64)
        dist.all_reduce(t)
        return t.tolist()

    # initial histogram: one all-reduce of the dense 256 x 256 table
    hist = [0] * 65536
    for w, c in zip(W, freq):
        for x, y in zip(w, w[1:]):
            hist[x * 256 + y] += c
    hist = allreduce(hist)
    count = {(i >> 8, i & 255): v for i, v in enumerate(hist) if v}   # present keys

    merges = []
    ncap = 256 + max(rounds, 0) + 1
    for _ in range(max(rounds, 0)):
        if not count:
            break
        best = max(count, key=lambda k: (count[k], tok[k[0]], tok[k[1]]))
        a, b = best
        nb = tok[a] + tok[b]
        if nb in tid:
            nw = tid[nb]
        else:
            nw = len(tok)
            tok.append(nb)
            tid[nb] = nw
        merges.append((tok[a], tok[b]))
        cells = [0] * (2 * ncap)
        for wi, w in enumerate(W):
            if not any(w[i] == a and w[i + 1] == b for i in range(len(w) - 1)):
                continue
            c = freq[wi]
            out, r = [], 0
            while r < len(w):
                if r + 1 < len(w) and w[r] == a and w[r + 1] == b:
                    if out:
                        cells[2 * out[-1]] += c
                    if r + 2 < len(w):
                        cells[2 * w[r + 2] + 1] += c
                    out.append(nw)
                    r += 2
                else:
                    out.append(w[r])
                    r += 1
            W[wi] = out
        cells = allreduce(cells)          # the one collective per merge round
        count.pop(best)
        for cell, d in enumerate(cells):
            if not d:
                continue
            x = cell >> 1
            if cell & 1:
                dec, inc = (b, x), (nw, x)
            else:
                dec, inc = (x, a), (x, nw)
            if dec != best:
                count[dec] = count.get(dec, 0) - d
            count[inc] = count.get(inc, 0) + d
    return merges


def _worker(rank, world, port, slabs, vocab_size, specials, q, mode):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, sharded_train(rank, world, slabs[rank], vocab_size, specials, mode)))
    finally:
        dist.destroy_process_group()


def run_sharded(data: bytes, world: int, vocab_size: int, specials, mode="rounds"):
    cuts = [0] + [safe_split(data, len(data) * r // world) for r in range(1, world)] + [len(data)]
    slabs = [data[cuts[r]:cuts[r + 1]] for r in range(world)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, slabs, vocab_size, specials, q, mode))
             for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("mode", ["words", "words-gather", "rounds"])
@pytest.mark.parametrize("name,world", [("corpus_en_500", 2), ("tiny_1200", 2),
                                        ("synth_mixed_200k", 2), ("corpus_en_1000", 3)])
def test_sharded_protocol_matches_reference(name, world, mode):
    o, _vocab, merges = G.train_expect(name)
    data = G.input_bytes(o["input"])   # raw bytes: slabs are cut at safe points, then decoded
    out = run_sharded(data, world, o["vocab_size"], o["special_tokens"], mode)
    for r in range(world):   # every rank holds the identical, global merge list
        assert out[r] == merges
