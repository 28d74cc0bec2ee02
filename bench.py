#!/usr/bin/env python3
"""bench.py -- BPE train input MB/s + merges/s at 32k vocab; encode MB/s (BASELINE.json metric).

One step = one full train_bpe (BASELINE.json configs[2]: OpenWebText sizing, vocab 32000 with
<|endoftext|>, perf/bpe/owt.py:4-6) over a synthetic OWT-like corpus already resident in HBM:
UTF-8 check, GPT-2 pre-tokenization, unique-word count, pair histogram, 31,743 merge rounds,
merges/vocab back on the host.  OWT itself is not available offline; the corpus is the
library's deterministic generator (bpe_synth_corpus_device), `--bytes` per GPU.

Multi-GPU (torchrun, one rank per GPU): each rank owns a slab of the same global corpus (weak
scaling: per-GPU bytes fixed) and pre-tokenizes/counts it; ONE RCCL all-gather of the slabs'
unique-word tables follows, and every rank trains on their union (no per-round collective;
BPE355_EXCHANGE=rounds selects the per-round all-reduce of the pair deltas instead).  Every rank
ends with the identical global merge list.

Prints ONE JSON line on rank 0.  Extra fields: merges_per_s, encode MB/s (Tokenizer.encode of
the same corpus with the trained merges), roofline of the dominant kernel (HIP events on the
library's stream), and cpu_baseline: the pure-Python port of the reference (oracle/cpu_ref.py)
on a bounded sample, timed on this host.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
for p in (ROOT / "transformer-lm_amd", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip parameters)
EOT = "<|endoftext|>"
BLOCK = 4096                   # synthetic generator block (every block boundary is a safe split)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--bytes", type=float, default=11.9e9, help="corpus bytes per GPU")
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--flavour", type=int, default=0, help="0 OWT-like, 1 TinyStories-like")
    ap.add_argument("--no-encode", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-mb", type=float, default=16.0)
    ap.add_argument("--cpu-cap-s", type=float, default=20.0)
    ap.add_argument("--no-timing", action="store_true", help="skip per-launch HIP event timing")
    return ap.parse_args()


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    from bpe_amd import _lib, train_bpe_device, Tokenizer

    torch.cuda.set_device(local_rank)
    L = _lib.lib()
    _lib.require_device()
    comm = None
    if world > 1:
        from bpe_amd.dist import Communicator
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        comm = Communicator.from_torch(local_rank)   # RCCL: one all-gather of the word tables

    # ---------------------------------------------------------------- corpus slab in HBM
    blocks = max(1, int(args.bytes) // BLOCK)
    n = blocks * BLOCK
    corpus = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    _lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(corpus.data_ptr()), n, args.seed,
                                         args.flavour, rank * blocks, None), "synth")
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    def train_once():
        return train_bpe_device(corpus.data_ptr(), n, args.vocab, [EOT], comm=comm)

    from bpe_amd.train import last_train_stats
    L.bpe_set_timing(0)
    for _ in range(args.warmup):
        vocab, merges = train_once()
    L.bpe_set_timing(0 if args.no_timing else 1)
    stats = []
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        vocab, merges = train_once()
        stats.append(last_train_stats())
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    L.bpe_set_timing(0)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    total_bytes = n * world
    value = total_bytes / (elapsed / args.steps) / 1e6

    merge_ms = sum(s["t_merge_ms"] for s in stats) / len(stats)
    rounds = len(merges)
    # dominant kernel (event-timed on the library's stream during the timed steps)
    k_merge_ms = sum(s["merge_kernel_ms"] for s in stats)
    k_merge_launch = sum(s["merge_kernel_launches"] for s in stats)
    k_merge_bytes = sum(s["merge_kernel_bytes"] for s in stats)
    k_count_ms = sum(s["count_kernel_ms"] for s in stats)
    k_count_bytes = sum(s["count_kernel_bytes"] for s in stats)
    roofline = None
    if k_merge_ms > 0 or k_count_ms > 0:
        # the merge kernel is event-timed on a sample of its launches: compare per-step
        # estimates (one launch per trip when rounds are batched, else one per round)
        trips = sum(s.get("n_trips", 0) for s in stats) / len(stats)
        merge_launches = trips if trips > 0 else rounds
        merge_step_ms = k_merge_ms / max(1, k_merge_launch) * merge_launches
        count_step_ms = k_count_ms / len(stats)
        if merge_step_ms >= count_step_ms:
            kname = "k_merge_batch" if trips > 0 else "k_merge"
            kms, kb, kl = k_merge_ms, k_merge_bytes, k_merge_launch
        else:
            kname, kms, kb, kl = "k_count_words", k_count_ms, k_count_bytes, len(stats)
        achieved = kb / (kms / 1e3) / 1e9
        traffic = None
        tf = ROOT / "profiles" / "traffic.json"
        if tf.exists():
            traffic = json.loads(tf.read_text()).get(kname)
        roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "kernel": kname,
                    "launches_per_step": round(merge_launches) if kname != "k_count_words" else 1,
                    "timed_launches": kl,
                    "avg_launch_us": round(kms / kl * 1e3, 3),
                    "bytes_per_launch": kb / kl}

    # ---------------------------------------------------------------- encode MB/s
    encode = None
    if not args.no_encode:
        tok = Tokenizer(vocab, merges, [EOT])
        h = tok._device()
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        n_out = ctypes.c_size_t(0)
        _lib.check(L.bpe_tok_encode_device(h, ctypes.c_void_p(corpus.data_ptr()), n,
                                           ctypes.c_void_p(out.data_ptr()), ctypes.byref(n_out),
                                           None), "encode")  # warm-up pass
        barrier()
        torch.cuda.synchronize()
        te = time.perf_counter()
        _lib.check(L.bpe_tok_encode_device(h, ctypes.c_void_p(corpus.data_ptr()), n,
                                           ctypes.c_void_p(out.data_ptr()), ctypes.byref(n_out),
                                           None), "encode")
        torch.cuda.synchronize()
        barrier()
        te = time.perf_counter() - te
        if world > 1:
            t = torch.tensor([te], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            te = float(t.item())
        encode = {"value": round(total_bytes / te / 1e6, 1), "unit": "MB/s",
                  "ids_per_gpu": int(n_out.value), "seconds": round(te, 4)}
        del out

    # ---------------------------------------------------------------- CPU baseline (rank 0, N=1)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import cpu_ref
        m = min(n, int(args.cpu_sample_mb * 1e6) // BLOCK * BLOCK)
        text = corpus[:m].cpu().numpy().tobytes().decode("utf-8")
        t0c = time.perf_counter()
        _, cmerges, info = cpu_ref.train(text, args.vocab, [EOT], deadline=t0c + args.cpu_cap_s)
        per_round = info["t_merge_s"] / max(1, info["rounds_done"])
        projected = info["t_count_s"] + per_round * info["rounds_total"]
        cpu = {"value": round(m / projected / 1e6, 5), "unit": "MB/s", "cores": 1, "kind": "port",
               "sample": (f"first {m / 1e6:.1f} MB of the same corpus, vocab {args.vocab}, "
                          f"oracle/cpu_ref.py (pure Python, reference structure) on 1 core of "
                          f"{os.cpu_count()}: pre-tokenize+count {info['t_count_s']:.2f}s measured, "
                          f"{info['rounds_done']}/{info['rounds_total']} merge rounds in "
                          f"{info['t_merge_s']:.1f}s measured, rest extrapolated at "
                          f"{per_round * 1e3:.1f} ms/round"),
               "merges_per_s": round(1.0 / per_round, 2) if per_round > 0 else None}

    if rank == 0:
        s0 = stats[-1]
        line = {
            "metric": "BPE train input MB/s (32k vocab)",
            "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (bpe_synth_corpus_device OWT-like, random-free deterministic text)",
            "config": {"workload": "train_bpe OWT-sized synthetic corpus, vocab 32000, "
                                   "special <|endoftext|> (BASELINE configs[2])",
                       "bytes_per_gpu": n, "vocab_size": args.vocab, "merges": rounds,
                       "seed": args.seed, "flavour": args.flavour,
                       "parallelism": (f"corpus slabs x{world}, " + (
                           "RCCL all-reduce of the pair deltas per merge round"
                           if os.environ.get("BPE355_EXCHANGE") == "rounds" else
                           "one RCCL all-gather of the unique-word tables, then every rank "
                           "trains on their union")) if world > 1 else "1 GPU"},
            "merges_per_s": round(rounds / (merge_ms / 1e3), 1) if merge_ms else None,
            "encode": encode,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "phases_ms": {k: round(s0[k], 2) for k in ("t_prepare_ms", "t_count_ms", "t_exchange_ms",
                                                        "t_words_ms", "t_merge_ms", "t_total_ms")},
            "counters": {k: s0[k] for k in ("n_pretokens", "n_words", "n_exchanged_words",
                                            "n_pairs_final", "n_rebuilds", "n_rounds_device",
                                            "n_rounds_host", "n_index_builds")},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
