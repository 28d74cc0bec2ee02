#!/usr/bin/env python3
"""bench.py -- BPE train input MB/s + merges/s at 32k vocab; encode MB/s (BASELINE.json metric).

One step = one drop-in `train_bpe(input_path, 32000, ["<|endoftext|>"])` (reference
models/tokenizer/train.py:142-231; BASELINE configs[2]: OpenWebText sizing, perf/bpe/owt.py:4-6)
over an OWT-sized synthetic corpus FILE, page-cache warm: the file read (train.py:22), UTF-8
check, GPT-2 pre-tokenization, unique-word count, pair histogram, 31,743 merge rounds, merges and
vocab back in host memory.  OWT itself is not available offline; the corpus is the library's
deterministic generator (bpe_synth_corpus_host), written once to a scratch file before timing.

`value` is that end-to-end rate ("input MB/s = N / end-to-end wall, file read ->
merges in host memory").  `device_resident` is the same training with the corpus already in HBM
(train_bpe_device), i.e. without the file read and the host->device copy.

GPUs (strong scaling: the corpus size is fixed, --bytes in total):
  * `python bench.py --gpus N` (no WORLD_SIZE): ONE process drives N devices, as the reference's
    single-process caller would (perf/bpe/util.py:16): train_bpe with set_num_gpus(N) -- one slab
    of the file per device, one RCCL all-gather of the word tables, the merge loop on device 0.
  * under torch.distributed.run (WORLD_SIZE = N): one process per GPU; every rank reads its share
    of the same file (train_bpe(..., comm, split_file=True)); same exchange.  --gpus must equal
    WORLD_SIZE.
`n_gpus` reports the ranks that actually took part (from the library's stats).

Prints ONE JSON line on rank 0.  Extra fields: merges_per_s, merge_loop (trips, time per trip),
encode (Tokenizer.encode of the corpus with the trained merges, device to device), roofline of
the dominant kernel (HIP events stamped by the kernel's own dispatch, on the library's stream),
and cpu_baseline: the pure-Python port of the reference (oracle/cpu_ref.py) on a bounded sample,
timed on this host (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import mmap
import os
import pathlib
import sys
import tempfile
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
    ap.add_argument("--bytes", type=float, default=11.9e9, help="corpus bytes in total (strong scaling)")
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--flavour", type=int, default=0, help="0 OWT-like, 1 TinyStories-like")
    ap.add_argument("--corpus-dir", default=os.environ.get("BPE355_BENCH_DIR", tempfile.gettempdir()))
    ap.add_argument("--keep-corpus", action="store_true")
    ap.add_argument("--no-device-resident", action="store_true")
    ap.add_argument("--no-encode", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exact-c3", action="store_true",
                    help="run the exact C oracle leg on the bench corpus itself (C3: ~5 min) instead of C2")
    ap.add_argument("--cpu-samples-mb", default="16,64", help="pure-Python training samples (MB)")
    ap.add_argument("--cpu-cap-s", type=float, default=20.0, help="wall cap of each sample's merge rounds")
    ap.add_argument("--cpu-encode-mb", type=float, default=64.0)
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="host cores for the encode pool / exact leg (0: the host's share, OMP_NUM_THREADS or "
                         "the affinity mask)")
    ap.add_argument("--no-timing", action="store_true", help="skip per-launch HIP event timing")
    ap.add_argument("--no-file", action="store_true",
                    help="profiling runs: skip the file path (every k_count2 launch then covers the whole "
                         "corpus); the line then reports the HBM-resident rate")
    return ap.parse_args()


def write_corpus(L, path: pathlib.Path, n: int, seed: int, flavour: int):
    """the generator's bytes [0, n) into `path` through a shared mapping (page-cache warm)"""
    tmp = path.with_suffix(".part")
    with open(tmp, "wb+") as f:
        f.truncate(n)
        with mmap.mmap(f.fileno(), n) as m:
            buf = (ctypes.c_char * n).from_buffer(m)
            rc = L.bpe_synth_corpus_host(ctypes.addressof(buf), n, seed, flavour, 0, 16)
            del buf
            assert rc == 0, rc
    os.replace(tmp, path)


def golden_name(n, seed, flavour, vocab_size):
    """the scale golden of (n, seed, flavour, vocab), e.g. "train_C3", or None"""
    import gzip
    for p in sorted((ROOT / "tests" / "golden" / "scale").glob("train_*.json.gz")):
        g = json.load(gzip.open(p, "rt"))
        if (g["n"], g["seed"], g["flavour"], g["vocab"]) == (n, seed, flavour, vocab_size):
            return p.name[:-len(".json.gz")]
    return None


def golden_parity(n, seed, flavour, vocab_size, vocab, merges):
    """The step's result against the committed scale golden of the same corpus, if there is one
    (tests/golden/scale/train_*.json.gz: the C oracle's merges and vocab sha256 for (n, seed,
    flavour, vocab), made by tests/golden/make_scale_golden.py; test data, not the oracle)."""
    import gzip
    import hashlib
    import struct
    for p in sorted((ROOT / "tests" / "golden" / "scale").glob("train_*.json.gz")):
        g = json.load(gzip.open(p, "rt"))
        if (g["n"], g["seed"], g["flavour"], g["vocab"]) != (n, seed, flavour, vocab_size):
            continue
        h = hashlib.sha256()
        for i in range(len(vocab)):
            h.update(struct.pack("<I", len(vocab[i])) + vocab[i])
        want = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in g["merges"]]
        ok_m, ok_v = merges == want, h.hexdigest() == g["vocab_sha256"]
        return {"parity": ok_m and ok_v, "golden": f"tests/golden/scale/{p.name}", "merges_equal": ok_m,
                "vocab_sha256_equal": ok_v}
    return {"parity": None, "golden": None,
            "note": f"no scale golden for n={n} seed={seed} flavour={flavour} vocab={vocab_size}"}


def cpu_baselines(args, path, vocab, merges, L):
    """The CPU legs (oracle/cpu_bench.py) in a child process that never touches the GPU: the
    pure-Python port on corpus.en in full and on 16 / 64 MB samples (one core each), the
    pure-Python encode port over 1 M-character pieces (a pool of cores), and the exact C oracle
    on the full bench corpus (C3; one counting thread per core of the host's share).  Returned as
    cpu_baseline; `value` is the largest training sample whose extrapolation follows a cost curve
    measured on that sample (one core, as the reference runs)."""
    import hashlib
    import struct
    import subprocess
    from bpe_amd import Tokenizer
    tmp = pathlib.Path(tempfile.mkdtemp(prefix="bpe355_cpu_"))
    mj, rj = tmp / "merges.json", tmp / "cpu.json"
    mj.write_text(json.dumps({"merges": [(a.hex(), b.hex()) for a, b in merges],
                              "vocab": [(i, b.hex()) for i, b in vocab.items()]}))
    from oracle.cpu_bench import host_threads
    procs = args.cpu_procs or host_threads()
    cmd = [sys.executable, "-m", "oracle.cpu_bench", "--corpus", str(path), "--vocab", str(args.vocab),
           "--samples-mb", args.cpu_samples_mb, "--cap-s", str(args.cpu_cap_s), "--merges-json", str(mj),
           "--encode-mb", str(args.cpu_encode_mb), "--procs", str(procs), "--out", str(rj)]
    gname = golden_name(path.stat().st_size, args.seed, args.flavour, args.vocab)
    # the exact leg on the bench corpus itself (the headline config) only on request:
    # its single-threaded merge loop alone takes ~5 min at C3 (profiles/r06/exact_cpu_C3.json),
    # past the few minutes a default bench run may take; by default it runs on C2 (2 GB, ~3 s)
    if gname and args.exact_c3:
        cmd += ["--exact-corpus", str(path), "--exact-golden", gname]
    subprocess.run(cmd, cwd=ROOT, check=True, timeout=900)
    r = json.loads(rj.read_text())
    for f in (mj, rj):
        f.unlink()
    tmp.rmdir()
    # the port's ids for piece 0 must be the GPU encoder's (a 1 M-character parity check)
    with open(path, "rb") as f:
        head = f.read(8 << 20).decode("utf-8", errors="ignore")
    piece0 = head[:r["encode"]["piece0_chars"]]
    gpu_ids = Tokenizer(vocab, merges, [EOT]).encode(piece0)
    gpu_sha = hashlib.sha256(struct.pack(f"<{len(gpu_ids)}I", *gpu_ids)).hexdigest()
    # the headline sample: the largest whose extrapolation is validated (complete, or corrected
    # along a cost curve measured on those very bytes)
    ok = [x for x in r["train"] if x.get("complete") or x.get("growth_validated")]
    big = max(ok or r["train"], key=lambda x: x["bytes"])
    cores = os.cpu_count()
    enc = r["encode"]
    c3 = None   # the newest committed run of the exact leg at C3 (tools/gpu_r06.sh exactc3, the box's host)
    c3s = sorted((p for p in (ROOT / "profiles").glob("r[0-9]*") if (p / "exact_cpu_C3.json").exists()),
                 key=lambda p: int(p.name[1:]) if p.name[1:].isdigit() else -1)
    c3f = c3s[-1] / "exact_cpu_C3.json" if c3s else None
    if c3f is not None and not (r.get("exact") or {}).get("config") == "train_C3":
        c3 = dict(json.loads(c3f.read_text()), source_file=str(c3f.relative_to(ROOT)),
                  note="committed run of this leg on the full C3 corpus (BASELINE configs[2]), not measured in "
                       "this bench run: python bench.py --exact-c3 measures it (~5 min of CPU legs)")
    return {
        "value": big["MBps"], "unit": "MB/s", "cores": 1, "kind": "port", "host_cpus": cores,
        "host_share_threads": r.get("threads"),
        "sample": (f"first {big['bytes'] / 1e6:.1f} MB of the same corpus at vocab {args.vocab}: "
                   f"oracle/cpu_ref.py (pure-Python port with the reference's structure) on 1 core "
                   f"(host shows {cores}); count {big['t_count_s']:.1f}s + build {big['t_build_s']:.1f}s "
                   f"measured, {big['rounds_done']}/{big['rounds_total']} merge rounds measured in "
                   f"{args.cpu_cap_s:.0f}s ({big['ms_per_round']:.1f} ms/round), the rest extrapolated along the "
                   f"port's measured cost curve (x{big.get('growth_factor') or 1:.2f} on the flat rate; "
                   f"oracle/cpu_port_growth.json, a complete run on these bytes). The port keeps the vocab's "
                   f"byte strings in a set where the reference's vocab.py:29 scans dict values, so it is "
                   f"faster than the reference itself (C1: see c1)"),
        "value_flat": big.get("MBps_flat"),
        "rounds_measured_frac": big["rounds_measured_frac"], "merges_per_s": big["merges_per_s"],
        "samples": r["train"],
        "c1": dict(r["c1"], note="tests/fixtures corpus.en at vocab 500 (reference test_train_bpe.py:28), "
                                 "in full, 1 core"),
        "encode": dict(enc, kind="port", cores=enc["procs"], matches_gpu_piece0=gpu_sha == r["encode_piece0_ids_sha256"],
                       note="cpu_ref.Encoder (tokenizer.py:92-138) over 1 M-character pieces encoded on their "
                            "own (encode.py:31-36), a pool of processes"),
        "exact_cpu": dict(r.get("exact") or {}, kind="port (C oracle)",
                          note="oracle/bpe_oracle.c (exact incremental trainer, lazy max-heap argmax) on the full "
                               "corpus of its config (the bench corpus itself when it is C3, BASELINE configs[2]): "
                               f"one counting thread per core of this host's share ({procs} of the {cores} the host "
                               "shows; OMP_NUM_THREADS / affinity), single-threaded exact merge loop; checked "
                               "against the scale golden"),
        "exact_cpu_c3": c3,
    }


def main():
    args = parse()
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    multiproc = env_world > 1
    if multiproc and args.gpus != env_world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} ranks were launched")
    import torch
    import torch.distributed as dist
    import bpe_amd
    from bpe_amd import _lib, train_bpe, train_bpe_device, Tokenizer
    from bpe_amd.train import last_train_stats

    n_dev = torch.cuda.device_count()
    if not multiproc and args.gpus > n_dev:
        sys.exit(f"bench.py: --gpus {args.gpus} but only {n_dev} GPU(s) are visible to this process")
    torch.cuda.set_device(local_rank)
    L = _lib.lib()
    _lib.require_device()
    comm = None
    if multiproc:
        from bpe_amd.dist import Communicator
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        comm = Communicator.from_torch(local_rank)   # RCCL: one all-gather of the word tables
    else:
        bpe_amd.set_num_gpus(args.gpus)

    def barrier():
        if multiproc:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if not multiproc:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ---------------------------------------------------------------- the corpus file
    n = max(1, int(args.bytes) // BLOCK) * BLOCK
    path = pathlib.Path(args.corpus_dir) / f"bpe355_bench_s{args.seed}_f{args.flavour}_{n}.txt"
    need_file = not args.no_file or not args.no_cpu_baseline
    if need_file and rank == 0 and not (path.exists() and path.stat().st_size == n):
        t = time.perf_counter()
        write_corpus(L, path, n, args.seed, args.flavour)
        print(f"[bench] wrote {n / 1e9:.2f} GB corpus to {path} in {time.perf_counter() - t:.1f}s",
              file=sys.stderr, flush=True)
    barrier()

    def note(msg):   # progress on stderr (a long run stays visibly alive)
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    def train_file():   # steps repeat, so the corpus buffer and the counter's scratch are kept
        if multiproc:
            return train_bpe(path, args.vocab, [EOT], comm=comm, split_file=True, keep_device_buffers=True)
        return train_bpe(path, args.vocab, [EOT], keep_device_buffers=True)

    # ---------------------------------------------------------------- end to end: file -> merges
    stats = []
    elapsed = 0.0
    if not args.no_file:
        L.bpe_set_timing(0)
        for _ in range(args.warmup):
            vocab, merges = train_file()
        L.bpe_set_timing(0 if args.no_timing else 1)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            vocab, merges = train_file()
            stats.append(last_train_stats())
        torch.cuda.synchronize()
        barrier()
        elapsed = max_over_ranks(time.perf_counter() - t0)
        L.bpe_set_timing(0)
        note(f"{args.steps} timed file steps: {elapsed / args.steps * 1e3:.1f} ms per step")

    def traffic_of(kernel):
        """HBM bytes per launch from the committed PMC passes (tools/gpu_pmc_all.sh): the newest
        round's profiles/rNN/traffic.json that has the kernel"""
        rounds = sorted((p for p in (ROOT / "profiles").glob("r[0-9]*") if (p / "traffic.json").exists()),
                        key=lambda p: int(p.name[1:]), reverse=True)
        for d in rounds:
            v = json.loads((d / "traffic.json").read_text()).get(kernel)
            if v is not None:
                return v, f"profiles/{d.name}/traffic.json (committed PMC passes, not measured in this run)"
        return None, None

    def merge_roofline(st, note):
        """the dominant kernel by device time, k_merge_batch (the merge-apply rewrite of a trip):
        algorithmic bytes per launch (the members' posting-list entries, 4 B each, and the slot
        words they name at the table's mean slot size; every slot on a full scan; the long words)
        over its mean launch duration, both from the launches HIP events time on the library's
        stream (stamped by the kernel's own dispatch packet; one trip in 8)"""
        a = {k: sum(x[k] for x in st) / len(st) for k in st[0]}
        if a["merge_kernel_launches"] <= 0:
            return None
        us = a["merge_kernel_ms"] * 1e3 / a["merge_kernel_launches"]
        bpl = a["merge_kernel_bytes"] / a["merge_kernel_launches"]
        achieved = bpl / (us * 1e-6) / 1e9
        tr, tsrc = traffic_of("k_merge_batch")
        return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": tr, "traffic_source": tsrc,
                "kernel": "k_merge_batch", "launches_per_step": int(a["n_trips"]),
                "timed_launches": int(sum(x["merge_kernel_launches"] for x in st)),
                "avg_launch_us": round(us, 3), "bytes_per_launch": round(bpl), "note": note}

    def roofline_of(st, per_step_launches, note):
        """k_count2 (pre-tokenize + count): algorithmic bytes (the corpus, read once) / its device
        time, event-timed on the library's stream by the launches' own dispatch packets"""
        a = {k: sum(x[k] for x in st) / len(st) for k in st[0]}
        if a["count_kernel_ms"] <= 0:
            return None
        kms, kb = a["count_kernel_ms"], a["count_kernel_bytes"]
        achieved = kb / (kms / 1e3) / 1e9
        traffic, tsrc = traffic_of("k_count2")
        return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": tsrc,
                "kernel": "k_count2", "launches_per_step": per_step_launches,
                "timed_launches": len(st) * (per_step_launches or 1), "avg_launch_us": round(kms * 1e3, 3),
                "bytes_per_launch": kb, "note": note}
    if not args.no_file:
        n_gpus = int(stats[-1]["n_gpus"])
    else:
        n_gpus = env_world if multiproc else 1

    # ---------------------------------------------------------------- corpus resident in HBM
    device_resident = None
    corpus = None
    need_corpus = not (args.no_device_resident and args.no_encode)
    if need_corpus and (multiproc or n_gpus == 1):
        world = env_world
        blocks = n // BLOCK
        b0, b1 = blocks * rank // world, blocks * (rank + 1) // world
        slab = (b1 - b0) * BLOCK
        corpus = torch.empty(max(1, slab), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        _lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(corpus.data_ptr()), slab, args.seed,
                                             args.flavour, b0, None), "synth")
        torch.cuda.synchronize()
    dstats = []
    if corpus is not None and not args.no_device_resident:
        def train_dev():
            return train_bpe_device(corpus.data_ptr(), slab, args.vocab, [EOT], comm=comm,
                                    keep_device_buffers=True)
        for _ in range(args.warmup):
            v2, m2 = train_dev()
        L.bpe_set_timing(0 if args.no_timing else 1)
        barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            v2, m2 = train_dev()
            dstats.append(last_train_stats())
        torch.cuda.synchronize()
        barrier()
        el = max_over_ranks(time.perf_counter() - t1)
        L.bpe_set_timing(0)
        if args.no_file:
            vocab, merges = v2, m2
            elapsed = el
            stats = dstats
        assert m2 == merges and v2 == vocab, "device-resident result differs from the file result"
        s0 = dstats[-1]
        davg = {k: sum(x[k] for x in dstats) / len(dstats) for k in dstats[0]}   # mean of the K steps
        device_resident = {
            "value": round(n / (el / args.steps) / 1e6, 2), "unit": "MB/s",
            "ms_per_step": round(el / args.steps * 1e3, 2),
            "phases_ms": {k: round(davg[k], 2) for k in ("t_prepare_ms", "t_count_ms", "t_exchange_ms",
                                                          "t_words_ms", "t_merge_ms", "t_total_ms")},
            "count_aggregation": {"records": s0["n_count_records"], "batches": s0["n_count_batches"],
                                  "ms": round(s0["count_reduce_ms"], 2)}}

    ms_per_step = elapsed / args.steps * 1e3
    value = n / (elapsed / args.steps) / 1e6
    rounds = len(merges)
    avg = {k: sum(x[k] for x in stats) / len(stats) for k in stats[0]}
    trips = avg["n_trips"]
    merge_loop = {
        "rounds": rounds, "trips": int(trips),
        "ms": round(avg["t_merge_ms"], 2),
        "us_per_trip": round(avg["t_merge_ms"] * 1e3 / trips, 2) if trips else None,
        "us_per_round": round(avg["t_merge_ms"] * 1e3 / max(1, rounds), 3),
        "k_merge_batch_us": (round(avg["merge_kernel_ms"] * 1e3 / avg["merge_kernel_launches"], 2)
                             if avg["merge_kernel_launches"] else None),
        "k_merge_batch_bytes_per_launch": (round(avg["merge_kernel_bytes"] / avg["merge_kernel_launches"])
                                           if avg["merge_kernel_launches"] else None),
        # the rewrite's algorithmic bytes over its mean launch: far below HBM, the loop is
        # latency-bound (merge-loop probe)
        "k_merge_batch_GBps": (round(avg["merge_kernel_bytes"] / (avg["merge_kernel_ms"] * 1e6), 1)
                               if avg["merge_kernel_launches"] and avg["merge_kernel_ms"] else None),
        # a trip is three dependent launches; an empty kernel boundary costs 1.4-2.6 us on this part
        # (tools/microbench/launch_floor.hip), so 3 x 1.4 us is the floor of a trip that did nothing
        "launch_floor_us_per_trip": 4.2,
    }
    # the roofline line: k_count2 over the HBM-resident corpus (one launch per step, the launches
    # rocprofv3 --no-file profiles see); without that run, the file path's per-segment launches
    if dstats:
        roofline_count = roofline_of(dstats, 1, ("corpus in HBM, one launch per step" +
                                                 ("; rank 0's slab" if n_gpus > 1 else "")))
        roofline = merge_roofline(dstats, "corpus in HBM; sampled launches of the timed steps")
    else:
        roofline_count = roofline_of(stats, None, "file path: summed over its per-segment launches")
        roofline = merge_roofline(stats, "file path; sampled launches of the timed steps")

    # ---------------------------------------------------------------- encode MB/s (device)
    encode = None
    if corpus is not None and not args.no_encode:
        tok = Tokenizer(vocab, merges, [EOT])
        h = tok._device()
        out = torch.empty(slab, dtype=torch.int32, device="cuda")
        n_out = ctypes.c_size_t(0)

        def enc():
            _lib.check(L.bpe_tok_encode_device(h, ctypes.c_void_p(corpus.data_ptr()), slab,
                                               ctypes.c_void_p(out.data_ptr()), ctypes.byref(n_out),
                                               None), "encode")
        enc()   # warm-up pass
        enc_reps = 3
        barrier()
        torch.cuda.synchronize()
        te = time.perf_counter()
        for _ in range(enc_reps):
            enc()
        torch.cuda.synchronize()
        barrier()
        te = max_over_ranks(time.perf_counter() - te) / enc_reps
        # B_enc = N + 4 n_ids (corpus read once, u32 ids written once)
        b_enc = slab + 4 * int(n_out.value)
        encode = {"value": round(n / te / 1e6, 1), "unit": "MB/s", "ids_rank0": int(n_out.value),
                  "seconds": round(te, 4), "passes": enc_reps, "scope": "corpus in HBM -> ids in HBM (mean of the passes)",
                  "roofline": {"bound": "hbm", "achieved": round(b_enc / te / 1e9, 2), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(b_enc / te / 1e9 / HBM_PEAK_GBS, 4),
                               "bytes": b_enc, "note": "whole encode (all its kernels) on rank 0's slab"}}
        del out
        if not args.no_file and not multiproc and n_gpus == 1:
            # the drop-in dataset encoder end to end: file -> np.uint16 ids in host memory
            # (encode.py:31-37 without the torch.save), 1 M-character pieces
            from bpe_amd.encode import encode_file, last_phases_ms
            runs = []
            for _ in range(2):   # the first call also sizes the tokenizer's kept device buffers
                torch.cuda.synchronize()
                tf0 = time.perf_counter()
                ids16 = encode_file(tok, path, keep_device_buffers=True)
                tf = time.perf_counter() - tf0
                runs.append((tf, int(ids16.size), {k: round(v, 1) for k, v in last_phases_ms.items()}))
                del ids16
            tf, k16, ph = runs[-1]
            encode["end_to_end"] = {"value": round(n / tf / 1e6, 1), "unit": "MB/s", "seconds": round(tf, 3),
                                    "ids": k16, "phases_ms": ph,
                                    "first_call": {"seconds": round(runs[0][0], 3), "phases_ms": runs[0][2]},
                                    "scope": "encode_file(path): file read -> np.uint16 ids in host memory, "
                                             "1 M-character pieces (encode.py:31-37); the second of two calls"}

    # ---------------------------------------------------------------- CPU baseline (rank 0, N=1)
    cpu = None
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline:
        note("GPU legs done; CPU baselines (oracle/cpu_bench.py)")
        t_cpu = time.perf_counter()
        cpu = cpu_baselines(args, path, vocab, merges, L)
        note(f"CPU baselines: {time.perf_counter() - t_cpu:.1f} s")

    if rank == 0:
        s0 = stats[-1]
        par = "1 GPU"
        if n_gpus > 1:
            par = (f"{n_gpus} GPUs ({'one process per GPU, RCCL' if multiproc else 'one process, RCCL'}): "
                   "one slab of the file per GPU, one all-gather of the unique-word tables, merge "
                   "loop on the union")
        line = {
            "metric": ("BPE train input MB/s (32k vocab), train_bpe(path) end to end" if not args.no_file else
                       "BPE train input MB/s (32k vocab), corpus in HBM (profiling run, --no-file)"),
            "value": round(value, 2), "unit": "MB/s", "n_gpus": n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (bpe_synth_corpus_host OWT-like deterministic text, page-cache-warm file)",
            "config": {"workload": "train_bpe OWT-sized synthetic corpus, vocab 32000, "
                                   "special <|endoftext|> (BASELINE configs[2])",
                       "corpus_bytes": n, "vocab_size": args.vocab, "merges": rounds,
                       "seed": args.seed, "flavour": args.flavour, "parallelism": par},
            # the timed steps' result against the committed scale golden of this corpus
            "parity": golden_parity(n, args.seed, args.flavour, args.vocab, vocab, merges),
            "merges_per_s": round(rounds / (avg["t_merge_ms"] / 1e3), 1) if avg["t_merge_ms"] else None,
            "device_resident": device_resident,
            "merge_loop": merge_loop,
            "encode": encode,
            "roofline": roofline,
            "roofline_count": roofline_count,
            "cpu_baseline": cpu,
            # mean over the K timed steps (the load varies step to step with the host's page
            # cache and PCIe); the library's own clock, so ms_per_step - t_total_ms is the call's
            # ctypes, result-conversion and Python overhead
            "phases_ms": {k: round(avg[k], 2) for k in ("t_load_ms", "t_prepare_ms", "t_count_ms",
                                                         "t_exchange_ms", "t_words_ms", "t_merge_ms",
                                                         "t_total_ms")},
            "load_ms_per_step": [round(x["t_load_ms"], 1) for x in stats],
            "counters": {k: s0[k] for k in ("n_pretokens", "n_words", "n_exchanged_words",
                                            "n_pairs_final", "n_rebuilds", "n_rounds_device",
                                            "n_rounds_host", "n_index_builds", "n_trips",
                                            "n_count_records", "n_count_batches")},
        }
        print(json.dumps(line), flush=True)
        if not args.keep_corpus and need_file:
            path.unlink(missing_ok=True)
    if multiproc:
        dist.barrier()
        comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
