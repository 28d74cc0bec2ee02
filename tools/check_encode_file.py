"""encode_file (the overlapped bulk path) on the bench corpus against one device encode of the
whole text cut at piece starts computed here with numpy (1 M-character pieces): piece starts,
id count and ids.  usage: python tools/check_encode_file.py [bytes]"""
import ctypes, pathlib, sys, time
import os as _os
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
sys.path[:0] = [_os.path.join(_ROOT, "transformer-lm_amd"), _ROOT]
import numpy as np
import torch
from bpe_amd import _lib, train_bpe_device, Tokenizer
from bpe_amd.encode import encode_file, last_phases_ms, read_file_device
from bench import write_corpus

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 11_899_998_208
K = 1 << 20
L = _lib.lib()
path = pathlib.Path("/tmp/bpe355_check.txt")
write_corpus(L, path, n, 2, 0)
mm = np.memmap(path, dtype=np.uint8, mode="r")
t0 = time.time()
starts, base = [], 0
for lo in range(0, n, 1 << 28):
    blk = np.asarray(mm[lo:lo + (1 << 28)])
    idx = np.flatnonzero((blk & 0xC0) != 0x80)
    c = base + np.arange(idx.size, dtype=np.int64)
    starts.append(idx[c % K == 0] + lo)
    base += idx.size
starts = np.concatenate(starts).astype(np.uint64)
print(f"numpy starts {starts.size} in {time.time() - t0:.1f}s, chars {base}", flush=True)
d = read_file_device(path)
ns = ctypes.c_size_t(0)
_lib.check(L.bpe_utf8_chunk_starts_device(ctypes.c_void_p(d.data_ptr()), n, K, None, 0, ctypes.byref(ns), None), "cs")
dev = np.zeros(ns.value, dtype=np.uint64)
_lib.check(L.bpe_utf8_chunk_starts_device(ctypes.c_void_p(d.data_ptr()), n, K, dev.ctypes.data, ns.value,
                                          ctypes.byref(ns), None), "cs")
print("device starts", dev.size, "equal", dev.size == starts.size and bool((dev == starts).all()), flush=True)
if dev.size == starts.size and not (dev == starts).all():
    i = int(np.flatnonzero(dev != starts)[0]); print("first diff at piece", i, dev[i], starts[i])
vocab, merges = train_bpe_device(d.data_ptr(), n, 32000, ["<|endoftext|>"])
tok = Tokenizer(vocab, merges, ["<|endoftext|>"])
out = torch.empty(n, dtype=torch.int32, device="cuda")
k = ctypes.c_size_t(0)
arr = starts.astype(np.uint64)
_lib.check(L.bpe_tok_encode_chunks_device(tok._device(), ctypes.c_void_p(d.data_ptr()), n, arr.ctypes.data, arr.size,
                                          ctypes.c_void_p(out.data_ptr()), ctypes.byref(k), None), "enc")
want = out[:k.value].to(torch.int32).cpu().numpy().astype(np.uint16)
del out
print("chunks encode ids", k.value, flush=True)
import os
tr = "/tmp/bpe355_trace.txt"
os.environ["BPE355_ENC_TRACE"] = tr
for rep in range(2):
    if os.path.exists(tr): os.unlink(tr)
    t0 = time.time()
    got = encode_file(tok, path)
    print(f"encode_file ids {got.size} in {time.time() - t0:.3f}s phases {last_phases_ms}", flush=True)
    regs = [l.split() for l in open(tr)]
    print("".join(open(tr)), flush=True)
    if got.size == want.size and (got == want).all():
        print("equal"); continue
    m = min(got.size, want.size)
    bad = np.flatnonzero(got[:m] != want[:m])
    print("first id mismatch at", int(bad[0]) if bad.size else m, "of", m, "mismatches", bad.size, flush=True)
    # each region on its own through the chunked encode: which one differs, and how
    koff = 0
    for r in regs:
        a, b, kk = int(r[1]), int(r[2]), int(r[4])
        buf = torch.empty(b - a, dtype=torch.uint8, device="cuda")
        buf.copy_(d[a:b]); torch.cuda.synchronize()
        cut = starts[(starts > a) & (starts < b)] - np.uint64(a)
        o2 = torch.empty(b - a, dtype=torch.int32, device="cuda")
        k2 = ctypes.c_size_t(0)
        cut = np.ascontiguousarray(cut, dtype=np.uint64)
        _lib.check(L.bpe_tok_encode_chunks_device(tok._device(), ctypes.c_void_p(buf.data_ptr()), b - a, cut.ctypes.data,
                                                  cut.size, ctypes.c_void_p(o2.data_ptr()), ctypes.byref(k2), None), "enc")
        torch.cuda.synchronize()
        exp = o2[:k2.value].cpu().numpy().astype(np.uint16)
        seg = got[koff:koff + kk]
        mm = min(exp.size, seg.size)
        bb = np.flatnonzero(exp[:mm] != seg[:mm])
        print(f"region [{a}, {b}) pipeline ids {kk} alone {k2.value} equal {exp.size == seg.size and bb.size == 0} "
              f"first diff {int(bb[0]) if bb.size else None}", flush=True)
        koff += kk
        del buf, o2
    # the piece holding the first mismatch: alone on the device, and saved for an oracle check
    i = int(bad[0])
    lens = np.zeros(max(vocab) + 1, dtype=np.int64)
    for t_, bs in vocab.items(): lens[t_] = len(bs)
    P = int(lens[want[:i].astype(np.int64)].sum())
    j = int(np.searchsorted(starts, np.uint64(P), side="right")) - 1
    a, b = int(starts[j]), int(starts[j + 1]) if j + 1 < starts.size else n
    ids_before = int(lens[want.astype(np.int64)].cumsum().searchsorted(a, side="right"))
    print(f"mismatch byte {P} in piece {j} [{a}, {b}); want ids before the piece {ids_before}", flush=True)
    buf = torch.empty(b - a, dtype=torch.uint8, device="cuda"); buf.copy_(d[a:b]); torch.cuda.synchronize()
    o2 = torch.empty(b - a, dtype=torch.int32, device="cuda"); k2 = ctypes.c_size_t(0)
    _lib.check(L.bpe_tok_encode_device(tok._device(), ctypes.c_void_p(buf.data_ptr()), b - a,
                                       ctypes.c_void_p(o2.data_ptr()), ctypes.byref(k2), None), "enc")
    torch.cuda.synchronize()
    alone = o2[:k2.value].cpu().numpy().astype(np.uint16)
    w = want[ids_before:ids_before + alone.size]
    g = got[ids_before:ids_before + alone.size]
    print("piece alone ids", alone.size, "== want slice", bool((w == alone).all()), "== got slice", bool((g == alone).all()))
    import json
    os.makedirs("gpurun_out/r03q", exist_ok=True)
    open("gpurun_out/r03q/piece.bin", "wb").write(d[a:b].cpu().numpy().tobytes())
    json.dump({"alone": alone.tolist(), "want": w.tolist(), "got": g.tolist(),
               "vocab": {str(t_): bs.hex() for t_, bs in vocab.items()},
               "merges": [[x.hex(), y.hex()] for x, y in merges]}, open("gpurun_out/r03q/piece.json", "w"))
    break
path.unlink()
