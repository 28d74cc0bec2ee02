"""Quality of short_hash (stage.h) on the bench corpus's distinct words of <= 16 bytes, the old
(four 64-bit multiplies) against the new (two) form: full-hash collisions, the spread of the bits
each consumer uses (record bins: top 12; LDS word cache sets: bits 41..48; the word table: low bits,
linear probing at load 1/2) and the mean probe length.  CPU only (numpy + regex); analysis tool.

  python tools/hash_quality.py [MB]
"""
import ctypes, json, sys
sys.path[:0] = ["transformer-lm_amd", "."]
import numpy as np
import regex
from bpe_amd import _lib

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def mix64(z):
    z = z ^ (z >> np.uint64(30)); z = z * np.uint64(0xBF58476D1CE4E5B9)
    z = z ^ (z >> np.uint64(27)); z = z * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def old_hash(lo, hi, ln):
    return mix64(lo ^ mix64(hi ^ (ln << np.uint64(56)) ^ np.uint64(0x9E3779B97F4A7C15)))


def new_hash(lo, hi, ln):
    z = lo ^ ((hi ^ ln) * np.uint64(0x9E3779B97F4A7C15))
    z = z ^ (z >> np.uint64(32))
    z = z * np.uint64(0xD6E8FEB86659FD93)
    return z ^ (z >> np.uint64(32))


def probe_mean(slots_bits, h):
    cap = 1 << slots_bits
    occ = np.zeros(cap, dtype=bool)
    total = 0
    for s in (h & np.uint64(cap - 1)).astype(np.int64):
        d = 0
        while occ[(s + d) & (cap - 1)]:
            d += 1
        occ[(s + d) & (cap - 1)] = True
        total += d + 1
    return total / len(h)


def main():
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 40
    n = int(mb * 1e6) // 4096 * 4096
    buf = (ctypes.c_char * n)()
    assert _lib.lib().bpe_synth_corpus_host(ctypes.addressof(buf), n, 2, 0, 0, 8) == 0
    text = bytes(buf).decode("utf-8")
    pat = regex.compile(r"""'(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")
    words = {w.encode() for w in pat.findall(text)}
    words = [w for w in words if 2 <= len(w) <= 16]
    lo = np.array([int.from_bytes(w[:8], "little") for w in words], dtype=np.uint64)
    hi = np.array([int.from_bytes(w[8:16], "little") for w in words], dtype=np.uint64)
    ln = np.array([len(w) for w in words], dtype=np.uint64)
    out = {"sample_MB": mb, "distinct_words_le16": len(words)}
    for name, f in (("old", old_hash), ("new", new_hash)):
        h = f(lo, hi, ln)
        bins = np.bincount((h >> np.uint64(52)).astype(np.int64), minlength=4096)
        sets = np.bincount(((h >> np.uint64(41)) & np.uint64(255)).astype(np.int64), minlength=256)
        exp_b, exp_s = len(h) / 4096, len(h) / 256
        bits = int(np.ceil(np.log2(len(h)))) + 1
        sub = h[: min(len(h), 200000)]
        out[name] = {"full_collisions": int(len(h) - len(np.unique(h))),
                     "bins12_chi2_per_dof": round(float(((bins - exp_b) ** 2 / exp_b).sum() / 4095), 3),
                     "cache_sets_chi2_per_dof": round(float(((sets - exp_s) ** 2 / exp_s).sum() / 255), 3),
                     "low_bits_probe_mean_load_half": round(probe_mean(int(np.ceil(np.log2(len(sub)))) + 1, sub), 4),
                     "table_bits": bits}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
