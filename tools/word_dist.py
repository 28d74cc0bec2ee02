"""Word-frequency profile of the bench corpus (a prefix of bpe_synth_corpus seed 2, flavour 0):
how much of the token stream the top-K distinct words cover, by word length -- sizing data for the
count kernel's caches and record format.  Timing-free analysis tool (GPU box: bpe_word_counts).

  python tools/word_dist.py [bytes]
"""
import ctypes, json, sys
sys.path[:0] = ["transformer-lm_amd", "."]
import numpy as np
from bpe_amd import _lib

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 2_000_000_000
L = _lib.lib()
buf = np.empty(n, dtype=np.uint8)
_lib.check(L.bpe_synth_corpus_host(ctypes.c_void_p(buf.ctypes.data), n, 2, 0, 0, 16), "synth")
arr, k, _keep = _lib.c_strings(["<|endoftext|>"])
blob = ctypes.c_void_p()
bn = ctypes.c_size_t()
_lib.check(L.bpe_word_counts(ctypes.cast(buf.ctypes.data, ctypes.c_char_p), n, arr, k, ctypes.byref(blob),
                             ctypes.byref(bn)), "word_counts")
raw = ctypes.string_at(blob.value, bn.value)
L.bpe_blob_free(blob)
lens, cnts = [], []
p = 0
mv = memoryview(raw)
while p < len(raw):
    ln = int.from_bytes(mv[p:p + 4], "little")
    lens.append(ln)
    cnts.append(int.from_bytes(mv[p + 4 + ln:p + 12 + ln], "little"))
    p += 12 + ln
lens = np.array(lens)
cnts = np.array(cnts, dtype=np.int64)
o = np.argsort(-cnts, kind="stable")
lens, cnts = lens[o], cnts[o]
tot = int(cnts.sum())
cum = np.cumsum(cnts)
out = {"bytes": n, "distinct": int(len(cnts)), "tokens_ge2": tot,
       "short_le7_share_of_tokens": round(float(cnts[lens <= 7].sum() / tot), 4),
       "long_gt16_share_of_tokens": round(float(cnts[lens > 16].sum() / tot), 4),
       "coverage_topK": {}, "tail_le7_share": {}}
for K in (256, 512, 2048, 8192, 32768, 65536, 262144, 1 << 20, 1 << 22):
    if K >= len(cnts):
        break
    out["coverage_topK"][K] = round(float(cum[K - 1] / tot), 4)
    tail = cnts[K:]
    out["tail_le7_share"][K] = round(float(tail[lens[K:] <= 7].sum() / max(1, tail.sum())), 4)
hist = np.bincount(np.minimum(lens, 17), weights=cnts, minlength=18)
out["token_len_hist"] = {int(i): round(float(hist[i] / tot), 4) for i in range(2, 18)}
lw = np.nonzero(lens > 16)[0][:12]
out["top_long_words"] = [[int(lens[i]), int(cnts[i])] for i in lw]
out["long_distinct"] = int((lens > 16).sum())
print(json.dumps(out))
