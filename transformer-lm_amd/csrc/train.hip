// BPE merge loop on the device.
//
// Reference semantics (models/tokenizer/train.py):
//   31-49    words -> byte ids, pair histogram weighted by word count
//   183-189  rounds = vocab_size - len(vocab); best = max(pairs, key=(count, (bytes a, bytes b)))
//            over every key still in the dict (count 0 included); stop early only if empty
//   190-224  new = a + b; rewrite every word left to right, non-overlapping; per occurrence
//            (x, a) -= c, (x, new) += c for the rewritten left neighbour x, and
//            (b, y) -= c, (new, y) += c for the original right neighbour y
//   226-228  pop best; append (a, b) to merges
// Tokens are identified by their bytes (vocab.py:29): a merge whose bytes already exist
// reuses that token's id (token dedupe below).
//
// HBM layout of the unique-word table (the stream every round reads):
//   words live in fixed-width SLOTS of W token ids, W in {8, 16, 32, 64}: slot[0] = current
//   length, slot[1..] = ids, the unused tail filled with a sentinel id that never matches a
//   pair.  A 16-byte slot (u16 ids) is one dwordx4 load per word, coalesced across the wave,
//   and the pair test is W-2 register compares with no branch on the length.  Words longer
//   than 63 ids sit in a CSR side table.  Counts (u64) are a parallel array read only on a hit.
//   Words that shrink to one id drop out, and words migrate to narrower slots, at compaction.
//
// Per round, three kernels on one HIP stream (host checks state once per batch of rounds):
//   K1 k_merge  : every workgroup reduces K3's per-block partials to the round's best pair and
//                 resolves the new token id (hash map over token bytes); block 0 records the merge.
//                 Then all workgroups rewrite the words containing (a, b) and accumulate, per
//                 neighbour token, the deltas L[x] (left) and R[y] (right) as int64.
//   [one all-reduce of L/R over ranks when the corpus is sharded]
//   K2 k_apply  : 4 threads per token: (x,a)-=L[x], (x,new)+=L[x], (b,y)-=R[y], (new,y)+=R[y]
//                 on the pair hash table; touched keys become present; increments that lift a
//                 key across the threshold T append it to the candidate list C.
//   K3 k_argmax : argmax over C of (count, bytes a, bytes b) -> per-block partials; bytes
//                 compare by 8-byte big-endian prefix, the pool only on equal prefixes.
// Every key with count >= T is in C, so max(C) is the global max whenever it is >= T;
// otherwise (or when C has bloated) the host rebuilds C with a fresh T.  Zero-count keys that
// are still present are the reference's leftover dict keys; once no positive count remains
// (every word is one token) the reference pops them in descending byte order, which the host
// reproduces.
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <unordered_map>

#include "internal.h"
#include "prims.h"

namespace bpe {

namespace {

constexpr unsigned kPresent = 1u, kInC = 2u;
enum : int { HALT_NONE = 0, HALT_REBUILD = 1, HALT_DONE = 2, HALT_HOST = 3 };
enum : unsigned { ERR_PAIRS_FULL = 1u, ERR_C_FULL = 2u, ERR_POOL = 4u };
constexpr unsigned long long kPolyP = 0x100000001B3ULL * 0x9E3779B97F4A7C15ULL | 1ULL;
constexpr int kNumCls = 4;
constexpr int kHistReplicas = 16;

struct RoundState {
    int halt;
    int round;
    int n_rounds;
    int ntok;
    long long T;
    unsigned nC, capC, c_limit, probe_merge_done;   // probe_*_done: BPE355_PROBE workgroup counters
    unsigned nC_base;           // |C| before this round's appends (set by k_merge)
    int cur_round, cur_ntok;    // for k_apply_argmax: this round, and ntok after it (k_merge)
    unsigned cur_a, cur_b, cur_new, cur_slot;
    long long cur_cnt;
    int new_is_new;
    unsigned err;
    unsigned n_single;
    unsigned n_single_new;      // batched: words the current trip's rewrite made single (the apply folds
                                // them into n_single, which the trip's own select phase reads)
    unsigned pool_used, pool_cap;
    unsigned long long pair_used;
    unsigned long long scan_slots;
    int nparts;                 // batched: apply workgroups whose top-M lists part[] holds
    unsigned probe_apply_done;
    unsigned long long* probe;  // BPE355_PROBE: phase stamps of sampled trips (else null)
    // batched rounds (k_select): the host's limits, checked before every trip
    int host_round;             // hand back to the host at this round (compaction schedule)
    unsigned single_limit;      // ... or when this many words became one token (compaction)
    unsigned max_len;           // longest word (bytes): the most one new token adds to the pool
    int max_batch;              // merges allowed per trip (1: one merge per trip)
    unsigned long long pair_limit;   // ... or when the pair table could pass this many keys
    long long narrow_limit;     // the merge sums a member's cells in 32-bit LDS words while count(P1) is
                                // below this: 2^32 (a cell never exceeds count(P_j) <= count(P1)), 0 under
                                // the test knob BPE355_LDS_CELLS=0 (every cell to the global 64-bit atomics)
};

struct Partial {
    long long cnt;
    unsigned long long ka, kb;   // key8 of a and of b (first 8 bytes, big-endian)
    unsigned slot, a, b, pad;
};

struct PairsDev {
    unsigned long long* key;  // ((a << 32) | b) + 1, 0 = empty
    long long* cnt;
    unsigned* flag;           // kPresent | kInC
    size_t mask;
    uint4* C;                 // candidate list: {slot, a, b, 0} (ids carried so the argmax loads
                              // the slot's count and the tokens' prefixes in one step)
};

struct ToksDev {
    uint8_t* pool;
    uint32_t* off;
    uint32_t* len;
    unsigned long long* hash;  // polynomial hash of the bytes
    unsigned long long* pw;    // P^len
    unsigned long long* key8;  // first 8 bytes, big-endian, zero padded
    unsigned long long* map;   // token dedupe map: (hash >> 32) << 32 | id + 1 (map_entry)
    uint32_t map_mask;
};

__host__ __device__ constexpr int slot_w(int c) { return 8 << c; }   // 8, 16, 32, 64 ids
__host__ __device__ inline int class_for(unsigned len) {
    return len <= 7 ? 0 : len <= 15 ? 1 : len <= 31 ? 2 : len <= 63 ? 3 : kNumCls;
}

template <class TokT>
struct SlotCls {
    TokT* slot;                  // n * slot_w(c) ids
    unsigned long long* cnt;
    unsigned n, blk0, nblk, pad;
};

template <class TokT>
struct WordsDev {
    SlotCls<TokT> c[kNumCls];
    TokT* ltok;                  // long words (> 63 ids): CSR
    unsigned long long* lbeg;
    uint32_t* llen;
    unsigned long long* lcnt;
    unsigned ln, lblk0, lnblk, pad;
    unsigned off[kNumCls + 1];   // flat word index: class c holds [off[c], off[c+1])
};

// Posting index over the slot words, rebuilt at every compaction: list[beg[t], beg[t]+len[t])
// holds the flat index of every word that contained token t at build time.  A token created
// later gets (beg, len) of the smaller covering list of its two parts (a word that contains it
// contained both parts when it was formed) -- stored per token, so the merge kernel finds its
// list in one dependent load; a token re-created through token dedupe (its bytes reached by
// another split) is marked uncovered (len = kNoAnc) until the next build.
constexpr unsigned kNoAnc = 0xffffffffu;
struct IndexDev {
    const uint32_t* list;
    uint32_t* beg;
    uint32_t* len;
    unsigned full_threshold;   // lists longer than this are cheaper to replace by a full scan
    unsigned n_slot_words;
};

template <class TokT> __host__ __device__ constexpr TokT sentinel() { return (TokT)~(TokT)0; }

// bytes(x) vs bytes(y) for tokens whose 8-byte prefixes are equal: -1 / 0 / +1
__device__ __forceinline__ int cmp_tok_tail(const uint8_t* __restrict__ pool, const uint32_t* __restrict__ off,
                                         const uint32_t* __restrict__ len, unsigned x, unsigned y) {
    const unsigned lx = len[x], ly = len[y], m = lx < ly ? lx : ly;
    const uint8_t* px = pool + off[x];
    const uint8_t* py = pool + off[y];
    for (unsigned i = 8; i < m; ++i)
        if (px[i] != py[i]) return px[i] < py[i] ? -1 : 1;
    return lx < ly ? -1 : (lx > ly ? 1 : 0);
}

// The reference's max key (count, bytes a, bytes b) (train.py:187-189).  Byte strings compare
// by their zero-padded big-endian 8-byte prefix first: a smaller prefix means smaller bytes;
// only equal prefixes of different tokens need the bytes themselves (rare: long tokens, or a
// prefix relation like "ab" vs "ab\0").
struct Cand {
    long long cnt;
    unsigned long long ka, kb;
    unsigned slot, a, b;
};
__device__ __forceinline__ bool cand_better(const Cand& x, const Cand& y, const uint8_t* pool,
                                            const uint32_t* off, const uint32_t* len) {
    if (x.cnt != y.cnt) return x.cnt > y.cnt;
    if (x.a != y.a) {
        if (x.ka != y.ka) return x.ka > y.ka;
        return cmp_tok_tail(pool, off, len, x.a, y.a) > 0;
    }
    if (x.b != y.b) {
        if (x.kb != y.kb) return x.kb > y.kb;
        return cmp_tok_tail(pool, off, len, x.b, y.b) > 0;
    }
    return false;
}
__device__ __forceinline__ Cand cand_none() { return Cand{LLONG_MIN, 0, 0, 0, 0, 0}; }
__device__ __forceinline__ Cand shfl_xor_cand(const Cand& c, int o) {
    Cand r;
    r.cnt = __shfl_xor(c.cnt, o);
    r.ka = __shfl_xor(c.ka, o);
    r.kb = __shfl_xor(c.kb, o);
    r.slot = __shfl_xor(c.slot, o);
    r.a = __shfl_xor(c.a, o);
    r.b = __shfl_xor(c.b, o);
    return r;
}


// Stores of the trip kernels: write-through (sc1) or plain.  A plain store leaves a dirty line in
// the XCD's L2 that the end of the kernel writes back before the next launch can start; a
// write-through store leaves while the kernel still runs (MI355X_MICROARCH.md: sc1 stores drop the
// line from L2).  Build knobs BPE355_WT_APPLY (pair-table updates) and BPE355_WT_MERGE (word
// rewrites and the cell clear).
#ifndef BPE355_WT_APPLY
#define BPE355_WT_APPLY 0
#endif
#ifndef BPE355_WT_MERGE
#define BPE355_WT_MERGE 0
#endif
template <bool WT, class T>
__device__ __forceinline__ void st_wt(T* p, T v) {
    if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
template <class T> __device__ __forceinline__ void st_apply(T* p, T v) { st_wt<BPE355_WT_APPLY != 0>(p, v); }
template <class T> __device__ __forceinline__ void st_merge(T* p, T v) { st_wt<BPE355_WT_MERGE != 0>(p, v); }

// ------------------------------------------------------------------ pair table
// returns the slot of key (inserting it if absent, *inserted = 1), or ~0 if the table is full
__device__ __forceinline__ size_t pair_slot(const PairsDev& P, unsigned long long key,
                                            RoundState* st, bool* inserted) {
    size_t s = mix64(key) & P.mask;
    *inserted = false;
    for (size_t probe = 0; probe <= P.mask; ++probe) {
        unsigned long long k = P.key[s];
        if (k == key) return s;
        if (k == 0) {
            k = atomicCAS(&P.key[s], 0ULL, key);
            if (k == 0) {
                atomicAdd(&st->pair_used, 1ULL);
                *inserted = true;
                return s;
            }
            if (k == key) return s;
        }
        s = (s + 1) & P.mask;
    }
    atomicOr(&st->err, ERR_PAIRS_FULL);
    return ~(size_t)0;
}

__device__ __forceinline__ unsigned long long pair_key(unsigned p, unsigned q) {
    return ((((unsigned long long)p) << 32) | q) + 1ULL;
}

// frequencies[(p, q)] -= d  (a missing key would be created, as defaultdict does)
__device__ __forceinline__ void pair_dec(const PairsDev& P, RoundState* st, unsigned p, unsigned q,
                                         long long d) {
    bool ins;
    const size_t s = pair_slot(P, pair_key(p, q), st, &ins);
    if (s == ~(size_t)0) return;
    atomicAdd((unsigned long long*)&P.cnt[s], (unsigned long long)(-d));
    if (ins) atomicOr(&P.flag[s], kPresent);
}

// frequencies[(p, q)] += d; the key is present from now on.  Returns the slot so the caller
// can list it as touched: whether it enters the candidate list is decided from its FINAL
// count in k_argmax -- never from the order the atomics happened to land in, which differs
// between ranks and would let replicated pair tables disagree about C.
__device__ __forceinline__ size_t pair_inc(const PairsDev& P, RoundState* st, unsigned p, unsigned q,
                                           long long d) {
    bool ins;
    const size_t s = pair_slot(P, pair_key(p, q), st, &ins);
    if (s == ~(size_t)0) return s;
    atomicAdd((unsigned long long*)&P.cnt[s], (unsigned long long)d);
    atomicOr(&P.flag[s], kPresent);
    return s;
}

// ------------------------------------------------------------------ token helpers
__device__ __forceinline__ unsigned long long concat_key8(const ToksDev& K, unsigned a, unsigned b) {
    const unsigned la = K.len[a];
    const unsigned long long ka = K.key8[a];
    if (la >= 8) return ka;
    return ka | (K.key8[b] >> (8 * la));
}

__device__ __forceinline__ uint8_t concat_byte(const ToksDev& K, unsigned a, unsigned la,
                                               unsigned b, unsigned i) {
    return i < la ? K.pool[K.off[a] + i] : K.pool[K.off[b] + (i - la)];
}

__device__ bool equals_concat(const ToksDev& K, unsigned x, unsigned a, unsigned b) {
    const unsigned la = K.len[a], ln = la + K.len[b];
    if (K.len[x] != ln) return false;
    const uint8_t* px = K.pool + K.off[x];
    for (unsigned i = 0; i < ln; ++i)
        if (px[i] != concat_byte(K, a, la, b, i)) return false;
    return true;
}

// The token dedupe map (vocab.py:29: a merge whose bytes exist reuses that id): open addressing
// on mix64(hash), entries tagged with the hash's high half, so a probe that meets another token
// moves on without loading that token's hash
__device__ __forceinline__ unsigned long long map_entry(unsigned long long h, unsigned id) {
    return (h & 0xffffffff00000000ull) | (unsigned long long)(id + 1);
}
// the id of the token whose bytes are a + b (hash h, ln bytes), or ~0
__device__ __forceinline__ unsigned map_find(const ToksDev& K, unsigned long long h, unsigned ln, unsigned a,
                                             unsigned b) {
    unsigned s = (unsigned)mix64(h) & K.map_mask;
    for (unsigned long long e = K.map[s]; e != 0; s = (s + 1) & K.map_mask, e = K.map[s]) {
        if ((e >> 32) != (h >> 32)) continue;
        const unsigned id = (unsigned)e - 1;
        if (K.hash[id] == h && K.len[id] == ln && equals_concat(K, id, a, b)) return id;
    }
    return ~0u;
}

// ------------------------------------------------------------------ word rewrite
// The reference's in-place merge of one word (train.py:196-224): t[0..len) -> t[0..j).
// Per occurrence: the left neighbour is already rewritten (t[j-1]); the right one is the
// original t[r+2].  With `pad`, the freed tail is refilled with the sentinel.
// Per-occurrence deltas are keyed by the neighbour token: cell 2x = L[x] for (x,a)-=c and
// (x,new)+=c, cell 2x+1 = R[x] for (b,x)-=c and (new,x)+=c.  Cells of ids below kLdsLR (the
// bytes and the first merges: neighbours hot enough to serialize a global atomic) are summed
// in LDS per workgroup and flushed once; the others go out directly.
constexpr unsigned kLdsLR = 512;

// (Applying the four pair updates of a cell inside the merge kernel instead was measured
// slower: one hit's updates form a serial chain on one thread; see DESIGN.md.)
typedef __attribute__((address_space(3))) unsigned long long LdsU64;   // an LDS cell
struct DeltaSink {
    unsigned long long* LR;     // global delta cells (all-reduced when sharded) for k_apply
    LdsU64* lds;
    __device__ __forceinline__ void add(unsigned cell, unsigned long long c) const {
        if (cell < 2 * kLdsLR) __hip_atomic_fetch_add(&lds[cell], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else atomicAdd(&LR[cell], c);
    }
};

template <class TokT, class Sink>
__device__ __forceinline__ uint32_t rewrite_word(TokT* __restrict__ t, uint32_t len, TokT a, TokT b,
                                                 TokT nw, unsigned long long c, const Sink& D, bool pad) {
    uint32_t j = 0, r = 0;
    while (r < len) {
        const TokT x = t[r];
        if (x == a && r + 1 < len && t[r + 1] == b) {
            if (j > 0) D.add(2u * (unsigned)t[j - 1], c);           // (x,a)-=c, (x,new)+=c
            if (r + 2 < len) D.add(2u * (unsigned)t[r + 2] + 1, c);  // (b,y)-=c, (new,y)+=c
            t[j++] = nw;
            r += 2;
        } else {
            t[j++] = x;
            ++r;
        }
    }
    if (pad)
        for (uint32_t k = j; k < len; ++k) t[k] = sentinel<TokT>();
    return j;
}

// rewrite_word for a slot word already in registers (e: the slot, e[0] = length, sentinel-padded):
// the matches are found on the registers (every index a compile-time constant), so the only
// memory traffic is the stores of the shifted tail, not a load per token
template <class TokT, int W, class Sink>
__device__ __forceinline__ uint32_t rewrite_slot(const TokT (&e)[W], TokT* __restrict__ s, TokT a, TokT b,
                                                 TokT nw, unsigned long long c, const Sink& D) {
    const TokT sent = sentinel<TokT>();
    uint32_t j = 0;      // output tokens so far
    TokT prev = sent;    // the last output token
    bool skip = false;   // this position is the b of the previous match
#pragma unroll
    for (int q = 1; q < W; ++q) {
        const TokT x = e[q];
        if (x == sent) break;
        if (skip) { skip = false; continue; }
        if (q + 1 < W && x == a && e[q + 1 < W ? q + 1 : q] == b) {
            if (j > 0) D.add(2u * (unsigned)prev, c);                      // (x,a)-=c, (x,new)+=c
            if (q + 2 < W && e[q + 2 < W ? q + 2 : q] != sent)
                D.add(2u * (unsigned)e[q + 2 < W ? q + 2 : q] + 1, c);     // (b,y)-=c, (new,y)+=c
            st_merge(&s[1 + j], nw);
            prev = nw;
            skip = true;
        } else {
            if (j != (uint32_t)(q - 1)) st_merge(&s[1 + j], x);
            prev = x;
        }
        ++j;
    }
    for (uint32_t p = j; p < (uint32_t)e[0]; ++p) st_merge(&s[1 + p], sent);
    st_merge(&s[0], (TokT)j);
    return j;
}

// Several members' rewrites of one slot word in registers, then one compacting store (batched
// trips).  rewrite_slot per member needed the word re-read from memory between members: a
// dependent load per extra member on the thread's chain.  Here member j's matches replace
// e[q] by new_j and leave a hole at q + 1 (a bit of `hole`, its value the sentinel), so every
// index stays a compile-time constant.  A hole only ever follows a new token, which is no
// member's a or b, so no match spans a hole and no hole starts a match; the left neighbour of a
// match is e[q - 1], or e[q - 2] behind a hole; the right one is e[q + 2] (e[q + 1] is b, an
// old token, so q + 2 is never a hole).  Matches of one member cannot overlap (a != b for
// k > 1), and the ascending pass sees the already-rewritten left and the original right, as
// rewrite_word (the reference's loop, train.py:196-224) does.  Returns the new length.
template <class TokT, int W, class PA, class SinkOf>
__device__ __forceinline__ uint32_t rewrite_slot_members(TokT (&e)[W], TokT* __restrict__ s, unsigned hits,
                                                         PA ta, PA tb, PA tn,
                                                         unsigned long long c, const SinkOf& sink_of) {
    static_assert(W <= 64, "one hole bit per position");
    const TokT sent = sentinel<TokT>();
    const uint32_t len0 = (uint32_t)e[0];
    unsigned long long hole = 0, chg = 0;
    while (hits) {
        const int j = __builtin_ctz(hits);
        hits &= hits - 1;
        const TokT a = (TokT)ta[j], b = (TokT)tb[j], nw = (TokT)tn[j];
        const auto D = sink_of(j);
#pragma unroll
        for (int q = 1; q + 1 < W; ++q) {
            if (e[q] == a && e[q + 1] == b) {
                if (q > 1) {
                    // e[q - 1], or e[q - 2] behind a hole (arithmetic, not a select of two array
                    // loads, which would keep e[] out of registers)
                    unsigned left = (unsigned)e[q - 1];
                    if (q > 2) {
                        const unsigned h = 0u - (unsigned)((hole >> (q - 1)) & 1);
                        left ^= (left ^ (unsigned)e[q > 2 ? q - 2 : 1]) & h;
                    }
                    D.add(2u * left, c);                                          // (x,a)-=c, (x,new)+=c
                }
                if (q + 2 < W && e[q + 2 < W ? q + 2 : q] != sent)
                    D.add(2u * (unsigned)e[q + 2 < W ? q + 2 : q] + 1, c);        // (b,y)-=c, (new,y)+=c
                e[q] = nw;
                e[q + 1] = sent;
                hole |= 1ull << (q + 1);
                chg |= 1ull << q;
            }
        }
    }
    uint32_t j = 0;   // output tokens so far
#pragma unroll
    for (int q = 1; q < W; ++q) {   // (no early exit: a data-dependent one un-unrolls the loop)
        if ((uint32_t)q <= len0 && !((hole >> q) & 1)) {
            if (j != (uint32_t)(q - 1) || ((chg >> q) & 1)) st_merge(&s[1 + j], e[q]);
            ++j;
        }
    }
    for (uint32_t p = j; p < len0; ++p) st_merge(&s[1 + p], sent);
    st_merge(&s[0], (TokT)j);
    return j;
}

// scan one slot class: U words in flight per thread, one 16-byte load per 16 bytes of slot
template <class TokT, int C, class Sink>
__device__ __forceinline__ void scan_class(const SlotCls<TokT>& S, unsigned bi, TokT a, TokT b,
                                           TokT nw, const Sink& D, unsigned& singles) {
    constexpr int W = slot_w(C);
    constexpr int V = W * (int)sizeof(TokT) / 16;
    constexpr int U = V == 1 ? 4 : (V == 2 ? 2 : 1);
    const unsigned stride = S.nblk * blockDim.x;
    for (unsigned base = bi * blockDim.x + threadIdx.x; base < S.n; base += stride * U) {
        uint4 r[U][V];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned i = base + u * stride;
#pragma unroll
            for (int v = 0; v < V; ++v)
                r[u][v] = i < S.n ? reinterpret_cast<const uint4*>(S.slot + (size_t)i * W)[v]
                                  : make_uint4(~0u, ~0u, ~0u, ~0u);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned i = base + u * stride;
            TokT e[W];
            __builtin_memcpy(e, r[u], sizeof(e));
            bool hit = false;
#pragma unroll
            for (int k = 1; k + 1 < W; ++k) hit |= (e[k] == a) & (e[k + 1] == b);
            if (hit) {
                const uint32_t j = rewrite_slot(e, S.slot + (size_t)i * W, a, b, nw, S.cnt[i], D);
                singles += (j < 2);
            }
        }
    }
}

// one word of class C addressed directly (index-list mode)
template <class TokT, int C, class Sink>
__device__ __forceinline__ void merge_one(const SlotCls<TokT>& S, unsigned i, TokT a, TokT b,
                                          TokT nw, const Sink& D, unsigned& singles) {
    constexpr int W = slot_w(C);
    constexpr int V = W * (int)sizeof(TokT) / 16;
    uint4 r[V];
#pragma unroll
    for (int v = 0; v < V; ++v) r[v] = reinterpret_cast<const uint4*>(S.slot + (size_t)i * W)[v];
    const unsigned long long c = S.cnt[i];   // issued with the slot: no extra dependent load on a hit
    TokT e[W];
    __builtin_memcpy(e, r, sizeof(e));
    bool hit = false;
#pragma unroll
    for (int k = 1; k + 1 < W; ++k) hit |= (e[k] == a) & (e[k + 1] == b);
    if (hit) {
        const uint32_t j = rewrite_slot(e, S.slot + (size_t)i * W, a, b, nw, c, D);
        singles += (j < 2);
    }
}

// ------------------------------------------------------------------ K1: merge
struct BestShared {
    int stop;
    unsigned a, b, nw, slot, isnew;
    long long cnt;
    unsigned long long hash, k8;
    int round, ntok;
    unsigned ln, list_beg, list_len, use_list, cov_beg, cov_len;
};

template <class TokT>
__global__ void __launch_bounds__(256) k_merge(RoundState* __restrict__ st,
                                               const Partial* __restrict__ part, int nparts,
                                               PairsDev P, ToksDev K, WordsDev<TokT> W,
                                               IndexDev X, unsigned long long* __restrict__ LR,
                                               uint32_t* __restrict__ m_a, uint32_t* __restrict__ m_b,
                                               uint32_t* __restrict__ m_new, uint32_t* __restrict__ m_mode,
                                               long long* __restrict__ m_cnt) {
    __shared__ BestShared sb;
    __shared__ unsigned long long l_lr[2 * kLdsLR];
    __shared__ Cand s_part[4];
    const int tid = threadIdx.x;
    for (unsigned k = tid; k < 2 * kLdsLR; k += blockDim.x) l_lr[k] = 0;
    {   // all four waves reduce the argmax partials (a few independent loads per thread)
        Cand pp = cand_none();
        for (int i = tid; i < nparts; i += blockDim.x) {
            const Partial q = part[i];
            const Cand c{q.cnt, q.ka, q.kb, q.slot, q.a, q.b};
            if (cand_better(c, pp, K.pool, K.off, K.len)) pp = c;
        }
        for (int o = 32; o > 0; o >>= 1) {
            const Cand oc = shfl_xor_cand(pp, o);
            if (cand_better(oc, pp, K.pool, K.off, K.len)) pp = oc;
        }
        if ((tid & 63) == 0) s_part[tid >> 6] = pp;
    }
    __syncthreads();
    if (tid < 64) {
        // Every workgroup redundantly decides the round (no extra launch, no grid sync).  The
        // loads are grouped by dependency level so the chain is ~4 memory latencies long:
        // state + partials | token metadata, posting-list ids | map slot, list bounds | (dedupe)
        const int halt = st->halt, round = st->round, ntok = st->ntok;
        const int n_rounds = st->n_rounds;
        const unsigned nC = st->nC, c_limit = st->c_limit;   // only k_apply_argmax appends to C
        const long long T = st->T;
        Cand pp = s_part[0];
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
            if (cand_better(s_part[k], pp, K.pool, K.off, K.len)) pp = s_part[k];
        int stop = HALT_NONE;
        if (halt) stop = -1;
        else if (round >= n_rounds) stop = HALT_DONE;
        else if (nC > c_limit) stop = HALT_REBUILD;   // C bloated: re-threshold
        else if (pp.cnt < T) stop = HALT_REBUILD;     // max(C) < T: re-threshold
        if (tid == 0) {
            sb.stop = stop;
            if (!stop) {
                const unsigned a = pp.a, b = pp.b;
                // level 1: everything keyed by a or b
                const unsigned long long ha = K.hash[a], pb = K.pw[b], hb = K.hash[b];
                const unsigned la = K.len[a], lb = K.len[b];
                const unsigned long long ka = pp.ka, kb = pp.kb;
                const unsigned za = X.len[a], zb = X.len[b];   // kNoAnc (uncovered) sorts last
                const unsigned ba = X.beg[a], bbg = X.beg[b];
                sb.a = a; sb.b = b; sb.slot = pp.slot; sb.cnt = pp.cnt;
                sb.hash = ha * pb + hb;
                sb.ln = la + lb;
                sb.k8 = la >= 8 ? ka : (ka | (kb >> (8 * la)));
                sb.round = round; sb.ntok = ntok;
                // which words can contain (a, b): the smaller covering posting list, or all
                const bool pick_a = za <= zb;
                const unsigned lu = pick_a ? za : zb, bu = pick_a ? ba : bbg;
                sb.use_list = lu != kNoAnc && lu <= X.full_threshold;
                sb.list_beg = sb.use_list ? bu : 0;
                sb.list_len = sb.use_list ? lu : 0;
                sb.cov_beg = bu;
                sb.cov_len = lu;
            }
        }
    }
    __syncthreads();
    if (sb.stop) {
        if (blockIdx.x == 0 && tid == 0 && sb.stop > 0) st->halt = sb.stop;
        return;
    }
    // While thread 0 resolves the new token's id (token dedupe: does bytes(a) + bytes(b) exist
    // already? usually an empty map slot), every thread pulls its first posting-list entry and
    // that word's slot line toward the CU; the barrier below waits for both.
    {
        const unsigned i = blockIdx.x * blockDim.x + tid;
        if (sb.use_list && blockIdx.x < W.lblk0 && i < sb.list_len) {
            const unsigned f = X.list[sb.list_beg + i];
            const TokT* line = f < W.off[1] ? W.c[0].slot + (size_t)f * slot_w(0)
                             : f < W.off[2] ? W.c[1].slot + (size_t)(f - W.off[1]) * slot_w(1)
                             : f < W.off[3] ? W.c[2].slot + (size_t)(f - W.off[2]) * slot_w(2)
                                            : W.c[3].slot + (size_t)(f - W.off[3]) * slot_w(3);
            (void)*reinterpret_cast<const volatile unsigned*>(line);   // kept: volatile
        }
        if (tid == 0) {
            const unsigned a = sb.a, b = sb.b, ln = sb.ln, ntok = (unsigned)sb.ntok;
            const unsigned long long h = sb.hash;
            const unsigned old = map_find(K, h, ln, a, b);
            const unsigned nw = old != ~0u ? old : ntok;
            sb.nw = nw;
            sb.isnew = nw == ntok;
            if (!sb.isnew) sb.cov_len = kNoAnc;   // dedupe: uncovered until the next build
        }
    }
    __syncthreads();
    const unsigned a = sb.a, b = sb.b, nw = sb.nw;

    if (blockIdx.x == 0) {  // record the merge, pop the pair, register a new token
        if (tid == 0) {
            st->nC_base = st->nC;     // C entries k_apply_argmax may scan without racing its appends
            st->cur_round = sb.round;
            st->cur_ntok = sb.ntok + (int)sb.isnew;
            P.cnt[sb.slot] = 0;                       // byte_pair_frequencies.pop(best_pair)
            atomicAnd(&P.flag[sb.slot], ~kPresent);   // (no other update touches this key)
            st->cur_a = a; st->cur_b = b; st->cur_new = nw; st->cur_slot = sb.slot;
            st->cur_cnt = sb.cnt; st->new_is_new = (int)sb.isnew;
            m_a[sb.round] = a; m_b[sb.round] = b; m_new[sb.round] = nw;
            if (m_cnt) m_cnt[sb.round] = sb.cnt;
            m_mode[sb.round] = sb.use_list ? sb.list_len : 0xffffffffu;
            X.beg[nw] = sb.cov_beg;
            X.len[nw] = sb.cov_len;
        }
        if (sb.isnew) {
            const unsigned la = K.len[a], ln = la + K.len[b];
            const unsigned base = st->pool_used;
            if (base + ln <= st->pool_cap) {
                for (unsigned i = tid; i < ln; i += blockDim.x)
                    K.pool[base + i] = concat_byte(K, a, la, b, i);
            }
            __syncthreads();
            if (tid == 0) {
                if (base + ln > st->pool_cap) atomicOr(&st->err, ERR_POOL);
                K.off[nw] = base; K.len[nw] = ln;
                K.hash[nw] = sb.hash; K.pw[nw] = K.pw[a] * K.pw[b]; K.key8[nw] = sb.k8;
                st->pool_used = base + ln;
            }
        }
    }

    // rewrite every word containing (a, b): this block's share of one slot class
    unsigned singles = 0;
    const unsigned bid = blockIdx.x;
    const TokT ta = (TokT)a, tb = (TokT)b, tn = (TokT)nw;
    const DeltaSink D{LR, (LdsU64*)l_lr};
    if (sb.use_list && bid < W.lblk0) {
        // index mode: only the words on the posting list (a gather of their slots)
        const uint32_t* L = X.list + sb.list_beg;
        for (unsigned i = bid * blockDim.x + tid; i < sb.list_len; i += W.lblk0 * blockDim.x) {
            const unsigned f = L[i];
            if (f < W.off[1]) merge_one<TokT, 0>(W.c[0], f, ta, tb, tn, D, singles);
            else if (f < W.off[2]) merge_one<TokT, 1>(W.c[1], f - W.off[1], ta, tb, tn, D, singles);
            else if (f < W.off[3]) merge_one<TokT, 2>(W.c[2], f - W.off[2], ta, tb, tn, D, singles);
            else merge_one<TokT, 3>(W.c[3], f - W.off[3], ta, tb, tn, D, singles);
        }
    } else if (bid < W.c[1].blk0) {
        if (bid < W.c[0].blk0 + W.c[0].nblk)
            scan_class<TokT, 0>(W.c[0], bid - W.c[0].blk0, ta, tb, tn, D, singles);
    } else if (bid < W.c[2].blk0) {
        scan_class<TokT, 1>(W.c[1], bid - W.c[1].blk0, ta, tb, tn, D, singles);
    } else if (bid < W.c[3].blk0) {
        scan_class<TokT, 2>(W.c[2], bid - W.c[2].blk0, ta, tb, tn, D, singles);
    } else if (bid < W.lblk0) {
        scan_class<TokT, 3>(W.c[3], bid - W.c[3].blk0, ta, tb, tn, D, singles);
    } else if (bid < W.lblk0 + W.lnblk) {
        for (unsigned i = (bid - W.lblk0) * blockDim.x + tid; i < W.ln; i += W.lnblk * blockDim.x) {
            const uint32_t len = W.llen[i];
            if (len < 2) continue;
            TokT* t = W.ltok + W.lbeg[i];
            bool hit = false;
            for (uint32_t k = 0; k + 1 < len && !hit; ++k) hit = (t[k] == ta) & (t[k + 1] == tb);
            if (!hit) continue;
            const uint32_t j = rewrite_word(t, len, ta, tb, tn, W.lcnt[i], D, false);
            W.llen[i] = j;
            singles += (j < 2);
        }
    }
    singles = wave_sum(singles);   // words that became one token (rare: no contention)
    if ((tid & 63) == 0 && singles) atomicAdd(&st->n_single, singles);
    __syncthreads();
    for (unsigned k = tid; k < 2 * kLdsLR; k += blockDim.x) {
        const unsigned long long v = l_lr[k];
        if (v) atomicAdd(&LR[k], v);
    }
}

// ------------------------------------------------------------------ K2: apply + argmax
// One launch applies the round's deltas and takes the argmax for the next round.
//  * cell threads (4 per token x, op = g & 3):  0 (x,a) -= L[x]   1 (x,new) += L[x]
//                                               2 (b,x) -= R[x]   3 (new,x) += R[x]
//    Only four keys can receive two of these updates -- (b,a), (b,new), (new,a), (new,new) --
//    and thread 0 applies those; every other key has ONE updater, so counts are updated with
//    plain loads/stores and the updater sees the key's final count: it evaluates the key for
//    the argmax and admits it to C when an increment lifts it to T (identical on every rank).
//  * C threads scan the candidate list C (entries before this round's appends).  An entry is
//    skipped iff this round's cells touch it -- exactly the rule above -- and its updater
//    evaluates it instead; the others' counts do not change during the launch.
// The cells are double-buffered by round parity: this launch reads LR (this round) and clears
// LRold (the previous round's, already applied).  Round state is written only into fields the
// other kernel reads (k_merge -> cur_*, this kernel -> round/ntok), so no grid-wide ordering.
// apply `delta` to the key (p, q) (its only updater this round); present if incremented or
// created (a decrement of a missing key creates it, as the reference's defaultdict does)
__device__ __forceinline__ size_t pair_update(const PairsDev& P, RoundState* st, unsigned p, unsigned q,
                                              long long delta, bool inc, long long* c_out, unsigned* f_out) {
    const unsigned long long key = pair_key(p, q);
    const size_t s0 = mix64(key) & P.mask;
    // the home slot's key, count and flags in one step: at load <= 1/2 the first probe usually
    // decides, so the usual chain is one dependent load
    const unsigned long long k0 = P.key[s0];
    long long c = P.cnt[s0];
    unsigned f = P.flag[s0];
    bool ins = false;
    size_t s = s0;
    if (k0 != key) {
        s = pair_slot(P, key, st, &ins);
        if (s == ~(size_t)0) return s;
        if (ins) {          // a slot this call claimed was empty: count and flags are 0
            c = 0;
            f = 0;
        } else {
            c = P.cnt[s];
            f = P.flag[s];
        }
    }
    c += delta;
    P.cnt[s] = c;
    if ((inc || ins) && !(f & kPresent)) {
        f |= kPresent;
        P.flag[s] = f;
    }
    *c_out = c;
    *f_out = f;
    return s;
}

// pair_update with the home slot's key, count and flags already loaded (k0, c0, f0): the
// caller issues several keys' home-slot loads before finishing any of them
// Inserted keys are counted in *n_ins (the caller adds them to st->pair_used once per workgroup:
// one same-address atomic per insert serialises thousands of them at the end of a trip).
__device__ __forceinline__ size_t pair_update_from(const PairsDev& P, RoundState* st, unsigned p, unsigned q,
                                                   long long delta, bool inc, unsigned long long k0, long long c0,
                                                   unsigned f0, long long* c_out, unsigned* f_out, unsigned& n_ins) {
    const unsigned long long key = pair_key(p, q);
    size_t s = mix64(key) & P.mask;
    long long c = c0;
    unsigned f = f0;
    bool ins = false;
    if (k0 != key) {   // the probe from the home slot on, its first key already known
        unsigned long long k = k0;
        size_t probe = 0;
        for (;;) {
            if (k == key) break;
            if (k == 0) {
                k = atomicCAS(&P.key[s], 0ULL, key);
                if (k == 0) {
                    ++n_ins;
                    ins = true;
                    break;
                }
                if (k == key) break;
            }
            if (++probe > P.mask) {
                atomicOr(&st->err, ERR_PAIRS_FULL);
                return ~(size_t)0;
            }
            s = (s + 1) & P.mask;
            k = P.key[s];
        }
        if (ins) {          // a slot this call claimed was empty: count and flags are 0
            c = 0;
            f = 0;
        } else {
            c = P.cnt[s];
            f = P.flag[s];
        }
    }
    c += delta;
    st_apply(&P.cnt[s], c);
    if ((inc || ins) && !(f & kPresent)) {
        f |= kPresent;
        st_apply(&P.flag[s], f);
    }
    *c_out = c;
    *f_out = f;
    return s;
}

constexpr unsigned kApplyThreads = 256;    // large workgroups: fewer argmax partials for k_merge
__global__ void __launch_bounds__(kApplyThreads) k_apply_argmax(RoundState* __restrict__ st, PairsDev P, ToksDev K,
                                                      const unsigned long long* __restrict__ LR,
                                                      unsigned long long* __restrict__ LRold,
                                                      unsigned ntb, unsigned cell_blocks,
                                                      Partial* __restrict__ part) {
    __shared__ Cand sw[kApplyThreads / 64];
    const unsigned g = blockIdx.x * blockDim.x + threadIdx.x;
    const bool cell_thread = blockIdx.x < cell_blocks;
    const unsigned x = g >> 2, op = g & 3;
    // the cell load needs no state (ntb bounds every id k_merge can have written)
    const long long d = cell_thread && x < ntb ? (long long)LR[2 * (size_t)x + (op >> 1)] : 0;
    if (cell_thread && (op & 1) && x < ntb) LRold[2 * (size_t)x + (op >> 1)] = 0;
    Cand best = cand_none();
    if (!st->halt) {
        const unsigned a = st->cur_a, b = st->cur_b, nw = st->cur_new;
        const long long T = st->T;
        // a key this thread updated: candidate if present and >= T; increments may admit it
        auto consider = [&](size_t s, unsigned p, unsigned q, unsigned long long ka, unsigned long long kb,
                            long long c, unsigned f, bool inc) -> bool {
            if (s == ~(size_t)0 || !(f & kPresent) || c < T) return false;
            const Cand cand{c, ka, kb, (unsigned)s, p, q};
            if (cand_better(cand, best, K.pool, K.off, K.len)) best = cand;
            if (inc && !(f & kInC)) {
                P.flag[s] = f | kInC;
                return true;
            }
            return false;
        };
        bool add = false;
        uint4 add_e = make_uint4(0, 0, 0, 0);
        if (cell_thread) {
            if (d) {
                const bool special = (op <= 1) ? (x == b || x == nw) : (x == a || x == nw);
                const bool popped = (op == 0 && x == a && a == b) || (op == 2 && x == b && a == b);
                if (!special && !popped) {
                    const unsigned p = op == 0 ? x : op == 1 ? x : op == 2 ? b : nw;
                    const unsigned q = op == 0 ? a : op == 1 ? nw : x;
                    const bool inc = op & 1;
                    const unsigned long long ka = K.key8[p], kb = K.key8[q];   // issued with the probe
                    long long c;
                    unsigned f;
                    const size_t s = pair_update(P, st, p, q, inc ? d : -d, inc, &c, &f);
                    if (consider(s, p, q, ka, kb, c, f, inc)) { add = true; add_e = make_uint4((unsigned)s, p, q, 0u); }
                }
            }
            if (g == 0) {   // the four keys two cells can update
                const long long Lb = (long long)LR[2 * (size_t)b], Ln = (long long)LR[2 * (size_t)nw];
                const long long Ra = (long long)LR[2 * (size_t)a + 1], Rn = (long long)LR[2 * (size_t)nw + 1];
                struct Sp { unsigned p, q; long long dec, inc; };
                const Sp sp[4] = {{b, a, a == b ? 0 : Lb + Ra, 0},   // (a,b) itself when a == b: popped
                                  {b, nw, Rn, Lb},
                                  {nw, a, Ln, Ra},
                                  {nw, nw, 0, Ln + Rn}};
                // (the decrements use the same cells as their single-updater twins above)
                for (int k = 0; k < 4; ++k) {
                    const bool touched = (k == 0) ? (a != b && (Lb || Ra))
                                       : (k == 1) ? (Lb || Rn)
                                       : (k == 2) ? (Ln || Ra)
                                                  : (Ln || Rn);
                    if (!touched) continue;
                    long long c;
                    unsigned f;
                    const bool inc = sp[k].inc != 0;
                    const size_t s = pair_update(P, st, sp[k].p, sp[k].q, sp[k].inc - sp[k].dec, inc, &c, &f);
                    if (consider(s, sp[k].p, sp[k].q, K.key8[sp[k].p], K.key8[sp[k].q], c, f, inc)) {
                        // thread 0 appends its own admissions here (at most four)
                        const unsigned idx = atomicAdd(&st->nC, 1u);
                        if (idx < st->capC) P.C[idx] = make_uint4((unsigned)s, sp[k].p, sp[k].q, 0u);
                        else atomicOr(&st->err, ERR_C_FULL);
                    }
                }
            }
        } else {
            // C scan: entries untouched this round keep their counts during this launch
            const unsigned nC = st->nC_base;
            const unsigned stride = (gridDim.x - cell_blocks) * blockDim.x;
            for (unsigned i = g - cell_blocks * blockDim.x; i < nC; i += stride) {
                const uint4 e = P.C[i];
                const unsigned p = e.y, q = e.z;
                const unsigned f = P.flag[e.x];
                const long long c = P.cnt[e.x];
                const unsigned long long ka = K.key8[p], kb = K.key8[q];
                bool touched = false;
                if (q == a || q == nw) touched = LR[2 * (size_t)p] != 0;
                if (!touched && (p == b || p == nw)) touched = LR[2 * (size_t)q + 1] != 0;
                if (touched || !(f & kPresent)) continue;
                const Cand cand{c, ka, kb, e.x, p, q};
                if (cand_better(cand, best, K.pool, K.off, K.len)) best = cand;
            }
        }
        const unsigned idx = wave_append(add, &st->nC);
        if (add) {
            if (idx < st->capC) P.C[idx] = add_e;
            else atomicOr(&st->err, ERR_C_FULL);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const Cand oc = shfl_xor_cand(best, o);
        if (cand_better(oc, best, K.pool, K.off, K.len)) best = oc;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sw[w] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
            if (cand_better(sw[k], best, K.pool, K.off, K.len)) best = sw[k];
        part[blockIdx.x] = Partial{best.cnt, best.ka, best.kb, best.slot, best.a, best.b, 0};
        if (blockIdx.x == 0 && !st->halt) {
            // finish the round: the new token enters the dedupe map; round/ntok advance (only
            // k_merge reads these, in the next launch)
            const unsigned nw = st->cur_new;
            if (st->new_is_new) {
                const unsigned long long h = K.hash[nw];
                unsigned s = (unsigned)mix64(h) & K.map_mask;
                while (K.map[s] != 0) s = (s + 1) & K.map_mask;
                K.map[s] = map_entry(h, nw);
            }
            st->round = st->cur_round + 1;
            st->ntok = st->cur_ntok;
        }
    }
}

// ------------------------------------------------------------------ argmax over C (rebuild)
// After the host re-thresholds C: per-block partials of the argmax over all of C.
__global__ void __launch_bounds__(256) k_argmax(RoundState* __restrict__ st, PairsDev P, ToksDev K,
                                                Partial* __restrict__ part) {
    __shared__ Cand sw[4];
    Cand best = cand_none();
    const unsigned nC = st->nC;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < nC; i += gridDim.x * blockDim.x) {
        const uint4 e = P.C[i];
        const unsigned f = P.flag[e.x];
        const long long c = P.cnt[e.x];
        const unsigned long long ka = K.key8[e.y], kb = K.key8[e.z];
        if (!(f & kPresent)) continue;
        const Cand x{c, ka, kb, e.x, e.y, e.z};
        if (cand_better(x, best, K.pool, K.off, K.len)) best = x;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const Cand oc = shfl_xor_cand(best, o);
        if (cand_better(oc, best, K.pool, K.off, K.len)) best = oc;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sw[w] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
            if (cand_better(sw[k], best, K.pool, K.off, K.len)) best = sw[k];
        part[blockIdx.x] = Partial{best.cnt, best.ka, best.kb, best.slot, best.a, best.b, 0};
    }
}

// ------------------------------------------------------------------ batched rounds
// Several merges per round trip, exactly.  At a state S, let P1 > P2 > ... be the candidates in
// the reference's order (count, then bytes; train.py:187-189).  The top k form a batch when
//   (1) no member's b is any member's a (members may share an a, or share a b) and
//   (2) a != b for each (k > 1),
//   (3) each a + b is new bytes: not an existing token, not another member's (vocab.py:29),
//   (4) count(Pk) >= T and count(Pk) > count of the next candidate in C (keys outside C are
//       below T), so every pair outside the batch has a count strictly below count(Pk).
// Then the reference takes P1, ..., Pk in exactly that order:
//   * merging Pi = (ai, bi) removes only the pairs (x, ai) and (bi, y) at its occurrences; with
//     no b equal to an a, no member has either shape and no two members' occurrences overlap, so
//     Pj's count is unchanged until its turn; with a != b every occurrence of Pi is merged;
//   * an occurrence of a pair created by the batch sits where, before the batch, two original
//     tokens met -- an occurrence of an old pair that is not a member (members' occurrences are
//     all merged) -- so its count is below count(Pk); old non-members only lose counts.
// The rewrite applies the members in order to each word (the deltas of member j see the word
// after members < j, as the reference's sequence of rounds does), so counts, present keys and
// words after the trip equal the state after k rounds.
#ifndef BPE355_MAX_BATCH
#define BPE355_MAX_BATCH 16
#endif
constexpr int kMaxBatch = BPE355_MAX_BATCH;   // members per trip (3 * kMaxBatch tokens fit one wave)
static_assert(kMaxBatch >= 1 && kMaxBatch <= 21, "BPE355_MAX_BATCH: 1..21 (3 * members fit one wave)");
// the largest power of two <= kMaxBatch - 1: the first step of a binary search over members
constexpr int top_step(int m) { int p = 1; while (2 * p <= m) p *= 2; return m >= 1 ? p : 0; }
constexpr int kListTopStep = top_step(kMaxBatch - 1);
constexpr int kTopM = kMaxBatch + 1;
// the select's clash check: candidates i < kClashI (a power of two >= kMaxBatch), kClashJ lanes each
constexpr int kClashI = kMaxBatch <= 16 ? 16 : 32;
constexpr int kClashJ = 64 / kClashI;
#ifndef BPE355_LDS_CELLS   // build-time default of the run-time knob of the same name
#define BPE355_LDS_CELLS 1
#endif
#ifndef BPE355_LDS_B
#define BPE355_LDS_B 128
#endif
constexpr unsigned kLdsB = BPE355_LDS_B;   // LDS-summed cells per member (ids below kLdsB)
// Batch members may share an a or a b (rule (1) below).  With 0, every member's tokens are
// distinct from the others' (rounds 1-4): on the bench corpus's merge sequence that rule alone
// ends 2583 of 3682 batches against 498 of 2430 (tools/sim_batch.py, cap 16)
#ifndef BPE355_SHARE_TOK
#define BPE355_SHARE_TOK 1
#endif
constexpr bool kShareTok = BPE355_SHARE_TOK != 0;
// Rule (4'): a tied non-member that seeds member j's new pairs cuts the batch after P_j (1), or
// back to the members above the tie (0, rounds 1-4)
#ifndef BPE355_TIE_BY_MEMBER
#define BPE355_TIE_BY_MEMBER 1
#endif
constexpr bool kTieByMember = BPE355_TIE_BY_MEMBER != 0;
// A word several members hit: all of them rewritten in registers, one store pass (1), or one
// member at a time through memory, the word re-read between members (0, rounds 1-4)
#ifndef BPE355_REG_REWRITE
#define BPE355_REG_REWRITE 1
#endif
constexpr bool kRegRewrite = BPE355_REG_REWRITE != 0;
// the widest slot class rewritten in registers (the 64-id class needs ~60 more VGPRs)
#ifndef BPE355_REG_REWRITE_MAXW
#define BPE355_REG_REWRITE_MAXW 32
#endif
constexpr int kRegRewriteMaxW = BPE355_REG_REWRITE_MAXW;
// Which members a word holds: with at least this many members, each adjacent pair of the word is
// looked up in an LDS table of the batch's pairs (hashed, 4096 one-byte slots: member + 1, 0xFF
// when two members share a slot) instead of compared with every member -- k x (W - 2) compares
// made the full scans of the first trips VALU-bound.  0: always compare with every member.
#ifndef BPE355_PAIR_FILTER_K
#define BPE355_PAIR_FILTER_K 4
#endif
constexpr int kPairFilterK = BPE355_PAIR_FILTER_K;
constexpr unsigned kPairSlots = 4096;
// list mode: a word's count is loaded only when the word holds a member (build knob)
#ifndef BPE355_LATE_COUNT
#define BPE355_LATE_COUNT 1
#endif
constexpr bool kLateCount = BPE355_LATE_COUNT != 0;
__device__ __forceinline__ unsigned pair_h12(unsigned x, unsigned y) {
    return ((x * 0x9E3779B1u) ^ (y * 0x85EBCA77u)) >> 20;
}
typedef __attribute__((address_space(3))) uint8_t LdsU8;

struct BatchMember {
    unsigned a, b, nw, slot;
    long long cnt;
    unsigned long long hash, k8, pw;
    unsigned ln, list_beg, list_len, use_list, cov_beg, cov_len, pool_off, isnew;
    // members sharing a token: the first member with this a (ga) / this b (gb) holds the mask of
    // every member with it, the others 0.  The apply updates (x, a) and (b, y) once, from the
    // group's summed cells (a key has one updater).
    unsigned ga, gb;
};
struct Batch {
    int stop;            // 0 run, -1 nothing to do, > 0 the halt the apply raises
    int k;               // members
    int round, ntok;     // round of member 0, token count before the batch
    int trip, prev_k;    // trip number (cell parity), members of the previous trip
    int prev_sparse;     // the previous trip's apply listed touched blocks (its merge clears by them)
    unsigned batch_id;   // word claims of this batch
    unsigned full_scan;  // a member has no usable posting list: scan every word once
    unsigned n_fresh;    // members that create a token
    unsigned nC_base;    // C entries before this trip's admissions (the apply scans them)
    unsigned idle_from;  // list mode: merge threads from this index on have no word (~0: scan mode)
    // state the select decided that its own kernel must not see change (every workgroup of the
    // fused trip kernel runs the select on the same inputs): the apply publishes them
    unsigned pool_after; // st->pool_used after this trip's new tokens
    long long T2next;    // the candidate-list threshold of this trip's apply (-> bs->T2)
    unsigned list_pre[kMaxBatch + 1];   // prefix sums of the members' list lengths
    BatchMember m[kMaxBatch];
};

// device-owned batch state (the host only initializes it; its limits live in RoundState)
struct BatchState {
    unsigned pend_insert;    // unused (k_apply_batch inserts the batch's new tokens into the map)
    unsigned batch_seq;      // last batch_id handed out
    int trip;                // trips completed
    int prev_k;              // members of the last trip (its cells are cleared by the next apply)
    int prev_sparse;         // the last trip's apply listed touched blocks (CellMarks)
    unsigned long long rounds_batched;   // statistics: rounds taken in batches of k > 1
    unsigned long long trips_batched;
    long long T2;            // candidate-list threshold (>= T): every present key >= T2 is listed
    // keys the apply appended to the list, by trip parity: trip t's select reads list (t & 1), its
    // apply fills list ((t + 1) & 1) (> kListCap: overflow)
    unsigned list_n[2];
    unsigned long long n_overflow, n_headmiss, n_short, k_hist[kMaxBatch + 1];   // diagnostics
    unsigned long long k1_why[6];   // single-merge trips: P1 a == b / P1 not fresh / no list / P2 fails / tie / end
    // what ended each batch: the cap / the ranked list ran out / candidate k failed the token or
    // freshness rules / the count gap or a tie at the boundary cut it / P1 not batchable
    unsigned long long end_why[5];
};
// the candidate list the select ranks, one thread per entry (build knob BPE355_LIST_CAP, a multiple
// of 64; a trip whose list overflows it takes P1 alone and raises T2).  128 took 56 more trips at
// the bench config for the same merge phase (255.6 ms, profiles/r05/g_bench_default.log; r04:
// zk_list_cap_ab.txt)
#ifndef BPE355_LIST_CAP
#define BPE355_LIST_CAP 256
#endif
constexpr unsigned kListCap = BPE355_LIST_CAP;
static_assert(kListCap % 64 == 0 && kListCap >= 64, "whole waves of list threads");
// k_apply_batch workgroups (k_select reads one partial each; build knob BPE355_APPLY_GRID)
#ifndef BPE355_APPLY_GRID
#define BPE355_APPLY_GRID 512
#endif
constexpr unsigned kApplyGrid = BPE355_APPLY_GRID;

struct SelKey {   // a listed candidate as k_select's ranking reads it
    long long cnt;
    unsigned long long ka, kb, ab;   // key8 of a and of b; b << 32 | a
};

struct TokMetaS {
    unsigned long long ha, pb, hb, pa;   // hash(a), P^len(b), hash(b), P^len(a)
    unsigned la, lb, za, zb, ba, bb;     // lengths; posting lists of a and b (len, begin)
};

// A member's cells: ids below N summed in LDS per workgroup (32-bit: a cell never exceeds the
// member's own count, count(P_j) <= count(P_1), so `narrow` = count(P_1) < 2^32 holds for the
// whole batch; otherwise every add goes to the global cells), the rest by global atomics.
typedef __attribute__((address_space(3))) unsigned LdsU32;   // an LDS word (explicit address space)
// Touched blocks (the apply visits only the cells that can hold a delta): a member's cells
// from `mark_from` on (2 x the densely scanned token prefix, >= 2 N) are grouped in blocks of 64
// cells (32 tokens); every global add there sets its block's bit in the workgroup's LDS bitmap
// (word = cell >> 11), which the flush ORs into one of kTBRep global replicas per trip parity
// (fewer same-address atomics); the apply ORs the replicas and lists the touched blocks.
constexpr unsigned kTBRep = 2;      // global bitmap replicas (a workgroup ORs into blockIdx % kTBRep)
constexpr unsigned kTBMax = 64;     // bitmap words per member: tokens up to 65 536 (else every cell scanned)
constexpr unsigned kTLCap = 4096;   // touched blocks the apply lists in LDS (more: every cell scanned)
struct CellMarks {
    unsigned* tb;        // [parity][kTBRep][kMaxBatch][tbw] touched-block bitmaps written by the merge
    unsigned* tbc;       // [kMaxBatch][tbw]: the last apply's OR of its replicas (the next merge clears by it)
    unsigned tbw;        // bitmap words per member (0: no marks, every cell scanned and cleared)
    unsigned dense_tok;  // tokens below this are scanned densely for every member (a multiple of 32)
    unsigned sparse_from;   // an apply lists touched blocks once the tokens pass this (below: every cell)
    unsigned long long* sig;   // BPE355_CHECK_MARKS: each apply workgroup's view of the list (else null)
};
template <unsigned N>
struct DeltaSinkN {
    unsigned long long* LR;     // this member's global cells
    LdsU32* lds;                // this member's LDS cells (ids below N)
    LdsU32* bm;                 // this member's touched-block bitmap (LDS)
    unsigned mark_from;         // cells from here on are marked (~0u: none)
    bool narrow;
    __device__ __forceinline__ void add(unsigned cell, unsigned long long c) const {
        if (narrow && cell < 2 * N) {
            __hip_atomic_fetch_add(&lds[cell], (unsigned)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            atomicAdd(&LR[cell], c);
            if (cell >= mark_from)
                __hip_atomic_fetch_or(&bm[cell >> 11], 1u << ((cell >> 6) & 31), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
};

// BPE355_PROBE: 100 MHz stamps of one trip in kProbeTrip, kProbeSlots per sampled trip
// (MergeLoop::report_probe): 0-13 phase stamps, 14/15 the last merge/apply workgroup done, 16 the
// next trip's select start, 17-19 inside select's rule, 20/21 the last merge/apply workgroup's index
constexpr int kProbeTrip = 8;
constexpr int kProbeSlots = 32;   // 24-28: inside k_select's first phase
// The stamps are compiled in only with -DBPE355_PROBE_CODE=1 (tools/build_variant.sh probe; then
// the run-time BPE355_PROBE switch turns them on).  Compiled in but off, their code and registers
// cost 4-6 ms of the 260 ms merge phase (r04r A/B, two reps, profiles/r04/r_*).
#ifndef BPE355_PROBE_CODE
#define BPE355_PROBE_CODE 0
#endif
// The select's diagnostic counters (list overflows, head misses, the k histogram and why trips
// took one merge; printed under BPE355_TRACE) are compiled in only with -DBPE355_STATS_CODE=1.
// n_rounds_batched comes from the trips' records on the host either way.
#ifndef BPE355_STATS_CODE
#define BPE355_STATS_CODE 0
#endif
__device__ __forceinline__ void probe_stamp(const RoundState* st, int trip, int k) {
    if (BPE355_PROBE_CODE && st->probe && (trip % kProbeTrip) == 0)
        st->probe[kProbeSlots * (size_t)(trip / kProbeTrip) + k] = __builtin_amdgcn_s_memrealtime();
}
// one workgroup of a sampled trip's kernel is done (thread 0, after the workgroup's work): the
// last of the grid stamps slot k
__device__ __forceinline__ void probe_done(RoundState* st, unsigned* ctr, int trip, int k) {
    if (BPE355_PROBE_CODE && st->probe && (trip % kProbeTrip) == 0) {
        const unsigned o = atomicAdd(ctr, 1u);
        if (o % gridDim.x == gridDim.x - 1) {
            probe_stamp(st, trip, k);
            st->probe[kProbeSlots * (size_t)(trip / kProbeTrip) + k + 6] = blockIdx.x + 1;
        }
    }
}

__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int j) {
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)v, j);
    const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(v >> 32), j);
    return ((unsigned long long)hi << 32) | lo;
}
// lane j's candidate, in every lane (scalar broadcast)
__device__ __forceinline__ Cand readlane_cand(const Cand& c, int j) {
    Cand r;
    r.cnt = (long long)readlane64((unsigned long long)c.cnt, j);
    r.ka = readlane64(c.ka, j);
    r.kb = readlane64(c.kb, j);
    r.slot = __builtin_amdgcn_readlane((int)c.slot, j);
    r.a = __builtin_amdgcn_readlane((int)c.a, j);
    r.b = __builtin_amdgcn_readlane((int)c.b, j);
    return r;
}

// The wave's best candidate in every lane.  The order is the count first (cand_better), so the
// wave's largest count is found with 64-bit shuffles alone; its holder's candidate is the best
// when it is the only one (then read from that lane), and only a tie at the top goes through the
// full order (shuffles of the whole candidate, and the bytes when the 8-byte prefixes tie).
// (kFastWaveBest = 0: the full order always.)
#ifndef BPE355_FAST_WAVE_BEST
#define BPE355_FAST_WAVE_BEST 1
#endif
__device__ __forceinline__ Cand wave_best(Cand best, const ToksDev& K) {
    if (BPE355_FAST_WAVE_BEST) {
        long long m = best.cnt;
        for (int o = 32; o > 0; o >>= 1) m = max(m, (long long)__shfl_xor(m, o));
        if (m == LLONG_MIN) return cand_none();
        const unsigned long long hold = __ballot(best.cnt == m);
        if (__popcll(hold) == 1) return readlane_cand(best, __ffsll((long long)hold) - 1);
        if (best.cnt != m) best = cand_none();
    }
    for (int o = 32; o > 0; o >>= 1) {
        const Cand oc = shfl_xor_cand(best, o);
        if (cand_better(oc, best, K.pool, K.off, K.len)) best = oc;
    }
    return best;
}

// A listed candidate's token metadata and dedupe lookup (does the pair's byte string exist as a
// token already?).  The map holds every token up to the last trip's (k_apply_batch inserts them).
__device__ __forceinline__ void cand_meta(const Cand& c, const ToksDev& K, const IndexDev& X, TokMetaS& m,
                                          unsigned& old) {
    const unsigned a = c.a, b = c.b;
    m.ha = K.hash[a]; m.pb = K.pw[b]; m.hb = K.hash[b]; m.pa = K.pw[a];
    m.la = K.len[a]; m.lb = K.len[b];
    m.za = X.len[a]; m.zb = X.len[b]; m.ba = X.beg[a]; m.bb = X.beg[b];
    const unsigned long long h = m.ha * m.pb + m.hb;
    const unsigned ln = m.la + m.lb;
    old = map_find(K, h, ln, a, b);
}

// One workgroup: the batch of this trip.  Waves 0-7 reduce the apply's per-workgroup partials
// to the exact best candidate P1; waves 8-11 hold the candidate list (every present key >= T2),
// look up its entries' metadata and rank them.  All global loads are issued before the first
// barrier, so the kernel costs about one memory round trip plus the dedupe lookups' chain, then
// the ranking, the rule and the record (wave 0).
#ifndef BPE355_LIST_TARGET
#define BPE355_LIST_TARGET 48
#endif
constexpr unsigned kListTarget = BPE355_LIST_TARGET;   // keys the next list should hold (T2 control)
// waves of k_select that reduce the apply's partials (kPartPer each per thread); the list's waves
// follow them (build knob BPE355_SEL_PART_WAVES).  4 waves with two partials per thread: a 512-
// thread select, 252.2-253.7 ms of HBM-resident merges against 255.0-268.0 with 8 waves and
// 258.3-260.6 with 2 (two paired reps, profiles/r04/zh_*)
#ifndef BPE355_SEL_PART_WAVES
#define BPE355_SEL_PART_WAVES 4
#endif
constexpr int kSelListWave = BPE355_SEL_PART_WAVES;   // first wave of the list
constexpr bool kSelMetaAll = true;     // metadata of every listed key before the ranking
constexpr int kSelThreads = 64 * kSelListWave + (int)kListCap;
// k_trip workgroups: 256 threads (four per CU).  One 1024-thread workgroup per CU decided faster
// (the partials' re-reads by four workgroups per CU cost 1.3 us) but left an 11.8 us merge ->
// apply gap: 289 vs 258 ms of merges (profiles/r05/d_fold_ab.txt)
constexpr unsigned kTripThreads = 256;

// The LDS of one batch decision
struct SelLds {
    Cand wave[8];                     // the partial waves' bests
    Cand all[kListCap];
    SelKey topkey[kListCap];          // the entries with fewer than kTopM larger counts,
    unsigned top[kListCap];           // packed for the exact ranking (key, list index)
    long long cnt[kListCap];
    Cand list[kTopM];
    TokMetaS meta[kTopM];
    unsigned nw_old[kTopM];
    Cand p1;                          // the exact best (wave 0, beside the ranking)
    long long cnt_target, cnt_last;   // counts at sorted positions kListTarget - 1, ln - 1
    unsigned ntop;
};

// where the publishing workgroup records a batch decision for the host (round records, the
// block's trip records)
constexpr int kTI = 8;   // ints per trip record: round, k, full scan, list entries, ntok, |C|, listed keys, fresh
struct SelOut {
    uint32_t *m_a, *m_b, *m_new, *m_mode;
    long long* m_cnt;
    int* trip_info;
    int trip_slot;
};

// The batch of a trip: reduce the apply's per-workgroup partials to the exact best candidate P1,
// rank the candidate list (every present key >= T2) and apply the batch rule.  All global loads
// are issued first, so the decision costs about one memory round trip plus the dedupe lookups'
// chain, then the ranking, the rule and the record (wave 0).
//   kNT = kSelThreads (k_select, one workgroup): waves 0-3 reduce the partials while the list
//         waves rank;
//   kNT = 256 (k_trip: EVERY workgroup of the fused trip kernel decides the same batch): each
//         thread reduces two partials and holds one list entry.
// The decision goes to OB (stop != 0: no trip this time; > 0 a halt code the apply raises).
// It reads only state that no kernel of the trip changes before the apply: the select phase of
// k_trip runs in every workgroup while other workgroups already rewrite, so everything it decides
// from (st->n_single, pool_used, halt, the list counts, batch_seq, T2) is updated by the apply,
// from the batch record.  `pub`: this workgroup publishes (the round records, trip records, the
// next list's counter, the statistics).  The caller's barrier makes OB visible.
template <int kNT>
__device__ __forceinline__ void select_core(const RoundState* __restrict__ st, BatchState* __restrict__ bs,
                                            const ToksDev& K, const IndexDev& X,
                                            const Partial* __restrict__ part, const Partial* __restrict__ lists,
                                            Batch& OB, SelLds& S, const SelOut& O, const bool pub) {
    static_assert(kNT == kSelThreads || kNT == 256 || kNT == 1024,
                  "k_select's shape, or one k_trip workgroup of 256 or 1024 threads");
    // threads that reduce partials (the first kPartT) and the list thread of each entry (a
    // 1024-thread k_trip workgroup decides as k_select does; its other waves wait at the barriers)
    constexpr int kPartT = kNT == 256 ? kNT : 64 * kSelListWave;
    constexpr int kPartW = kPartT / 64;
    constexpr int kListT0 = kNT == 256 ? 0 : 64 * kSelListWave;
    static_assert(kPartW <= 8 && (int)kListCap <= kNT - kListT0, "one list entry per list thread");
    constexpr int kPartPer = (int)((kApplyGrid + kPartT - 1) / kPartT);
    static_assert(kPartPer >= 1 && kPartPer <= 4, "partials per thread of the partial waves");
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ptrip = bs->trip;
    if (pub && tid == 0) {
        probe_stamp(st, ptrip, 0);
        if (BPE355_PROBE_CODE && ptrip > 0 && st->probe && ((ptrip - 1) % kProbeTrip) == 0)
            st->probe[kProbeSlots * (size_t)((ptrip - 1) / kProbeTrip) + 16] = __builtin_amdgcn_s_memrealtime();
    }
    // ---- every independent load first
    Partial q[kPartPer] = {};
    if (tid < kPartT) {   // the buffer holds kApplyGrid entries
#pragma unroll
        for (int u = 0; u < kPartPer; ++u)
            if (tid + u * kPartT < (int)kApplyGrid) q[u] = part[tid + u * kPartT];
    }
    const Partial* list = lists + (size_t)(ptrip & 1) * kListCap;   // this trip's list (trip parity)
    Partial lq{};
    // list entry of this thread (>= 0: list threads)
    const int li = tid >= kListT0 && tid < kListT0 + (int)kListCap ? tid - kListT0 : -1;
    if (li >= 0) lq = list[li];
    const int nparts = st->nparts;
    const unsigned ln = bs->list_n[ptrip & 1];
    if (st->halt) {   // a trip queued behind a halt: nothing to do (the host takes over)
        if (tid == 0) {
            OB.stop = -1;
            if (pub && O.trip_info) {
                int* ti = O.trip_info + kTI * O.trip_slot;
                ti[0] = -1; ti[1] = 0; ti[2] = 0; ti[3] = 0;
            }
        }
        return;
    }
    // the rule's scalars (uniform: scalar loads, in flight with the vector loads above)
    const int round = st->round, n_rounds = st->n_rounds, host_round = st->host_round;
    const unsigned nC = st->nC, c_limit = st->c_limit;
    const long long T = st->T;
    const unsigned n_single = st->n_single, single_limit = st->single_limit;
    const unsigned long long pair_used = st->pair_used, pair_limit = st->pair_limit;
    const unsigned pool_used = st->pool_used, pool_cap = st->pool_cap;
    const unsigned max_len = st->max_len;
    const int ntok = st->ntok, max_batch = st->max_batch;
    const int prev_k = bs->prev_k, prev_sparse = bs->prev_sparse;
    const unsigned bid = bs->batch_seq + 1;
    const long long T2old = bs->T2;
    if (pub && tid == 0) probe_stamp(st, ptrip, 1);
    // the list: each entry's metadata first (its chain of dependent loads overlaps the partials'
    // arrival), then each entry's rank among the entries
    const int nl = ln <= kListCap ? (int)ln : 0;
    const bool have = li >= 0 && li < nl;
    const Cand x = have ? Cand{lq.cnt, lq.ka, lq.kb, lq.slot, lq.a, lq.b} : cand_none();
    TokMetaS lm{};
    unsigned lold = ~0u;
    if (li >= 0) {
        if (li < kTopM) S.list[li] = cand_none();
        if (li == 0) { S.cnt_target = LLONG_MAX; S.cnt_last = LLONG_MAX; S.ntop = 0; }
        S.all[li] = x;
        S.cnt[li] = x.cnt;
        if (pub && li == 0 && lq.slot != 0xfffffffeu) probe_stamp(st, ptrip, 24);   // the list entry arrived
        if (have && kSelMetaAll) cand_meta(x, K, X, lm, lold);
        if (pub && li == 0 && lold != 0xfffffffeu && lm.la != 0xfffffffeu) probe_stamp(st, ptrip, 25);   // metadata + dedupe
    }
    if (tid < kPartT) {   // P1: the exact best over the partials
        Cand best = cand_none();
#pragma unroll
        for (int u = 0; u < kPartPer; ++u) {
            const int idx = tid + u * kPartT;
            if (idx < nparts) {
                const Cand c{q[u].cnt, q[u].ka, q[u].kb, q[u].slot, q[u].a, q[u].b};
                if (cand_better(c, best, K.pool, K.off, K.len)) best = c;
            }
        }
        best = wave_best(best, K);
        if (lane == 0) S.wave[wv] = best;
    }
    if (pub && tid == 0) probe_stamp(st, ptrip, 26);   // wave 0's partials reduced
    if (BPE355_PROBE_CODE && pub && tid == 0 && st->probe && (ptrip % kProbeTrip) == 0)
        st->probe[kProbeSlots * (size_t)(ptrip / kProbeTrip) + 30] = ln + 1;
    __syncthreads();
    if (pub && li == 0) probe_stamp(st, ptrip, 27);
    if (wv == 0) {   // P1 over the waves' bests, while the list waves rank (off the rule's path)
        Cand p = S.wave[0];
        for (int w = 1; w < kPartW; ++w)
            if (cand_better(S.wave[w], p, K.pool, K.off, K.len)) p = S.wave[w];
        if (lane == 0) S.p1 = p;
    }
    long long tgt = LLONG_MAX, last = LLONG_MAX;
    // rank by count alone first (one 8-byte compare per entry); only an entry with fewer than
    // kTopM larger counts can be among the first kTopM, and every entry ordered before such an
    // entry has its count or a larger one, so it has fewer than kTopM larger counts too: the
    // exact order among that small set is the exact order overall
    int rc = kTopM, ec = 0;   // entries with a larger count, with an equal count (itself included)
    if (have) {
        rc = 0;
#pragma unroll 8
        for (int j = 0; j < nl; ++j) {
            const long long cj = S.cnt[j];
            rc += cj > x.cnt ? 1 : 0;
            ec += cj == x.cnt ? 1 : 0;
        }
        if (rc < kTopM) {
            const unsigned pos = atomicAdd(&S.ntop, 1u);
            S.top[pos] = li;
            S.topkey[pos] = SelKey{x.cnt, x.ka, x.kb, (unsigned long long)x.b << 32 | x.a};
        }
        // the count at sorted position t is the least count whose first position is <= t
        tgt = rc <= (int)kListTarget - 1 ? x.cnt : LLONG_MAX;
        last = x.cnt;
    }
    if (pub && li == 0) probe_stamp(st, ptrip, 29);   // count ranks done
    __syncthreads();
    if (pub && li == 0) probe_stamp(st, ptrip, 31);   // every list thread's count rank done
    if (have && rc < kTopM) {
        // (count, a's 8-byte prefix, b's) branch-free over the small set; only equal prefixes of
        // different tokens need the bytes (rare: then cand_better).  With no other entry of its
        // count, the count rank is the exact rank (the usual case); otherwise the ties are ordered
        // by bytes over the packed top entries, which hold every entry of this count (each has
        // the same rc < kTopM)
        const int m = ec > 1 ? (int)S.ntop : 0;
        int rank = ec > 1 ? 0 : rc;
        bool tail = false;
#pragma unroll 4
        for (int t = 0; t < m; ++t) {
            const int j = (int)S.top[t];
            const SelKey y = S.topkey[t];
            const unsigned ya = (unsigned)y.ab, yb = (unsigned)(y.ab >> 32);
            const bool gt = y.cnt > x.cnt, eq = y.cnt == x.cnt && j != li;
            const bool ad = ya != x.a, bd = yb != x.b;
            rank += gt | (eq & ad & (y.ka > x.ka)) | (eq & !ad & bd & (y.kb > x.kb));
            tail |= eq & ((ad & (y.ka == x.ka)) | (!ad & bd & (y.kb == x.kb)));
        }
        if (tail) {
            rank = 0;
            for (int t = 0; t < m; ++t) {
                const int j = (int)S.top[t];
                rank += (j != li && cand_better(S.all[j], x, K.pool, K.off, K.len)) ? 1 : 0;
            }
        }
        if (rank < kTopM) {
            if (!kSelMetaAll) cand_meta(x, K, X, lm, lold);
            S.list[rank] = x;
            S.meta[rank] = lm;
            S.nw_old[rank] = lold;
        }
    }
    if (pub && li == 0) probe_stamp(st, ptrip, 28);   // ranked
    if (li >= 0 && (kListT0 > 0 || wv < (int)(kListCap / 64))) {   // wave minima, then one LDS atomic per wave
        for (int o = 32; o > 0; o >>= 1) {
            tgt = min(tgt, (long long)__shfl_xor(tgt, o));
            last = min(last, (long long)__shfl_xor(last, o));
        }
        if (lane == 0 && last != LLONG_MAX) {
            atomicMin(&S.cnt_target, tgt);
            atomicMin(&S.cnt_last, last);
        }
    }
    __syncthreads();
    if (pub && tid == 0) probe_stamp(st, ptrip, 2);
    if (wv != 0) return;
    // ---- wave 0: the rule and the record, lane i holding candidate i (no workgroup barrier)
    const Cand p1 = S.p1;
    // the list's head is the global best whenever the best is >= T2 and nothing overflowed; the
    // ranks are distinct, so S.list holds a prefix
    if (pub && lane == 0) probe_stamp(st, ptrip, 17);
    const bool list_ok = ln <= kListCap && S.list[0].cnt != LLONG_MIN && S.list[0].slot == p1.slot &&
                         S.list[0].a == p1.a && S.list[0].b == p1.b;
    int nf = 1;
    if (list_ok) {
        const unsigned long long vm =
            __ballot(lane >= 1 && lane < kTopM && S.list[lane < kTopM ? lane : 0].cnt != LLONG_MIN) | 1ull;
        nf = __builtin_ctzll(~vm);
    }
    int stop = HALT_NONE;
    if (round >= n_rounds) stop = HALT_DONE;
    else if (nC > c_limit) stop = HALT_REBUILD;                        // C bloated: re-threshold
    else if (p1.cnt == LLONG_MIN || p1.cnt < T) stop = HALT_REBUILD;   // max(C) < T: re-threshold
    else if (round >= host_round || n_single > single_limit ||
             pair_used + 2ull * (unsigned)(ntok + kMaxBatch) * kMaxBatch > pair_limit ||
             pool_used + (unsigned long long)kMaxBatch * max_len > pool_cap)
        stop = HALT_HOST;
    if (BPE355_STATS_CODE && pub && lane == 0) {   // no-return atomics: nothing waits on them
        if (ln > kListCap) atomicAdd(&bs->n_overflow, 1ull);
        else if (!list_ok) atomicAdd(&bs->n_headmiss, 1ull);
        else if (nf < kTopM) atomicAdd(&bs->n_short, 1ull);
    }
    if (stop) {   // the apply raises the halt (nothing this trip's kernels read changes before it)
        if (lane == 0) {
            OB.stop = stop;
            if (pub && O.trip_info) {
                int* ti = O.trip_info + kTI * O.trip_slot;
                ti[0] = -1; ti[1] = 0; ti[2] = 0; ti[3] = 0;
            }
        }
        return;
    }
    const int i = lane;
    Cand e = cand_none();
    TokMetaS m{};
    unsigned old = ~0u;
    if (i == 0) {
        e = p1;
        if (list_ok) { m = S.meta[0]; old = S.nw_old[0]; }
        else cand_meta(p1, K, X, m, old);   // rare: P1 alone, its metadata here
    } else if (i < nf) {
        e = S.list[i];
        m = S.meta[i];
        old = S.nw_old[i];
    }
    const bool fr = i < nf && old == ~0u;
    if (pub && lane == 0) probe_stamp(st, ptrip, 18);
    const unsigned long long h = m.ha * m.pb + m.hb;
    const unsigned lk = m.la + m.lb;
    // (1) a different from every earlier candidate's b and b from every earlier a (kShareTok;
    // else all four tokens distinct), and (3) new bytes different from every earlier candidate's.
    // The kClashI x kClashI (i, j) pairs are spread over the wave: lane L checks i = L % kClashI
    // against j = L / kClashI + t * kClashJ, then the kClashJ lanes of each i combine (one pass of
    // lane shuffles instead of a serial readlane chain over j)
    // each candidate's posting list (the shorter of a's and b's) and whether the merge uses it
    const unsigned lu = m.za <= m.zb ? m.za : m.zb, bu = m.za <= m.zb ? m.ba : m.bb;
    const bool use = lu != kNoAnc && lu <= X.full_threshold;
    const unsigned long long lkey = use && lu > 0 ? (unsigned long long)bu << 32 | lu : 0ull;
    bool clash = false;
    // beside the clash check, for the members' token groups (kShareTok): the candidates with i's
    // a (sa) and with i's b (sb), and whether an earlier candidate walks i's posting list (dl)
    unsigned sa = 0, sb = 0;
    bool dl = false;
    {
        const int ci = lane % kClashI, cj0 = lane / kClashI;
        const unsigned ai = __shfl((int)e.a, ci), bi = __shfl((int)e.b, ci);
        const unsigned long long hi = __shfl(h, ci);
        const unsigned li_ = __shfl((int)lk, ci), lai = __shfl((int)m.la, ci);
        const unsigned long long lki = kShareTok ? __shfl(lkey, ci) : 0ull;
        const bool iv = ci < nf;
#pragma unroll
        for (int t = 0; t < (kTopM + kClashJ - 1) / kClashJ && t < kClashI / kClashJ; ++t) {
            const int j = cj0 + t * kClashJ;   // (candidates past kTopM - 1 are never ranked)
            const unsigned aj = __shfl((int)e.a, j), bj = __shfl((int)e.b, j);
            const unsigned long long hj = __shfl(h, j);
            const unsigned lj = __shfl((int)lk, j), laj = __shfl((int)m.la, j);
            if (kShareTok) {
                const unsigned long long lkj = __shfl(lkey, j);
                sa |= (unsigned)(aj == ai) << j;
                sb |= (unsigned)(bj == bi) << j;
                dl |= j < ci && lki != 0 && lkj == lki;
            }
            if (j < ci && iv) {
                const bool tc = aj == bi || bj == ai || (!kShareTok && (aj == ai || bj == bi));
                clash |= tc;
                if (!tc && hj == hi && lj == li_) {   // equal hashes: compare the bytes (rare)
                    bool eq = true;
                    for (unsigned y = 0; y < li_ && eq; ++y)
                        eq = concat_byte(K, aj, laj, bj, y) == concat_byte(K, ai, lai, bi, y);
                    clash |= eq;
                }
            }
        }
        for (int o = kClashI; o < 64; o <<= 1) {
            clash |= __shfl_xor((int)clash, o) != 0;
            if (kShareTok) {
                sa |= (unsigned)__shfl_xor((int)sa, o);
                sb |= (unsigned)__shfl_xor((int)sb, o);
                dl |= __shfl_xor((int)dl, o) != 0;
            }
        }
        if (i >= kClashI) clash = false;   // lanes < kClashI hold their own i's result
    }
    // k: the first candidate that fails (count >= T, (2) a != b, fresh, no clash), within the
    // allowed batch; one merge when P1 itself is not batchable
    const int maxb = min(max_batch, kMaxBatch);
    const bool okb = i >= 1 && i < nf && e.cnt >= T && e.a != e.b && fr && !clash;
    int k = __builtin_ctzll(~(__ballot(okb) | 1ull));
    k = min(k, min(maxb, nf));
    const int k_rule = k;
    if (!(p1.a != p1.b && __builtin_amdgcn_readlane((int)fr, 0))) k = 1;
    // (4) strictly above the next candidate: listed (candidate k), or unlisted (below T2, and
    // every member is listed, so >= T2): the largest k' <= k with that gap
    {
        const long long cprev = __shfl(e.cnt, i > 0 ? i - 1 : 0);
        const unsigned long long gm =
            __ballot(i >= 1 && (i >= nf || cprev > e.cnt)) & ((2ull << k) - 1) & ~1ull;
        const int k_strict = gm ? 63 - __builtin_clzll(gm) : 1;
        // (4') a tie at the boundary is harmless unless a tied non-member could seed a new pair:
        // a pair created by the batch has at most the count of the old pair (x, a_j) or (b_j, y)
        // it replaces, so with every tied non-member free of those shapes, no new pair reaches
        // count(Pk).  Every key >= T2 is listed, so the tied keys are all in S.all.  A pair
        // member j creates exists only after P_j's merge, so it can precede only members after j:
        // with j the first member a tied non-member seeds, the batch keeps P1 .. P_j (and at
        // least the members above the tie).  Former members past the cut never seed one (no b
        // of one member is another's a), so the shorter batch needs no second check.
        if (k_strict < k && k > 1) {
            const long long c = readlane64((unsigned long long)e.cnt, k - 1);
            unsigned ma[kMaxBatch], mb[kMaxBatch], ms[kMaxBatch];
#pragma unroll
            for (int j = 0; j < kMaxBatch; ++j) {
                ma[j] = __builtin_amdgcn_readlane((int)e.a, j);
                mb[j] = __builtin_amdgcn_readlane((int)e.b, j);
                ms[j] = __builtin_amdgcn_readlane((int)e.slot, j);
            }
            int jb = k;   // the first member a tied non-member seeds (k: none)
            for (int t = lane; t < nl; t += 64) {
                const Cand y = S.all[t];
                if (y.cnt != c) continue;
                bool member = false;
                int js = k;
#pragma unroll
                for (int j = 0; j < kMaxBatch; ++j) {
                    if (j >= k) break;
                    member |= y.slot == ms[j];
                    if (js == k && (y.b == ma[j] || y.a == mb[j])) js = j;
                }
                if (!member) jb = min(jb, js);
            }
            for (int o = 32; o > 0; o >>= 1) jb = min(jb, __shfl_xor(jb, o));
            k = min(k, max(kTieByMember ? jb + 1 : (jb < k ? 0 : k), k_strict));
        } else {
            k = k_strict;
        }
    }
    if (pub && lane == 0) probe_stamp(st, ptrip, 19);
    const bool fr0 = __builtin_amdgcn_readlane((int)fr, 0);
    if (BPE355_STATS_CODE && pub && k == 1 && lane == 0) {
        const int why = p1.a == p1.b ? 0 : !fr0 ? 1 : nf == 1 ? 2 : k_rule == 1 ? 3 : 4;
        atomicAdd(&bs->k1_why[why], 1ull);
    }
    if (BPE355_STATS_CODE && pub && lane == 0) {
        const int why = !(p1.a != p1.b && fr0) ? 4 : k < k_rule ? 3 : k_rule == maxb ? 0 : k_rule == nf ? 1 : 2;
        atomicAdd(&bs->end_why[why], 1ull);
    }
    k = min(k, n_rounds - round);
    // per member: pool offset, new id, posting-list prefix (exclusive scans over lanes < k)
    const bool mem = i < k;
    // the members' token groups (equal a's, equal b's: the group's first member carries the
    // group's mask) and posting lists two members share (the later one walks none of it: the
    // word is claimed once and every member's hits are found on it)
    unsigned ga, gb;
    bool dup_list = false;
    if (kShareTok) {
        const unsigned km = (unsigned)((1ull << k) - 1), below = (1u << (i & 31)) - 1;
        ga = sa & km;
        gb = sb & km;
        if (ga & below) ga = 0;
        if (gb & below) gb = 0;
        dup_list = dl;   // (an earlier candidate with the list is a member when i is)
    } else {
        ga = gb = 1u << (i & 31);
    }
    const unsigned add_pool = mem && fr ? lk : 0u, add_fresh = mem && fr ? 1u : 0u,
                   add_list = mem && use && !dup_list ? lu : 0u;
    unsigned pre_pool = add_pool, pre_fresh = add_fresh, pre_list = add_list;   // inclusive scans
    for (int d = 1; d <= kMaxBatch; d <<= 1) {
        const unsigned tp = __shfl_up((int)pre_pool, d), tf = __shfl_up((int)pre_fresh, d),
                       tl = __shfl_up((int)pre_list, d);
        if (lane >= d) { pre_pool += tp; pre_fresh += tf; pre_list += tl; }
    }
    pre_pool -= add_pool; pre_fresh -= add_fresh; pre_list -= add_list;   // exclusive: lanes < i
    // one scan of every word once the members' lists together pass the scan threshold
    const bool full = __ballot(mem && !use) != 0 || __builtin_amdgcn_readlane((int)pre_list, k) > (int)X.full_threshold;
    const unsigned tot_pool = __builtin_amdgcn_readlane((int)pre_pool, k);
    const unsigned tot_list = __builtin_amdgcn_readlane((int)pre_list, k);
    const unsigned tot_fresh = __builtin_amdgcn_readlane((int)pre_fresh, k);
    if (i <= k) OB.list_pre[i] = pre_list;
    if (mem) {
        BatchMember M;
        M.a = e.a; M.b = e.b; M.slot = e.slot; M.cnt = e.cnt;
        M.nw = fr ? (unsigned)ntok + pre_fresh : old;
        M.isnew = fr;
        M.hash = h;
        M.pw = m.pa * m.pb;
        M.ln = lk;
        M.k8 = m.la >= 8 ? e.ka : (e.ka | (e.kb >> (8 * m.la)));
        M.use_list = use;
        M.list_beg = use ? bu : 0;
        M.list_len = use ? lu : 0;
        M.cov_beg = bu;
        M.cov_len = fr ? lu : kNoAnc;   // dedupe: uncovered until the next index build
        M.pool_off = pool_used + pre_pool;
        M.ga = ga;
        M.gb = gb;
        OB.m[i] = M;
        if (pub) {
            O.m_a[round + i] = e.a; O.m_b[round + i] = e.b; O.m_new[round + i] = M.nw;
            O.m_mode[round + i] = use ? lu : 0xffffffffu;
            if (O.m_cnt) O.m_cnt[round + i] = e.cnt;
        }
    }
    if (lane == 0) {
        OB.stop = 0;
        OB.k = k;
        OB.round = round;
        OB.ntok = ntok;
        OB.trip = ptrip;
        OB.prev_k = prev_k;
        OB.prev_sparse = prev_sparse;
        OB.batch_id = bid;
        OB.nC_base = nC;
        OB.full_scan = full;
        {   // the merge's idle workgroups: past the listed words, when every member has a list
            const bool lists_ok = k > 1 ? !full : use;   // lane 0: member 0's own flag
            OB.idle_from = lists_ok ? tot_list : ~0u;
        }
        OB.n_fresh = tot_fresh;
        OB.pool_after = pool_used + tot_pool;
        {   // the next list: about kListTarget keys.  With the list ranked, T2 = the count of the
            // kListTarget-th best (this trip pops at most kMaxBatch of those above it); on overflow
            // raise T2 halfway to the top; with too few keys, extend the range below the last one
            const long long top = p1.cnt;
            const long long t2 = T2old < T ? T : T2old;
            long long nt;
            if (ln > kListCap) nt = t2 + (top - t2) / 2;
            else if (ln >= kListTarget) nt = S.cnt_target;
            else if (ln > 0) nt = S.cnt_last - (top - S.cnt_last) - 1;
            else nt = T;
            OB.T2next = nt < T ? T : (nt > top ? top : nt);
        }
        if (pub) {
            bs->list_n[(ptrip + 1) & 1] = 0;   // the list this trip's apply fills (nothing reads it before)
            if (BPE355_STATS_CODE) {
                if (k > 1) {
                    atomicAdd(&bs->rounds_batched, (unsigned long long)k);
                    atomicAdd(&bs->trips_batched, 1ull);
                }
                atomicAdd(&bs->k_hist[k], 1ull);
            }
            if (O.trip_info) {   // for the host: first round, members, scan mode, list entries
                int* ti = O.trip_info + kTI * O.trip_slot;
                ti[0] = round; ti[1] = k; ti[2] = full; ti[3] = (int)tot_list;
                // (the trip log's extra fields: tokens, C entries the apply scans, listed keys, fresh tokens)
                ti[4] = ntok; ti[5] = (int)nC; ti[6] = (int)ln; ti[7] = (int)tot_fresh;
            }
            probe_stamp(st, ptrip, 3);
            probe_stamp(st, ptrip, 4);
        }
    }
}

__global__ void __launch_bounds__(kSelThreads) k_select(const RoundState* __restrict__ st, BatchState* __restrict__ bs,
                                                        ToksDev K, IndexDev X, Batch* __restrict__ bt,
                                                        const Partial* __restrict__ part,
                                                        const Partial* __restrict__ lists, SelOut O) {
    __shared__ SelLds S;
    select_core<kSelThreads>(st, bs, K, X, part, lists, *bt, S, O, true);
}

// Test knob BPE355_CHECK_MARKS: after a trip's merge, the other parity (cleared by it from the
// dense prefix and the previous apply's touched-block list) must be zero in every cell and bitmap:
// a nonzero cell there is a delta the marks missed.  dbg[0] counts them, dbg[1..3] the first one
// (trip, member, cell).
__global__ void k_check_clear(const Batch* __restrict__ bt, const unsigned long long* __restrict__ LRbase,
                              size_t lr_member, size_t lr_parity, const unsigned* __restrict__ tb, unsigned tbw,
                              unsigned long long* __restrict__ dbg) {
    const Batch& B = *bt;
    if (B.stop) return;
    const unsigned long long* LRo = LRbase + (size_t)((B.trip + 1) & 1) * lr_parity;
    const size_t n = (size_t)kMaxBatch * lr_member;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (size_t)gridDim.x * blockDim.x)
        if (LRo[q] != 0 && atomicAdd(&dbg[0], 1ull) == 0) {
            dbg[1] = (unsigned long long)B.trip;
            dbg[2] = q / lr_member;
            dbg[3] = q % lr_member;
        }
    if (tbw) {
        const unsigned* TBo = tb + (size_t)((B.trip + 1) & 1) * kTBRep * kMaxBatch * tbw;
        for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < (size_t)kTBRep * kMaxBatch * tbw;
             q += (size_t)gridDim.x * blockDim.x)
            if (TBo[q]) atomicAdd(&dbg[4], 1ull);
    }
}

// BPE355_CHECK_MARKS after an apply: every workgroup must have seen the same touched blocks
__global__ void k_check_sig(const Batch* __restrict__ bt, unsigned long long* __restrict__ sig, unsigned n,
                            unsigned long long* __restrict__ dbg) {
    const Batch& B = *bt;
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x) {
        if (!B.stop && sig[1 + i] != sig[1] && atomicAdd(&dbg[5], 1ull) == 0) {
            dbg[6] = (unsigned long long)B.trip;
            dbg[7] = i;
        }
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x) sig[1 + i] = 0;
}

// end of a block of trips: the state and the trips' records -> pinned host memory (plain vector
// stores; the block's event orders them before the host reads)
__global__ void __launch_bounds__(256) k_snapshot(const uint32_t* __restrict__ st, unsigned n_st,
                                                  const uint32_t* __restrict__ ti, unsigned n_ti,
                                                  uint32_t* __restrict__ h_st, uint32_t* __restrict__ h_ti) {
    for (unsigned i = threadIdx.x; i < n_st; i += blockDim.x) h_st[i] = st[i];
    for (unsigned i = threadIdx.x; i < n_ti; i += blockDim.x) h_ti[i] = ti[i];
}


// the slot word of class C addressed directly, every member applied in order.  claim: the word
// (global slot index f) may be on several members' lists; the first thread to claim it rewrites
// it.  The word is loaded before the claim: only the claimant writes it during this batch.
template <class TokT, int C>
__device__ __forceinline__ void merge_word_batch(const SlotCls<TokT>& S, unsigned i, const Batch& B,
                                                 unsigned long long* LRt, size_t lr_member,
                                                 unsigned* lds, bool narrow, const LdsU32* sm_a,
                                                 const LdsU32* sm_b, const LdsU32* sm_n, const LdsU8* pm, bool use_pm,
                                                 unsigned& singles, LdsU32* bm, unsigned tbw, unsigned mark_from,
                                                 uint32_t* tags = nullptr, unsigned f = 0) {
    constexpr int W = slot_w(C);
    constexpr int V = W * (int)sizeof(TokT) / 16;
    TokT* s = S.slot + (size_t)i * W;
    uint4 r[V];
#pragma unroll
    for (int v = 0; v < V; ++v) r[v] = reinterpret_cast<const uint4*>(s)[v];
    // the count: issued with the slot in a full scan (most words hit early); in list mode, where
    // most entries miss, only on a hit, beside the claim (one random line less per missing entry,
    // and the claim's round trip covers the load)
    unsigned long long c = 0;
    if (!(kLateCount && tags)) c = S.cnt[i];
    TokT e[W];
    __builtin_memcpy(e, r, sizeof(e));
    // the members this word holds: no member's b is another's a and the new tokens are fresh, so
    // a rewrite neither makes nor breaks another member's pair and the original word decides
    unsigned hits = 0;
    if (use_pm && W <= 32) {   // each pair of the word looked up in the batch's pair table, eight
        // lookups in flight at a time (the 64-id class, rare, compares with every member)
        const uint32_t len = (uint32_t)e[0];
#pragma unroll
        for (int q0 = 1; q0 + 1 < W; q0 += 8) {
            unsigned v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = q0 + u;
                v[u] = q + 1 < W ? (unsigned)pm[pair_h12((unsigned)e[q + 1 < W ? q : 1], (unsigned)e[q + 1 < W ? q + 1 : 1])] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int q = q0 + u;
                if (q + 1 < W && (uint32_t)q < len && v[u]) {
                    const unsigned x = (unsigned)e[q + 1 < W ? q : 1], y = (unsigned)e[q + 1 < W ? q + 1 : 1];
                    if (v[u] != 0xFFu) {
                        const unsigned j = v[u] - 1;
                        hits |= (unsigned)((x == sm_a[j]) & (y == sm_b[j])) << j;
                    } else {   // two members share the slot
                        for (int j = 0; j < B.k; ++j) hits |= (unsigned)((x == sm_a[j]) & (y == sm_b[j])) << j;
                    }
                }
            }
        }
    } else {
        for (int j = 0; j < B.k; ++j) {
            const TokT ta = (TokT)sm_a[j], tb = (TokT)sm_b[j];
            bool hit = false;
#pragma unroll
            for (int q = 1; q + 1 < W; ++q) hit |= (e[q] == ta) & (e[q + 1] == tb);
            hits |= (unsigned)hit << j;
        }
    }
    // claimed only on a hit (most list entries miss: no atomic for them).  A word rewritten under
    // another thread's claim was loaded after that claim, so its copy here, torn or not, ends in a
    // failed claim or in no hit: only the claimant ever writes it.
    if (!hits) return;
    if (kLateCount && tags) c = S.cnt[i];
    if (tags && atomicMax(&tags[f], B.batch_id) >= B.batch_id) return;
    if (kRegRewrite && W <= kRegRewriteMaxW) {   // every member in registers, one compacting store
        const auto sink_of = [&](int j) {
            return DeltaSinkN<kLdsB>{LRt + (size_t)j * lr_member, (LdsU32*)(lds + 2 * kLdsB * j), bm + j * tbw,
                                     mark_from, narrow};
        };
        const uint32_t nl = rewrite_slot_members(e, s, hits, sm_a, sm_b, sm_n, c, sink_of);
        singles += nl < 2;
        return;
    }
    bool first = true;
    while (hits) {
        const int j = __builtin_ctz(hits);
        hits &= hits - 1;
        if (!first) {   // a second member: the word as rewritten (this thread's own stores)
#pragma unroll
            for (int v = 0; v < V; ++v) r[v] = reinterpret_cast<const uint4*>(s)[v];
            __builtin_memcpy(e, r, sizeof(e));
        }
        first = false;
        const DeltaSinkN<kLdsB> D{LRt + (size_t)j * lr_member, (LdsU32*)(lds + 2 * kLdsB * j), bm + j * tbw,
                                  mark_from, narrow};
        const uint32_t nl = rewrite_slot(e, s, (TokT)sm_a[j], (TokT)sm_b[j], (TokT)sm_n[j], c, D);
        if (nl < 2) { ++singles; break; }
    }
}

// The merge-apply rewrite of a trip's batch B (the batch record in memory for k_merge_batch, the
// workgroup's own LDS copy in k_trip).  l_lr: the workgroup's LDS-summed cells (2 kLdsB per member).
template <class TokT>
__device__ __forceinline__ void merge_body(RoundState* __restrict__ st, const Batch& B, PairsDev P, ToksDev K,
                                           WordsDev<TokT> W, IndexDev X, unsigned long long* __restrict__ LRbase,
                                           size_t lr_member, size_t lr_parity, uint32_t* __restrict__ tags,
                                           const CellMarks CM, unsigned* l_lr) {
    __shared__ unsigned s_ma[kMaxBatch], s_mb[kMaxBatch], s_mn[kMaxBatch];   // the members' tokens
    __shared__ unsigned s_bm[kMaxBatch * kTBMax];   // the members' touched-block bitmaps (CellMarks)
    __shared__ unsigned s_pre[kMaxBatch + 1], s_lbeg[kMaxBatch];   // list prefix sums, list starts
    __shared__ unsigned s_pm[kPairSlots / 4];   // the batch's pair table (bytes; kPairFilterK)
    const int tid = threadIdx.x;
    // every field the prologue needs in one round trip (none depends on another)
    const int stop = B.stop, k = B.k, b_trip = B.trip, b_ntok = B.ntok, b_prev_k = B.prev_k,
              b_prev_sparse = B.prev_sparse;
    const unsigned idle_from = B.idle_from;
    // 32-bit LDS cells hold every member's sums (run-time test knob BPE355_LDS_CELLS=0: every cell
    // global, the path of a batch whose P1 count reaches 2^32)
    const bool narrow = B.m[0].cnt < st->narrow_limit;
    unsigned ma = 0, mb = 0, mn = 0, mlb = 0, mpre = 0;
    if (tid < kMaxBatch) { ma = B.m[tid].a; mb = B.m[tid].b; mn = B.m[tid].nw; mlb = B.m[tid].list_beg; }
    if (tid <= kMaxBatch) mpre = B.list_pre[tid];
    if (stop) return;
    const unsigned tbw = CM.tbw;
    const unsigned mark_from = tbw ? 2 * CM.dense_tok : ~0u;
    // the previous trip's cells (the other parity, read by its apply) are cleared here, spread
    // over the whole grid: workgroups without words do their share at once, the others after
    // their flush, so the stores never wait in front of a rewrite's loads.  With marks: the dense
    // token prefix, the blocks the previous apply listed (CM.tbc), and that parity's bitmaps
    auto clear_prev = [&]() {
        unsigned long long* LRo = LRbase + (size_t)((b_trip + 1) & 1) * lr_parity;
        const unsigned S = gridDim.x * blockDim.x, g = blockIdx.x * blockDim.x + tid;
        const unsigned pk = (unsigned)b_prev_k;
        unsigned* TBo = CM.tb + (size_t)((b_trip + 1) & 1) * kTBRep * kMaxBatch * tbw;
        if (tbw)   // that parity's bitmaps (the marks its merge made, whatever its apply did with them)
            for (unsigned q = g; q < kTBRep * kMaxBatch * tbw; q += S) TBo[q] = 0u;
        if (!tbw || !b_prev_sparse) {   // the previous apply scanned every cell: clear every cell
            const unsigned nprev = (unsigned)b_ntok;   // 16-byte cell pairs per member
            for (unsigned q = g; q < pk * nprev; q += S)
                st_merge(reinterpret_cast<uint4*>(&LRo[(size_t)(q / nprev) * lr_member + 2 * (q % nprev)]),
                         make_uint4(0, 0, 0, 0));
            return;
        }
        const unsigned nd2 = min(CM.dense_tok, (unsigned)b_ntok);   // 16-byte cell pairs per member
        for (unsigned q = g; q < pk * nd2; q += S)
            st_merge(reinterpret_cast<uint4*>(&LRo[(size_t)(q / nd2) * lr_member + 2 * (q % nd2)]), make_uint4(0, 0, 0, 0));
        const unsigned nbk = 32 * tbw;   // blocks per member
        for (unsigned q = g; q < pk * nbk; q += S) {
            const unsigned j = q / nbk, blk = q % nbk;
            if ((CM.tbc[j * tbw + (blk >> 5)] >> (blk & 31)) & 1u) {
                uint4* c = reinterpret_cast<uint4*>(&LRo[(size_t)j * lr_member + 64 * (size_t)blk]);
#pragma unroll 8
                for (int u = 0; u < 32; ++u) st_merge(&c[u], make_uint4(0, 0, 0, 0));
            }
        }
    };
    // Member j's pop and new-token registration (nothing in this launch reads them: the apply
    // and the next trip do) go to the first k workgroups without words when there are enough of
    // them, else to workgroups 0..k-1 after their rewrite: either way no rewrite waits behind the
    // registration's chain of dependent loads (the token bytes of a and b)
    const unsigned gl = min(gridDim.x, W.lblk0);   // the slot-class blocks that exist
    const unsigned busy = idle_from == ~0u ? gl : min(gl, (idle_from + blockDim.x - 1) / blockDim.x);
    const unsigned reg0 = busy + (unsigned)k <= gl ? busy : 0u;   // (the grid has >= kMaxBatch blocks)
    const int reg_j = (int)blockIdx.x - (int)reg0;
    auto register_member = [&]() {
        if (reg_j < 0 || reg_j >= k) return;
        const BatchMember& M = B.m[reg_j];
        if (tid == 0) {
            P.cnt[M.slot] = 0;                       // byte_pair_frequencies.pop(best_pair)
            atomicAnd(&P.flag[M.slot], ~kPresent);
            X.beg[M.nw] = M.cov_beg;
            X.len[M.nw] = M.cov_len;
        }
        if (M.isnew) {
            if (M.pool_off + M.ln <= st->pool_cap) {
                const unsigned la = K.len[M.a];
                for (unsigned i = tid; i < M.ln; i += blockDim.x) K.pool[M.pool_off + i] = concat_byte(K, M.a, la, M.b, i);
            } else if (tid == 0) {
                atomicOr(&st->err, ERR_POOL);
            }
            if (tid == 0) {
                K.off[M.nw] = M.pool_off; K.len[M.nw] = M.ln;
                K.hash[M.nw] = M.hash; K.pw[M.nw] = M.pw; K.key8[M.nw] = M.k8;
            }
        }
    };
    {   // list mode: workgroups past the listed words have no rewrite -- skip their LDS clear,
        // barriers and flush
        const unsigned bid = blockIdx.x;
        if (bid >= busy && bid < gl) {
            register_member();
            clear_prev();
            if (tid == 0) probe_done(st, &st->probe_merge_done, b_trip, 14);
            return;
        }
    }
    if (tid < k) {
        s_ma[tid] = ma; s_mb[tid] = mb; s_mn[tid] = mn;
        s_lbeg[tid] = mlb;
    }
    if (tid <= k) s_pre[tid] = mpre;
    if (blockIdx.x == 0 && tid == 0) probe_stamp(st, B.trip, 5);
    for (unsigned q = tid; q < 2 * kLdsB * (unsigned)k; q += blockDim.x) l_lr[q] = 0;
    for (unsigned q = tid; q < tbw * (unsigned)k; q += blockDim.x) s_bm[q] = 0;
    LdsU32* lbm = (LdsU32*)s_bm;
    unsigned long long* LRt = LRbase + (size_t)(B.trip & 1) * lr_parity;   // member j at + j * lr_member
    const bool use_pm = kPairFilterK > 0 && k >= kPairFilterK;   // (uniform)
    if (use_pm)
        for (unsigned q = tid; q < kPairSlots / 4; q += blockDim.x) s_pm[q] = 0;

    __syncthreads();   // l_lr cleared
    if (use_pm) {   // member j's pair -> slot: j + 1, or 0xFF where two members share a slot
        if (tid < 64) {
            const bool m = tid < k;
            const unsigned h = pair_h12(ma, mb);
            bool coll = false;
#pragma unroll
            for (int j = 0; j < kMaxBatch; ++j) {
                const int hj = __shfl((int)h, j);   // (every lane active: lane j supplies its slot)
                coll |= j < k && j != tid && hj == (int)h;
            }
            if (m) reinterpret_cast<uint8_t*>(s_pm)[h] = coll ? (uint8_t)0xFFu : (uint8_t)(tid + 1);
        }
        __syncthreads();
    }
    const LdsU8* pmp = (const LdsU8*)s_pm;
    if (blockIdx.x == 0 && tid == 0) probe_stamp(st, B.trip, 6);

    unsigned singles = 0;
    const unsigned bid = blockIdx.x;
    // the host may launch fewer blocks than the slot-class layout has (short posting lists late
    // in training): every loop below strides over the nb blocks that exist
    const unsigned nb = gridDim.x < W.lblk0 ? gridDim.x : W.lblk0;
    if (k == 1) {
        // one member: the per-round rewrite (index list or a scan of every slot)
        const BatchMember& M = B.m[0];
        const TokT ta = (TokT)M.a, tb = (TokT)M.b, tn = (TokT)M.nw;
        const DeltaSinkN<kLdsB> D{LRt, (LdsU32*)l_lr, lbm, mark_from, narrow};
        if (M.use_list && bid < nb) {
            const uint32_t* L = X.list + M.list_beg;
            for (unsigned i = bid * blockDim.x + tid; i < M.list_len; i += nb * blockDim.x) {
                const unsigned f = L[i];
                if (f < W.off[1]) merge_one<TokT, 0>(W.c[0], f, ta, tb, tn, D, singles);
                else if (f < W.off[2]) merge_one<TokT, 1>(W.c[1], f - W.off[1], ta, tb, tn, D, singles);
                else if (f < W.off[3]) merge_one<TokT, 2>(W.c[2], f - W.off[2], ta, tb, tn, D, singles);
                else merge_one<TokT, 3>(W.c[3], f - W.off[3], ta, tb, tn, D, singles);
            }
        } else if (!M.use_list) {
            for (unsigned bb = bid; bb < W.lblk0; bb += nb) {
                if (bb < W.c[1].blk0) {
                    if (bb < W.c[0].blk0 + W.c[0].nblk)
                        scan_class<TokT, 0>(W.c[0], bb - W.c[0].blk0, ta, tb, tn, D, singles);
                } else if (bb < W.c[2].blk0) {
                    scan_class<TokT, 1>(W.c[1], bb - W.c[1].blk0, ta, tb, tn, D, singles);
                } else if (bb < W.c[3].blk0) {
                    scan_class<TokT, 2>(W.c[2], bb - W.c[2].blk0, ta, tb, tn, D, singles);
                } else {
                    scan_class<TokT, 3>(W.c[3], bb - W.c[3].blk0, ta, tb, tn, D, singles);
                }
            }
        }
    } else if (bid < nb) {
        // several members: every word that can contain one of them, once, all members in order
        if (B.full_scan) {
            const unsigned total = W.off[kNumCls];
            for (unsigned f = bid * blockDim.x + tid; f < total; f += nb * blockDim.x) {
                if (f < W.off[1]) merge_word_batch<TokT, 0>(W.c[0], f,  B, LRt, lr_member, l_lr, narrow, (const LdsU32*)s_ma, (const LdsU32*)s_mb, (const LdsU32*)s_mn, pmp, use_pm, singles, lbm, tbw, mark_from);
                else if (f < W.off[2]) merge_word_batch<TokT, 1>(W.c[1], f - W.off[1],  B, LRt, lr_member, l_lr, narrow, (const LdsU32*)s_ma, (const LdsU32*)s_mb, (const LdsU32*)s_mn, pmp, use_pm, singles, lbm, tbw, mark_from);
                else if (f < W.off[3]) merge_word_batch<TokT, 2>(W.c[2], f - W.off[2],  B, LRt, lr_member, l_lr, narrow, (const LdsU32*)s_ma, (const LdsU32*)s_mb, (const LdsU32*)s_mn, pmp, use_pm, singles, lbm, tbw, mark_from);
                else merge_word_batch<TokT, 3>(W.c[3], f - W.off[3],  B, LRt, lr_member, l_lr, narrow, (const LdsU32*)s_ma, (const LdsU32*)s_mb, (const LdsU32*)s_mn, pmp, use_pm, singles, lbm, tbw, mark_from);
            }
        } else {
            const unsigned total = B.list_pre[k];
            for (unsigned i = bid * blockDim.x + tid; i < total; i += nb * blockDim.x) {
                int j = 0;
                // the member whose list holds entry i: binary search of the LDS prefix sums, steps
                // from the largest power of two below kMaxBatch (any cap, not only powers of two)
                for (int step = kListTopStep; step > 0; step >>= 1)
                    if (j + step < k && i >= s_pre[j + step]) j += step;
                const unsigned f = X.list[s_lbeg[j] + (i - s_pre[j])];
                // a word on several members' lists is rewritten by the first thread to claim it
                if (f < W.off[1]) merge_word_batch<TokT, 0>(W.c[0], f,  B, LRt, lr_member, l_lr, narrow, (const LdsU32*)s_ma, (const LdsU32*)s_mb, (const LdsU32*)s_mn, pmp, use_pm, singles, lbm, tbw, mark_from, tags, f);
                else if (f < W.off[2]) merge_word_batch<TokT, 1>(W.c[1], f - W.off[1],  B, LRt, lr_member, l_lr, narrow, (const LdsU32*)s_ma, (const LdsU32*)s_mb, (const LdsU32*)s_mn, pmp, use_pm, singles, lbm, tbw, mark_from, tags, f);
                else if (f < W.off[3]) merge_word_batch<TokT, 2>(W.c[2], f - W.off[2],  B, LRt, lr_member, l_lr, narrow, (const LdsU32*)s_ma, (const LdsU32*)s_mb, (const LdsU32*)s_mn, pmp, use_pm, singles, lbm, tbw, mark_from, tags, f);
                else merge_word_batch<TokT, 3>(W.c[3], f - W.off[3],  B, LRt, lr_member, l_lr, narrow, (const LdsU32*)s_ma, (const LdsU32*)s_mb, (const LdsU32*)s_mn, pmp, use_pm, singles, lbm, tbw, mark_from, tags, f);
            }
        }
    }
    if (bid >= W.lblk0 && bid < W.lblk0 + W.lnblk) {   // long words: every member in order
        for (unsigned i = (bid - W.lblk0) * blockDim.x + tid; i < W.ln; i += W.lnblk * blockDim.x) {
            uint32_t len = W.llen[i];
            if (len < 2) continue;
            TokT* t = W.ltok + W.lbeg[i];
            for (int j = 0; j < k && len >= 2; ++j) {
                const TokT ta = (TokT)B.m[j].a, tb = (TokT)B.m[j].b;
                bool hit = false;
                for (uint32_t q = 0; q + 1 < len && !hit; ++q) hit = (t[q] == ta) & (t[q + 1] == tb);
                if (!hit) continue;
                const DeltaSinkN<kLdsB> D{LRt + (size_t)j * lr_member, (LdsU32*)(l_lr + 2 * kLdsB * j), lbm + j * tbw,
                                          mark_from, narrow};
                len = rewrite_word(t, len, ta, tb, (TokT)B.m[j].nw, W.lcnt[i], D, false);
                W.llen[i] = len;
                singles += (len < 2);
            }
        }
    }
    singles = wave_sum(singles);   // words that became one token (rare: no contention)
    // (the apply adds them to n_single, which this trip's select phase reads in every workgroup)
    if ((tid & 63) == 0 && singles) atomicAdd(&st->n_single_new, singles);
    __syncthreads();
    if (blockIdx.x == 0 && tid == 0) probe_stamp(st, B.trip, 7);
    for (unsigned q = tid; q < 2 * kLdsB * (unsigned)k; q += blockDim.x) {
        const unsigned v = l_lr[q];
        if (v) atomicAdd(&LRt[(size_t)(q / (2 * kLdsB)) * lr_member + q % (2 * kLdsB)], (unsigned long long)v);
    }
    if (tbw) {   // the touched blocks, into this workgroup's replica of this parity's bitmaps
        unsigned* TBt = CM.tb + ((size_t)(B.trip & 1) * kTBRep + blockIdx.x % kTBRep) * kMaxBatch * tbw;
        for (unsigned q = tid; q < tbw * (unsigned)k; q += blockDim.x) {
            const unsigned v = s_bm[q];
            if (v) atomicOr(&TBt[q], v);
        }
    }
    if (blockIdx.x == 0 && tid == 0) probe_stamp(st, B.trip, 8);
    clear_prev();
    register_member();
    if (BPE355_PROBE_CODE && st->probe) {
        __syncthreads();
        if (tid == 0) probe_done(st, &st->probe_merge_done, B.trip, 14);
    }
}

// the rewrite of the batch k_select decided (BPE355_FOLD=0)
template <class TokT>
#ifndef BPE355_MERGE_WAVES
#define BPE355_MERGE_WAVES 4
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sizeof(TokT) == 2 ? BPE355_MERGE_WAVES : 2))) k_merge_batch(RoundState* __restrict__ st, const Batch* __restrict__ bt,
                                                     PairsDev P, ToksDev K, WordsDev<TokT> W, IndexDev X,
                                                     unsigned long long* __restrict__ LRbase, size_t lr_member,
                                                     size_t lr_parity, uint32_t* __restrict__ tags, CellMarks CM) {
    __shared__ unsigned l_lr[2 * kLdsB * kMaxBatch];
    merge_body<TokT>(st, *bt, P, K, W, X, LRbase, lr_member, lr_parity, tags, CM, l_lr);
}

// One trip's select and merge in ONE launch.  Every workgroup decides the
// batch itself -- the decision is a function of state that nothing in this launch changes
// (select_core) -- so no workgroup waits for another and the select's kernel boundary is gone.
// Block 0 also publishes the batch record the apply reads.  Measured on the bench config it is
// no faster than k_select + k_merge_batch (257.4-258.3 vs 255.4 ms of merges): the boundary it
// saves (2-4 us) is paid back by the decision's own loads, which every workgroup repeats (the
// apply's 24 KB of partials arrive 1.3 us later with 1024 readers than with one), so it is the
// BPE355_FOLD=1 option, not the default.  The select's LDS and the
// rewrite's LDS-summed cells share one union: the cells are cleared after the decision.
template <class TokT>
__global__ void __launch_bounds__(kTripThreads) k_trip(RoundState* __restrict__ st, BatchState* __restrict__ bs,
                                              PairsDev P, ToksDev K, WordsDev<TokT> W, IndexDev X,
                                              Batch* __restrict__ bt, const Partial* __restrict__ part,
                                              const Partial* __restrict__ lists, SelOut O,
                                              unsigned long long* __restrict__ LRbase, size_t lr_member,
                                              size_t lr_parity, uint32_t* __restrict__ tags, CellMarks CM) {
    __shared__ union TripLds {
        SelLds sel;
        unsigned lr[2 * kLdsB * kMaxBatch];
    } u;
    __shared__ Batch s_b;
    const bool pub = blockIdx.x == 0;
    select_core<kTripThreads>(st, bs, K, X, part, lists, s_b, u.sel, O, pub);
    __syncthreads();
    if (pub) {   // the apply's copy of the decision
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&s_b);
        uint32_t* dst = reinterpret_cast<uint32_t*>(bt);
        for (unsigned i = threadIdx.x; i < (unsigned)(sizeof(Batch) / 4); i += blockDim.x) dst[i] = src[i];
    }
    if (s_b.stop) return;
    merge_body<TokT>(st, s_b, P, K, W, X, LRbase, lr_member, lr_parity, tags, CM, u.lr);
}

// Apply the trip's deltas and list the next trip's candidates.  Items:
//   v < k * 4 * ntb        member j = v / (4 ntb), token x, op as in k_apply_argmax; its key has
//                          ONE updater unless x is one of the batch's tokens S = {a_j, b_j, new_j};
//   next |S|^2 items       every key with both tokens in S: one item sums all the members'
//                          contributions to it;
//   next nC_base items     C entries: untouched ones keep their counts during the apply, touched
//                          ones are evaluated by their updater (final count).
// Every present key >= T among them is a candidate; each workgroup writes its exact top-kTopM
// (sorted) to part[blockIdx.x * kTopM ...] and k_select merges the lists.  scan_only: the C
// entries alone (after a rebuild of C).
#ifndef BPE355_APPLY_ITEMS
#define BPE355_APPLY_ITEMS 2
#endif
constexpr unsigned kBatchApplyItems = BPE355_APPLY_ITEMS;   // items per thread per pass of k_apply_batch
#ifndef BPE355_APPLY_C_FIRST
#define BPE355_APPLY_C_FIRST 0
#endif
constexpr bool kApplyCFirst = BPE355_APPLY_C_FIRST != 0;
constexpr unsigned kApplyBatchThreads = 256;
constexpr unsigned kApplyCLds = 256;
constexpr unsigned kSFilterWords = 128;   // C admissions a workgroup stages in LDS (more: direct appends)
__global__ void __launch_bounds__(kApplyBatchThreads) k_apply_batch(RoundState* __restrict__ st,
                                                                    BatchState* __restrict__ bs,
                                                                    const Batch* __restrict__ bt, PairsDev P, ToksDev K,
                                                                    unsigned long long* __restrict__ LRbase,
                                                                    size_t lr_member, size_t lr_parity, unsigned ntb,
                                                                    Partial* __restrict__ part,
                                                                    Partial* __restrict__ list, int scan_only,
                                                                    CellMarks CM, int sparse_hint) {
    __shared__ unsigned s_tok[3 * kMaxBatch];
    __shared__ unsigned s_tw[kMaxBatch * kTBMax];   // touched-block bitmaps (the replicas' OR)
    __shared__ unsigned short s_tl[kTLCap];         // touched blocks past the dense prefix: j << 11 | block
    __shared__ unsigned s_wsum[kApplyBatchThreads / 64];
    __shared__ unsigned s_role[3 * kMaxBatch];   // S entry: members' mask << 3 | role (1 a, 2 b, 4 new)
    __shared__ unsigned s_grp[2 * kMaxBatch];    // member j's a group (2j) and b group (2j + 1)
    __shared__ unsigned s_filt[kSFilterWords];   // bit (x mod 4096): x may be in S
    __shared__ int s_ns;
    __shared__ Cand s_wave[kApplyBatchThreads / 64];
    __shared__ Partial s_lst[kListCap];
    __shared__ uint4 s_cadd[kApplyCLds];
    __shared__ unsigned s_nl, s_nc, s_lbase, s_cbase, s_ins;
    const Batch& B = *bt;
    const int tid = threadIdx.x;
    // every field the prologue needs in one round trip (none depends on another); the batch is
    // valid memory even when stale (scan_only), so its loads need no guard
    static_assert(offsetof(BatchMember, b) == 4 && offsetof(BatchMember, nw) == 8, "a, b, nw adjacent");
    const int b_stop = B.stop, b_k = B.k, b_trip = B.trip, b_ntok = B.ntok;
    const unsigned b_fresh = B.n_fresh, b_nC = B.nC_base;
    const long long b_T2 = B.T2next;
    const long long T = st->T, T2bs = bs->T2;
    const int bs_trip = bs->trip;
    const unsigned st_nC = st->nC;   // scan_only: no admissions during the scan, so stable
    const unsigned t_raw = tid < 3 * kMaxBatch ? reinterpret_cast<const unsigned*>(&B.m[tid / 3])[tid % 3] : ~0u;
    static_assert(offsetof(BatchMember, gb) == offsetof(BatchMember, ga) + 4, "ga, gb adjacent");
    const unsigned g_raw = tid < 3 * kMaxBatch && tid % 3 < 2 ? (&B.m[tid / 3].ga)[tid % 3] : 0u;
    // touched-block bitmaps of both parities (CellMarks), issued with the batch record's loads
    // rather than behind them (the parity is the batch's); kTBW words per thread
    constexpr unsigned kTBW = (kMaxBatch * kTBMax + kApplyBatchThreads - 1) / kApplyBatchThreads;
    unsigned t2[2][kTBW];
    {
        const bool want = sparse_hint && !scan_only && CM.tbw != 0;
#pragma unroll
        for (unsigned pty = 0; pty < 2; ++pty)
#pragma unroll
            for (unsigned u = 0; u < kTBW; ++u) {
                const unsigned q = tid * kTBW + u;
                unsigned v = 0;
                if (want && q < kMaxBatch * CM.tbw)
#pragma unroll
                    for (unsigned r = 0; r < kTBRep; ++r)
                        v |= CM.tb[((size_t)pty * kTBRep + r) * kMaxBatch * CM.tbw + q];
                t2[pty][u] = v;
            }
    }
    if (!scan_only && b_stop) {   // no trip: part[] and the list keep what the next select reads
        if (b_stop > 0 && blockIdx.x == 0 && tid == 0) st->halt = b_stop;   // the select's halt
        return;
    }
    // the threshold of the list this apply fills (the trip's decision, or after a rebuild the
    // last one), and which of the two lists: the next trip's parity
    const long long T2raw = scan_only ? T2bs : b_T2;
    const unsigned lpar = (unsigned)(scan_only ? bs_trip : b_trip + 1) & 1u;
    list += (size_t)lpar * kListCap;
    const int k = scan_only ? 0 : b_k;
    const bool pw0 = !scan_only && blockIdx.x == 0 && tid == 0;
    if (pw0) probe_stamp(st, b_trip, 9);
    // touched blocks (CellMarks): listed from cm.sparse_from tokens on (below, the dense scan of
    // every cell is cheaper than building the list)
    const unsigned tbw = CM.tbw;
    const unsigned ntb_all = scan_only ? ntb : min(ntb, (unsigned)b_ntok + b_fresh);
    const bool sparse = sparse_hint && !scan_only && tbw != 0 && ntb_all > CM.sparse_from;   // (uniform)
    unsigned tw[kTBW];
#pragma unroll
    for (unsigned u = 0; u < kTBW; ++u)
        tw[u] = sparse && tid * kTBW + u < (unsigned)k * tbw ? t2[b_trip & 1][u] : 0u;
    if (tid < 64) {   // wave 0: S deduplicated (a == b is possible only when k == 1), lane i = entry i
        static_assert(3 * kMaxBatch <= 64, "S fits one wave");
        const int i = tid;
        const bool have = i < 3 * k;
        const unsigned ti = have ? t_raw : ~0u;
        // For k > 1 a token has one role: no member's b is another's a, a != b, and the new tokens
        // are fresh ids (select_core's rule); an a (a b) several members share is kept once, by
        // the group's first member, with the group's mask.  For k == 1 only a == b can repeat (a
        // new token's bytes are longer than a's and b's), so no general dedupe pass is needed.
        unsigned roles = 1u << (i % 3);
        const unsigned gm = i % 3 == 2 ? 1u << (i / 3) : g_raw;   // the members behind this entry
        bool dup = false;
        if (k == 1 && __builtin_amdgcn_readlane((int)ti, 0) == __builtin_amdgcn_readlane((int)ti, 1)) {
            if (i == 0) roles = 3u;   // a == b: one entry, both roles
            dup = i == 1;
        }
        if (have && i % 3 < 2) s_grp[2 * (i / 3) + i % 3] = gm;
        const bool keep = have && !dup && gm != 0;
        const unsigned long long km = __ballot(keep);
        for (unsigned w = i; w < kSFilterWords; w += 64) s_filt[w] = 0;
        if (keep) {
            const unsigned pos = __builtin_amdgcn_mbcnt_hi((unsigned)(km >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)km, 0u));
            s_tok[pos] = ti;
            s_role[pos] = gm << 3 | roles;
            atomicOr(&s_filt[(ti >> 5) % kSFilterWords], 1u << (ti & 31));
        }
        if (i == 0) {
            s_ns = __popcll(km);
            s_nl = 0;
            s_nc = 0;
            s_ins = 0;
        }
    }
    __syncthreads();
    const int ns = s_ns;
    const unsigned long long* LRc = LRbase + (size_t)(b_trip & 1) * lr_parity;
    ntb = ntb_all;   // token ids after this trip
    const unsigned per_member = 4 * ntb;
    // the cell items: every (member, token, op) densely, or (sparse) the dense token prefix of every
    // member plus the touched blocks past it, 128 items (32 tokens x 4 ops) per block
    const unsigned nD = CM.dense_tok / 32;   // dense-prefix blocks per member
    unsigned n_cell = (unsigned)k * per_member;
    bool listed = false;
    if (sparse) {
        // a token group's first member updates (x, a) / (b, y) for the whole group from the
        // group's summed cells: its blocks must cover every group member's
#pragma unroll
        for (unsigned u = 0; u < kTBW; ++u) {
            const unsigned q = tid * kTBW + u;
            if (q < (unsigned)k * tbw) s_tw[q] = tw[u];
        }
        __syncthreads();
        // (from the members' own bitmaps only: every workgroup must list exactly the same blocks,
        // since the items are numbered across the grid -- a leader that is itself in another
        // leader's group must not pass on bits in an order that depends on timing)
        unsigned c = 0;
#pragma unroll
        for (unsigned u = 0; u < kTBW; ++u) {
            const unsigned q = tid * kTBW + u;
            if (q >= (unsigned)k * tbw) continue;
            const unsigned j = q / tbw, w = q % tbw;
            unsigned gm = (s_grp[2 * j] | s_grp[2 * j + 1]) & ~(1u << j);
            while (gm) {
                const unsigned m = (unsigned)__builtin_ctz(gm);
                gm &= gm - 1;
                tw[u] |= s_tw[m * tbw + w];
            }
            c += __popc(tw[u]);
        }
        // exclusive scan of the counts over the workgroup
        unsigned inc = c;
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned t = __shfl_up(inc, d);
            if ((tid & 63) >= d) inc += t;
        }
        if ((tid & 63) == 63) s_wsum[tid >> 6] = inc;
        __syncthreads();
        unsigned base = 0, T = 0;
        for (int w = 0; w < (int)(kApplyBatchThreads / 64); ++w) {
            const unsigned ws = s_wsum[w];
            base += w < (tid >> 6) ? ws : 0u;
            T += ws;
        }
        base += inc - c;
        if (T <= kTLCap) {
            listed = true;
#pragma unroll
            for (unsigned u = 0; u < kTBW; ++u) {
                unsigned v = tw[u];
                const unsigned q = tid * kTBW + u;
                while (v) {
                    const unsigned bit = (unsigned)__builtin_ctz(v);
                    v &= v - 1;
                    s_tl[base++] = (unsigned short)((q / tbw) << 11 | ((q % tbw) * 32 + bit));
                }
            }
            n_cell = ((unsigned)k * nD + T) * 128;
        }
        if (CM.sig) {   // (test knob) this workgroup's view: T and a hash of its bitmaps
            unsigned long long hsh = 0;
#pragma unroll
            for (unsigned u = 0; u < kTBW; ++u) hsh += (unsigned long long)tw[u] * (0x9E3779B97F4A7C15ull * (tid * kTBW + u + 1));
            for (int o = 32; o > 0; o >>= 1) hsh += __shfl_xor(hsh, o);
            if ((tid & 63) == 0) atomicAdd(&CM.sig[1 + blockIdx.x], hsh + ((unsigned long long)T << 48));
        }
        if (blockIdx.x == 0)   // for the next merge's clear
#pragma unroll
            for (unsigned u = 0; u < kTBW; ++u) {
                const unsigned q = tid * kTBW + u;
                if (q < (unsigned)k * tbw) CM.tbc[q] = tw[u];
            }
        __syncthreads();
    }
    // cell item v -> member j, token x, op (false: no such cell)
    auto cell_of = [&](unsigned v, unsigned& j, unsigned& x, unsigned& op) -> bool {
        if (!listed) {
            j = v / per_member;
            const unsigned r = v % per_member;
            x = r >> 2;
            op = r & 3;
            return true;
        }
        const unsigned slot = v >> 7, r = v & 127;
        unsigned blk;
        if (slot < (unsigned)k * nD) {
            j = slot / nD;
            blk = slot % nD;
        } else {
            const unsigned e = s_tl[slot - (unsigned)k * nD];
            j = e >> 11;
            blk = e & 2047u;
        }
        x = blk * 32 + (r >> 2);
        op = r & 3;
        return x < ntb;
    };
    const unsigned n_sp = (unsigned)(ns * ns);
    const unsigned nC0 = scan_only ? st_nC : b_nC;
    const unsigned n_items = n_cell + n_sp + nC0;
    const unsigned g = blockIdx.x * blockDim.x + tid;
    const unsigned S = gridDim.x * blockDim.x;
    // (the previous trip's cells were cleared by this trip's merge)
    if (pw0) probe_stamp(st, b_trip, 10);
    auto find_S = [&](unsigned x) -> int {   // x's entry in S, or -1
        if (!((s_filt[(x >> 5) % kSFilterWords] >> (x & 31)) & 1u)) return -1;
        int r = -1;
        for (int u = 0; u < ns; ++u) r = s_tok[u] == x ? u : r;
        return r;
    };
    auto in_S = [&](unsigned x) { return find_S(x) >= 0; };
    // the cells at index ci of the members in mask (one load unless members share the token)
    auto cell_sum = [&](unsigned mask, size_t ci) -> unsigned long long {
        unsigned long long t = 0;
        while (mask) {
            const unsigned j = (unsigned)__builtin_ctz(mask);
            mask &= mask - 1;
            t += LRc[(size_t)j * lr_member + ci];
        }
        return t;
    };
    const long long T2 = T2raw < T ? T : T2raw;
    Cand best = cand_none();   // this thread's best candidate (exact argmax)
    unsigned n_ins = 0;        // pair-table keys this thread inserted
    // a candidate for the list (>= T2) and for this thread's best
    auto offer = [&](const Cand& c) {
        if (cand_better(c, best, K.pool, K.off, K.len)) best = c;
        const bool listed = c.cnt != LLONG_MIN && c.cnt >= T2;
        const unsigned li = wave_append(listed, &s_nl);   // one LDS atomic per wave
        if (listed && li < kListCap) s_lst[li] = Partial{c.cnt, c.ka, c.kb, c.slot, c.a, c.b, 0};
    };
    // an increment across T admits the key to C
    auto admit = [&](bool pred, size_t s, unsigned p, unsigned q) {
        const unsigned ci = wave_append(pred, &s_nc);
        if (!pred) return;
        if (ci < kApplyCLds) {
            s_cadd[ci] = make_uint4((unsigned)s, p, q, 0u);
        } else {
            const unsigned idx = atomicAdd(&st->nC, 1u);
            if (idx < st->capC) P.C[idx] = make_uint4((unsigned)s, p, q, 0u);
            else atomicOr(&st->err, ERR_C_FULL);
        }
    };
    // an updated key: a candidate if present and >= T
    auto updated = [&](size_t s, unsigned p, unsigned q, long long c, unsigned f, bool inc,
                       unsigned long long kp, unsigned long long kq) {
        if (s == ~(size_t)0 || !(f & kPresent) || c < T) return;
        offer(Cand{c, kp, kq, (unsigned)s, p, q});
        const bool adm = inc && !(f & kInC);
        if (adm) st_apply(&P.flag[s], f | kInC);
        admit(adm, s, p, q);
    };
    // step u of a pass takes items base + u * S + g: a wave's 64 items are contiguous (coalesced)
    // and its steps far apart, so the dense start of each member's cells (the byte tokens, which
    // neighbour everything) spreads over many waves instead of serialising in a few
    // item order: cells, S pairs, C entries; kApplyCFirst puts the C entries (every one a live
    // offer) and the S pairs first -- measured no faster (the apply's tail moves into its items,
    // profiles/r03/h_apply_c_first_ab.txt), so it is off
    auto item = [&](unsigned v) -> unsigned {   // position -> index in the cells, S, C numbering
        if (!kApplyCFirst || v >= n_items) return v;
        if (v < nC0) return n_cell + n_sp + v;
        if (v < nC0 + n_sp) return n_cell + (v - nC0);
        return v - nC0 - n_sp;
    };
    for (unsigned base = 0; base < n_items; base += S * kBatchApplyItems) {
        // three stages over the thread's items, so that their dependent loads overlap instead of
        // chaining item after item: (1) each item's first load -- its cell, an S key's two cells, a
        // C entry; (2) each item's key and the loads it needs -- the key's home slot and both
        // tokens' prefixes (an update), or the slot state and the touched cells (a C entry);
        // (3) the updates and offers
        unsigned long long dv[kBatchApplyItems], dw[kBatchApplyItems];
        uint4 ce[kBatchApplyItems];
#pragma unroll
        for (unsigned u = 0; u < kBatchApplyItems; ++u) {
            const unsigned v = item(base + u * S + g);
            dv[u] = 0;
            dw[u] = 0;
            ce[u] = make_uint4(0, 0, 0, 0);
            unsigned j, x, op;
            if (v < n_cell) {
                if (!cell_of(v, j, x, op)) continue;
                const size_t ci = 2 * (size_t)x + (op >> 1);
                dv[u] = LRc[(size_t)j * lr_member + ci];
                if (kShareTok && !(op & 1)) {   // (x, a_j) or (b_j, x): one updater per token group
                    const unsigned gmask = s_grp[2 * j + (op >> 1)];
                    if (gmask != 1u << j) dv[u] = gmask ? cell_sum(gmask, ci) : 0ull;
                }
            } else if (v < n_cell + n_sp) {
                const unsigned sp = v - n_cell;
                const unsigned p = s_tok[sp / ns], q = s_tok[sp % ns];
                const unsigned rp = s_role[sp / ns], rq = s_role[sp % ns];
                // q's members see p on their left (cell 2p), p's see q on their right (2q + 1)
                if (rq & 5) dv[u] = cell_sum(rq >> 3, 2 * (size_t)p);
                if (rp & 6) dw[u] = cell_sum(rp >> 3, 2 * (size_t)q + 1);
            } else if (v < n_items) {
                ce[u] = P.C[v - n_cell - n_sp];
            }
        }
        unsigned ip[kBatchApplyItems], iq[kBatchApplyItems], how[kBatchApplyItems];   // how: 1 update, 2 inc, 4 C entry
        long long delta[kBatchApplyItems], hc[kBatchApplyItems];
        unsigned long long hk[kBatchApplyItems], kp[kBatchApplyItems], kq[kBatchApplyItems];
        unsigned hf[kBatchApplyItems];
        bool touched[kBatchApplyItems];
#pragma unroll
        for (unsigned u = 0; u < kBatchApplyItems; ++u) {
            const unsigned v = item(base + u * S + g);
            how[u] = 0; ip[u] = 0; iq[u] = 0; delta[u] = 0; touched[u] = false;
            hk[u] = 0; hc[u] = 0; hf[u] = 0; kp[u] = 0; kq[u] = 0;
            unsigned j, x, op;
            if (v < n_cell) {
                const long long d = cell_of(v, j, x, op) ? (long long)dv[u] : 0ll;
                if (d && !in_S(x)) {
                    const BatchMember& M = B.m[j];
                    ip[u] = op <= 1 ? x : (op == 2 ? M.b : M.nw);
                    iq[u] = op == 0 ? M.a : (op == 1 ? M.nw : x);
                    const bool inc = op & 1;
                    delta[u] = inc ? d : -d;
                    how[u] = 1 | (inc ? 2 : 0);
                }
            } else if (v < n_cell + n_sp) {
                const unsigned sp = v - n_cell;
                const unsigned rp = s_role[sp / ns], rq = s_role[sp % ns];
                const long long lq = (long long)dv[u], lp = (long long)dw[u];
                const bool popped = ((rp >> 3) & (rq >> 3)) != 0 && (rp & 1) && (rq & 2);
                long long inc = 0, dec = 0;
                if (rq & 1) dec += lq;
                if (rq & 4) inc += lq;
                if (rp & 2) dec += lp;
                if (rp & 4) inc += lp;
                if (!popped && (inc || dec)) {
                    ip[u] = s_tok[sp / ns];
                    iq[u] = s_tok[sp % ns];
                    delta[u] = inc - dec;
                    how[u] = 1 | (inc != 0 ? 2 : 0);
                }
            } else if (v < n_items) {
                const unsigned p = ce[u].y, q = ce[u].z;
                ip[u] = p;
                iq[u] = q;
                how[u] = 4;
                // does an item of this trip update the key?
                const int sp_ = find_S(p), sq_ = find_S(q);
                const unsigned rp = sp_ >= 0 ? s_role[sp_] : 0u, rq = sq_ >= 0 ? s_role[sq_] : 0u;
                const unsigned long long t1 = (rq & 5) ? cell_sum(rq >> 3, 2 * (size_t)p) : 0ull;
                const unsigned long long t2 = (rp & 6) ? cell_sum(rp >> 3, 2 * (size_t)q + 1) : 0ull;
                touched[u] = (t1 | t2) != 0;
                hf[u] = P.flag[ce[u].x];
                hc[u] = P.cnt[ce[u].x];
            }
            if (how[u] & 1) {   // the key's home slot: at load <= 1/2 it usually decides
                const size_t s0 = mix64(pair_key(ip[u], iq[u])) & P.mask;
                hk[u] = P.key[s0];
                hc[u] = P.cnt[s0];
                hf[u] = P.flag[s0];
            }
            if (how[u]) {
                kp[u] = K.key8[ip[u]];
                kq[u] = K.key8[iq[u]];
            }
        }
#pragma unroll
        for (unsigned u = 0; u < kBatchApplyItems; ++u) {
            if (how[u] & 1) {
                long long c;
                unsigned f;
                const size_t s = pair_update_from(P, st, ip[u], iq[u], delta[u], (how[u] & 2) != 0, hk[u], hc[u],
                                                  hf[u], &c, &f, n_ins);
                updated(s, ip[u], iq[u], c, f, (how[u] & 2) != 0, kp[u], kq[u]);
            } else if (how[u] & 4) {
                if (!touched[u] && (hf[u] & kPresent)) offer(Cand{hc[u], kp[u], kq[u], ce[u].x, ip[u], iq[u]});
            }
        }
    }
    if (pw0) probe_stamp(st, B.trip, 11);
    best = wave_best(best, K);
    n_ins = wave_sum(n_ins);
    if ((tid & 63) == 0 && n_ins) atomicAdd(&s_ins, n_ins);
    if ((tid & 63) == 0) s_wave[tid >> 6] = best;
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < (int)(kApplyBatchThreads / 64); ++w)
            if (cand_better(s_wave[w], best, K.pool, K.off, K.len)) best = s_wave[w];
        part[blockIdx.x] = Partial{best.cnt, best.ka, best.kb, best.slot, best.a, best.b, 0};
        // the workgroup's list entries and C admissions: one reservation each
        const unsigned nl = s_nl, nc = min(s_nc, kApplyCLds);
        s_lbase = nl ? atomicAdd(&bs->list_n[lpar], nl) : 0u;
        s_cbase = nc ? atomicAdd(&st->nC, nc) : 0u;
        if (s_ins) atomicAdd(&st->pair_used, (unsigned long long)s_ins);   // read by the next select
    }
    if (s_nl | s_nc) {   // (uniform: read after the barrier) only workgroups with entries wait
        __syncthreads();
        const unsigned nl = min(s_nl, kListCap), nc = min(s_nc, kApplyCLds);
        const unsigned lb = s_lbase, cb = s_cbase;
        if ((unsigned)tid < nl && lb + tid < kListCap) list[lb + tid] = s_lst[tid];
        for (unsigned i = tid; i < nc; i += blockDim.x) {
            if (cb + i < st->capC) P.C[cb + i] = s_cadd[i];
            else atomicOr(&st->err, ERR_C_FULL);
        }
    }
    if (pw0) probe_stamp(st, B.trip, 12);
    if (blockIdx.x == gridDim.x - 1 && tid < k && B.m[tid].isnew) {   // the new tokens enter the dedupe map
        const unsigned nw = B.m[tid].nw;
        const unsigned long long h = B.m[tid].hash;
        unsigned s = (unsigned)mix64(h) & K.map_mask;
        while (atomicCAS(&K.map[s], 0ull, map_entry(h, nw)) != 0ull) s = (s + 1) & K.map_mask;
    }
    if (blockIdx.x == 0 && tid == 0) {
        st->nparts = gridDim.x;
        if (!scan_only) {   // finish the trip: k rounds done; the state its select decided from
            st->round = B.round + k;
            st->ntok = B.ntok + (int)B.n_fresh;
            bs->trip = B.trip + 1;
            bs->prev_k = k;
            bs->prev_sparse = sparse;
            st->pool_used = B.pool_after;
            bs->batch_seq = B.batch_id;
            bs->T2 = b_T2;
            st->n_single += st->n_single_new;
            st->n_single_new = 0;
        }
    }
    if (pw0) probe_stamp(st, B.trip, 13);
    if (BPE355_PROBE_CODE && !scan_only && st->probe) {
        __syncthreads();
        if (tid == 0 && (B.trip % kProbeTrip) == 0) {   // workgroups that reserved list / C space
            unsigned long long* pr = st->probe + kProbeSlots * (size_t)(B.trip / kProbeTrip);
            if (s_nl) atomicAdd(&pr[22], 1ull);
            if (s_nc) atomicAdd(&pr[23], 1ull);
        }
        if (tid == 0) probe_done(st, &st->probe_apply_done, B.trip, 15);
    }
}

// ------------------------------------------------------------------ word table build
// Occupied count-table slots -> (offset, len, count) words.  Each workgroup takes
// kCollectPer * 256 slots and reserves its words' positions with ONE global atomic (one per
// wave, 262 K same-address atomics at a 16 M-slot table, serialised into ~6 ms).
constexpr unsigned kCollectThreads = 256;
constexpr unsigned kCollectPer = 8;
__global__ void __launch_bounds__(kCollectThreads) k_collect_words(
    const unsigned long long* __restrict__ kv, const unsigned long long* __restrict__ pos, size_t cap,
    const uint8_t* __restrict__ text, const uint8_t* __restrict__ sp_bytes, const uint32_t* __restrict__ sp_off,
    const uint32_t* __restrict__ sp_len, int n_sp, unsigned long long* __restrict__ w_off,
    uint32_t* __restrict__ w_len, unsigned long long* __restrict__ w_cnt, unsigned* __restrict__ n_words,
    unsigned* __restrict__ max_len) {
    __shared__ unsigned s_n, s_base, s_ml;
    if (threadIdx.x == 0) { s_n = 0; s_ml = 0; }
    const size_t s0 = (size_t)blockIdx.x * kCollectThreads * kCollectPer + threadIdx.x;
    unsigned long long key[kCollectPer];
#pragma unroll
    for (unsigned u = 0; u < kCollectPer; ++u) {   // coalesced: slot s0 + u * 256
        const size_t s = s0 + (size_t)u * kCollectThreads;
        key[u] = s < cap ? kv[2 * s] : 0ULL;
    }
    // {key, count} entries (text.hip): the key's top bit marks a word stored inline (length in
    // bits 56..62, an occurrence in pos[]), else key = len << 40 | offset + 1
    unsigned long long off[kCollectPer];
    unsigned len[kCollectPer];
    unsigned mine = 0, ml = 0, keepm = 0;
#pragma unroll
    for (unsigned u = 0; u < kCollectPer; ++u) {
        const size_t s = s0 + (size_t)u * kCollectThreads;
        const unsigned long long k = key[u];
        bool keep = k != 0;
        const bool inl = (k >> 63) != 0;
        len[u] = inl ? (unsigned)((k >> 56) & 0x7f) : (unsigned)(k >> 40);
        off[u] = inl ? (keep ? pos[s] : 0ULL) : (k & ((1ULL << 40) - 1)) - 1;
        for (int i = 0; keep && i < n_sp; ++i) {  // train.py:25 skips matches equal to a special
            if (sp_len[i] != len[u]) continue;
            bool eq = true;
            for (unsigned j = 0; j < len[u] && eq; ++j) eq = text[off[u] + j] == sp_bytes[sp_off[i] + j];
            if (eq) keep = false;
        }
        keepm |= (unsigned)keep << u;
        mine += keep;
        ml = keep && len[u] > ml ? len[u] : ml;
    }
    __syncthreads();   // s_n, s_ml initialised
    const unsigned at = mine ? atomicAdd(&s_n, mine) : 0u;   // LDS: this thread's first position
    ml = wave_max(ml);
    if ((threadIdx.x & 63) == 0 && ml) atomicMax(&s_ml, ml);
    __syncthreads();
    if (threadIdx.x == 0) {
        s_base = s_n ? atomicAdd(n_words, s_n) : 0u;
        if (s_ml) atomicMax(max_len, s_ml);
    }
    __syncthreads();
    unsigned idx = s_base + at;
#pragma unroll
    for (unsigned u = 0; u < kCollectPer; ++u) {
        if (!((keepm >> u) & 1u)) continue;
        const size_t s = s0 + (size_t)u * kCollectThreads;
        w_off[idx] = off[u]; w_len[idx] = len[u]; w_cnt[idx] = kv[2 * s + 1];
        ++idx;
    }
}

__global__ void k_len_u64(const uint32_t* __restrict__ w_len, unsigned n, unsigned long long* __restrict__ o) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = w_len[i];
}

// words -> a CSR of byte ids (the "long" side table)
template <class TokT>
__global__ void k_fill_words(const uint8_t* __restrict__ text, const unsigned long long* __restrict__ w_off,
                             const uint32_t* __restrict__ w_len, const unsigned long long* __restrict__ beg,
                             unsigned n, TokT* __restrict__ tok) {
    const unsigned w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n) return;
    const unsigned long long bg = beg[w];
    const uint32_t len = w_len[w];
    const uint8_t* src = text + w_off[w];
    for (uint32_t i = 0; i < len; ++i) tok[bg + i] = (TokT)src[i];
}

// the initial pair histogram into kHistReplicas copies, so the hottest pairs do not
// serialize on one address
__global__ void k_hist_words(const unsigned long long* __restrict__ w_off, const uint32_t* __restrict__ w_len,
                             const unsigned long long* __restrict__ w_cnt, const uint8_t* __restrict__ text,
                             unsigned n, unsigned long long* __restrict__ hist) {
    const unsigned w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n) return;
    const uint8_t* src = text + w_off[w];
    const uint32_t len = w_len[w];
    const unsigned long long c = w_cnt[w];
    unsigned long long* h = hist + (size_t)(blockIdx.x % kHistReplicas) * 65536;
    unsigned prev = src[0];
    for (uint32_t i = 1; i < len; ++i) {   // train.py:45-46
        const unsigned cur = src[i];
        atomicAdd(&h[prev * 256 + cur], c);
        prev = cur;
    }
}

__global__ void k_hist_reduce(unsigned long long* __restrict__ hist) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 65536) return;
    unsigned long long s = 0;
    for (int r = 0; r < kHistReplicas; ++r) s += hist[(size_t)r * 65536 + i];
    hist[i] = s;
}

__global__ void k_init_pairs(const unsigned long long* __restrict__ hist, PairsDev P,
                             RoundState* st) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 65536) return;
    const long long c = (long long)hist[i];
    if (c <= 0) return;
    bool ins;
    const size_t s = pair_slot(P, pair_key(i >> 8, i & 255u), st, &ins);
    if (s == ~(size_t)0) return;
    P.cnt[s] = c;
    P.flag[s] = kPresent;
}

__global__ void k_init_tokens(ToksDev K) {
    const unsigned i = threadIdx.x;  // 256 threads
    K.pool[i] = (uint8_t)i;
    K.off[i] = i;
    K.len[i] = 1;
    K.hash[i] = i;
    K.pw[i] = kPolyP;
    K.key8[i] = (unsigned long long)i << 56;
    __syncthreads();
    if (i == 0) {
        for (unsigned t = 0; t < 256; ++t) {
            unsigned s = (unsigned)mix64(t) & K.map_mask;   // a byte token's hash is its byte
            while (K.map[s] != 0) s = (s + 1) & K.map_mask;
            K.map[s] = map_entry(t, t);
        }
    }
}

// ------------------------------------------------------------------ compaction
// flat word index -> (class, index); class kNumCls = long table
template <class TokT>
__device__ __forceinline__ void word_at(const WordsDev<TokT>& W, unsigned g, int* c, unsigned* i) {
    unsigned acc = 0;
    for (int k = 0; k < kNumCls; ++k) {
        if (g < acc + W.c[k].n) { *c = k; *i = g - acc; return; }
        acc += W.c[k].n;
    }
    *c = kNumCls;
    *i = g - acc;
}

template <class TokT>
__device__ __forceinline__ uint32_t word_len(const WordsDev<TokT>& W, int c, unsigned i) {
    return c < kNumCls ? (uint32_t)W.c[c].slot[(size_t)i * slot_w(c)] : W.llen[i];
}

struct MoveCounts {
    unsigned n[kNumCls + 1];
    unsigned fill[kNumCls + 1];
    unsigned long long long_tokens, long_fill;
};

// Compaction in three launches, with no same-address atomics on the hot path: every workgroup
// owns a contiguous range of words; k_move_count writes its per-class counts, k_move_scan turns
// them into per-workgroup bases (one workgroup), k_move places each word at base + running
// offset + rank in its chunk.  Words keep their relative order within a class.
constexpr unsigned kMoveBlocks = 1024;
constexpr int kMoveK = kNumCls + 1;   // destination classes: the slot classes and "long"

__device__ __forceinline__ unsigned move_per_block(unsigned total) { return (total + kMoveBlocks - 1) / kMoveBlocks; }

template <class TokT>
__device__ __forceinline__ int move_class(const WordsDev<TokT>& W, unsigned g, unsigned total, int* c, unsigned* i,
                                          uint32_t* len) {
    int d = -1;
    *len = 0;
    if (g < total) {
        word_at(W, g, c, i);
        *len = word_len(W, *c, *i);
        if (*len >= 2) d = class_for(*len);
    }
    return d;
}

template <class TokT>
__global__ void __launch_bounds__(256) k_move_count(WordsDev<TokT> W, unsigned total, unsigned* __restrict__ blk_cnt,
                                                    MoveCounts* mc) {
    __shared__ unsigned s_c[4][kMoveK];
    const unsigned per = move_per_block(total);
    const unsigned beg = blockIdx.x * per, end = min(total, beg + per);
    unsigned cnt[kMoveK] = {};
    unsigned long long lt = 0;
    for (unsigned g = beg + threadIdx.x; g < end; g += blockDim.x) {
        int c;
        unsigned i;
        uint32_t len;
        const int d = move_class(W, g, total, &c, &i, &len);
#pragma unroll
        for (int k = 0; k < kMoveK; ++k) cnt[k] += d == k;
        if (d == kNumCls) lt += len;
    }
    const int wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kMoveK; ++k) {
        const unsigned v = (unsigned)wave_sum((unsigned long long)cnt[k]);
        if ((threadIdx.x & 63) == 0) s_c[wv][k] = v;
    }
    lt = wave_sum(lt);
    if ((threadIdx.x & 63) == 0 && lt) atomicAdd(&mc->long_tokens, lt);
    __syncthreads();
    if (threadIdx.x < kMoveK)
        blk_cnt[blockIdx.x * kMoveK + threadIdx.x] =
            s_c[0][threadIdx.x] + s_c[1][threadIdx.x] + s_c[2][threadIdx.x] + s_c[3][threadIdx.x];
}

// one workgroup of kMoveBlocks threads: exclusive scan of every class's per-block counts
__global__ void __launch_bounds__(kMoveBlocks) k_move_scan(unsigned* __restrict__ blk_cnt, MoveCounts* mc) {
    __shared__ unsigned s_w[kMoveBlocks / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int k = 0; k < kMoveK; ++k) {
        const unsigned v = blk_cnt[t * kMoveK + k];
        unsigned x = v;   // inclusive scan in the wave
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_w[wv] = x;
        __syncthreads();
        unsigned base = 0;
        for (int w = 0; w < wv; ++w) base += s_w[w];
        blk_cnt[t * kMoveK + k] = base + x - v;   // exclusive
        if (t == kMoveBlocks - 1) mc->n[k] = base + x;
        __syncthreads();
    }
}

template <class TokT>
__global__ void __launch_bounds__(256) k_move(WordsDev<TokT> W, unsigned total, WordsDev<TokT> D,
                                              const unsigned* __restrict__ blk_off, MoveCounts* mc) {
    __shared__ unsigned s_run[kMoveK];        // words of each class placed by earlier chunks
    __shared__ unsigned s_wc[4][kMoveK];      // this chunk: per-wave counts
    const unsigned per = move_per_block(total);
    const unsigned beg = blockIdx.x * per, end = min(total, beg + per);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x < kMoveK) s_run[threadIdx.x] = blk_off[blockIdx.x * kMoveK + threadIdx.x];
    for (unsigned g0 = beg; g0 < end; g0 += blockDim.x) {
        const unsigned g = g0 + threadIdx.x;
        int c = 0;
        unsigned i = 0;
        uint32_t len = 0;
        const int d = g < end ? move_class(W, g, total, &c, &i, &len) : -1;
        unsigned rank = 0;
#pragma unroll
        for (int k = 0; k < kMoveK; ++k) {
            const unsigned long long m = __ballot(d == k);
            if (d == k) rank = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            if (lane == 0) s_wc[wv][k] = (unsigned)__popcll(m);
        }
        __syncthreads();   // s_run from the previous chunk, s_wc of this one
        unsigned j = ~0u;
        if (d >= 0) {
            unsigned below = 0;
            for (int w = 0; w < wv; ++w) below += s_wc[w][d];
            j = s_run[d] + below + rank;
        }
        __syncthreads();
        if (threadIdx.x < kMoveK)
            s_run[threadIdx.x] += s_wc[0][threadIdx.x] + s_wc[1][threadIdx.x] + s_wc[2][threadIdx.x] + s_wc[3][threadIdx.x];
        if (d < 0) continue;
        const TokT* src = c < kNumCls ? W.c[c].slot + (size_t)i * slot_w(c) + 1 : W.ltok + W.lbeg[i];
        const unsigned long long cnt = c < kNumCls ? W.c[c].cnt[i] : W.lcnt[i];
        if (d < kNumCls) {
            TokT* dst = D.c[d].slot + (size_t)j * slot_w(d);
            dst[0] = (TokT)len;
            for (uint32_t k = 0; k < len; ++k) dst[1 + k] = src[k];
            for (int k = (int)len + 1; k < slot_w(d); ++k) dst[k] = sentinel<TokT>();
            D.c[d].cnt[j] = cnt;
        } else {
            const unsigned long long bg = atomicAdd(&mc->long_fill, (unsigned long long)len);
            for (uint32_t k = 0; k < len; ++k) D.ltok[bg + k] = src[k];
            D.lbeg[j] = bg;
            D.llen[j] = len;
            D.lcnt[j] = cnt;
        }
    }
}

// ------------------------------------------------------------------ posting index build
template <class TokT>
__device__ __forceinline__ const TokT* slot_of(const WordsDev<TokT>& W, unsigned f, uint32_t* len) {
    int c = 0;
    while (c + 1 < kNumCls && f >= W.off[c + 1]) ++c;
    const TokT* s = W.c[c].slot + (size_t)(f - W.off[c]) * slot_w(c);
    *len = s[0];
    return s + 1;
}

template <class TokT>
__global__ void k_index_count(WordsDev<TokT> W, unsigned n, uint32_t* __restrict__ cnt) {
    const unsigned f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n) return;
    uint32_t len;
    const TokT* t = slot_of(W, f, &len);
    uint32_t d = 0;
    if (len >= 2)
        for (uint32_t k = 0; k < len; ++k) {
            bool first = true;
            for (uint32_t q = 0; q < k && first; ++q) first = t[q] != t[k];
            d += first;
        }
    cnt[f] = d;
}

template <class TokT>
__global__ void k_index_emit(WordsDev<TokT> W, unsigned n, const uint32_t* __restrict__ pos,
                             uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const unsigned f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n) return;
    uint32_t len;
    const TokT* t = slot_of(W, f, &len);
    if (len < 2) return;
    uint32_t o = pos[f];
    for (uint32_t k = 0; k < len; ++k) {
        bool first = true;
        for (uint32_t q = 0; q < k && first; ++q) first = t[q] != t[k];
        if (first) { keys[o] = t[k]; vals[o] = f; ++o; }
    }
}

// The same two passes per slot class, the slot in registers (one 16-byte load per 16 bytes of
// slot, every index a compile-time constant): the first occurrence of each token of a word is a
// register compare, not a dependent load per pair (k_index_count / k_index_emit load element by
// element; kept for reference and the A/B)
template <class TokT, int C, bool kEmit>
__global__ void __launch_bounds__(256) k_index_cls(WordsDev<TokT> W, const uint32_t* __restrict__ pos,
                                                   uint32_t* __restrict__ cnt, uint32_t* __restrict__ keys,
                                                   uint32_t* __restrict__ vals) {
    constexpr int Wd = slot_w(C);
    constexpr int V = Wd * (int)sizeof(TokT) / 16;
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= W.c[C].n) return;
    const unsigned f = W.off[C] + i;
    uint4 r[V];
#pragma unroll
    for (int v = 0; v < V; ++v) r[v] = reinterpret_cast<const uint4*>(W.c[C].slot + (size_t)i * Wd)[v];
    TokT e[Wd];
    __builtin_memcpy(e, r, sizeof(e));
    const uint32_t len = e[0];
    uint32_t o = kEmit ? pos[f] : 0u, d = 0;
    if (len >= 2) {
#pragma unroll
        for (int k = 1; k < Wd; ++k) {   // no early exit: a constant trip count keeps e[] in registers
            bool first = (uint32_t)k <= len;
#pragma unroll
            for (int q = 1; q < k; ++q) first &= e[q] != e[k];
            if (first) {
                if (kEmit) { keys[o] = e[k]; vals[o] = f; ++o; }
                else ++d;
            }
        }
    }
    if (!kEmit) cnt[f] = d;
}

template <class TokT, bool kEmit>
void index_pass(const WordsDev<TokT>& W, const uint32_t* pos, uint32_t* cnt, uint32_t* keys, uint32_t* vals,
                hipStream_t s) {
    if (W.c[0].n) hipLaunchKernelGGL((k_index_cls<TokT, 0, kEmit>), dim3(ceil_div(W.c[0].n, 256u)), dim3(256), 0, s, W, pos, cnt, keys, vals);
    if (W.c[1].n) hipLaunchKernelGGL((k_index_cls<TokT, 1, kEmit>), dim3(ceil_div(W.c[1].n, 256u)), dim3(256), 0, s, W, pos, cnt, keys, vals);
    if (W.c[2].n) hipLaunchKernelGGL((k_index_cls<TokT, 2, kEmit>), dim3(ceil_div(W.c[2].n, 256u)), dim3(256), 0, s, W, pos, cnt, keys, vals);
    if (W.c[3].n) hipLaunchKernelGGL((k_index_cls<TokT, 3, kEmit>), dim3(ceil_div(W.c[3].n, 256u)), dim3(256), 0, s, W, pos, cnt, keys, vals);
}
#ifndef BPE355_INDEX_REGS
#define BPE355_INDEX_REGS 1
#endif

__global__ void k_index_bounds(const uint32_t* __restrict__ keys, unsigned long long e,
                               uint32_t* __restrict__ beg, uint32_t* __restrict__ len) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e) return;
    const uint32_t k = keys[i];
    if (i == 0 || keys[i - 1] != k) beg[k] = (uint32_t)i;
    if (i + 1 == e || keys[i + 1] != k) len[k] = (uint32_t)(i + 1);   // end; beg subtracted below
}

__global__ void k_index_lens(const uint32_t* __restrict__ beg, uint32_t* __restrict__ len, unsigned ntok) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ntok && len[t]) len[t] -= beg[t];
}


// ------------------------------------------------------------------ rebuild helpers
struct RebuildStats {
    unsigned long long bins[64];
    unsigned long long ghosts;
    unsigned long long sub[1024];
};

__global__ void k_rebuild_hist(PairsDev P, size_t cap, RebuildStats* rs) {
    __shared__ unsigned long long sh[64];
    if (threadIdx.x < 64) sh[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long ghosts = 0;
    for (size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap;
         s += (size_t)gridDim.x * blockDim.x) {
        if (!(P.flag[s] & kPresent)) continue;
        const long long c = P.cnt[s];
        if (c <= 0) { ghosts += (c == 0); continue; }
        atomicAdd(&sh[63 - __clzll((unsigned long long)c)], 1ULL);
    }
    ghosts = wave_sum(ghosts);
    if ((threadIdx.x & 63) == 0 && ghosts) atomicAdd(&rs->ghosts, ghosts);
    __syncthreads();
    if (threadIdx.x < 64 && sh[threadIdx.x]) atomicAdd(&rs->bins[threadIdx.x], sh[threadIdx.x]);
}

__global__ void k_rebuild_sub(PairsDev P, size_t cap, long long lo, long long hi, long long width,
                              RebuildStats* rs) {
    __shared__ unsigned sh[1024];
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) sh[k] = 0;
    __syncthreads();
    for (size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap;
         s += (size_t)gridDim.x * blockDim.x) {
        if (!(P.flag[s] & kPresent)) continue;
        const long long c = P.cnt[s];
        if (c < lo || c >= hi) continue;
        atomicAdd(&sh[(c - lo) / width], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 1024; k += blockDim.x)
        if (sh[k]) atomicAdd(&rs->sub[k], (unsigned long long)sh[k]);
}

__global__ void k_build_C(PairsDev P, size_t cap, long long T, RoundState* st) {
    for (size_t s0 = (size_t)blockIdx.x * blockDim.x; s0 < cap; s0 += (size_t)gridDim.x * blockDim.x) {
        const size_t s = s0 + threadIdx.x;
        const unsigned f = s < cap ? P.flag[s] : 0u;
        const bool in = (f & kPresent) && P.cnt[s] >= T;
        const unsigned idx = wave_append(in, &st->nC);
        if (in) {
            const unsigned long long key = P.key[s] - 1ULL;
            if (idx < st->capC) P.C[idx] = make_uint4((unsigned)s, (unsigned)(key >> 32), (unsigned)key, 0u);
            else atomicOr(&st->err, ERR_C_FULL);
            if (!(f & kInC)) P.flag[s] = f | kInC;
        } else if (f & kInC) {
            P.flag[s] = f & ~kInC;
        }
    }
}

__global__ void k_collect_present(PairsDev P, size_t cap, unsigned long long* out,
                                  unsigned* n_out) {
    for (size_t s0 = (size_t)blockIdx.x * blockDim.x; s0 < cap; s0 += (size_t)gridDim.x * blockDim.x) {
        const size_t s = s0 + threadIdx.x;
        const bool in = s < cap && (P.flag[s] & kPresent);
        const unsigned idx = wave_append(in, n_out);
        if (in) out[idx] = P.key[s] - 1ULL;
    }
}

__global__ void k_rehash(const unsigned long long* __restrict__ okey, const long long* __restrict__ ocnt,
                         const unsigned* __restrict__ oflag, size_t ocap, PairsDev P, RoundState* st) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ocap) return;
    const unsigned long long k = okey[i];
    if (!k) return;
    bool ins;
    const size_t s = pair_slot(P, k, st, &ins);
    if (s == ~(size_t)0) return;
    P.cnt[s] = ocnt[i];
    P.flag[s] = oflag[i] & kPresent;
}

// ------------------------------------------------------------------ host driver
double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

template <class TokT>
struct HostWords {   // owns the device arrays behind a WordsDev
    DevBuf<TokT> slot[kNumCls];
    DevBuf<unsigned long long> cnt[kNumCls];
    unsigned n[kNumCls] = {0, 0, 0, 0};
    DevBuf<TokT> ltok;
    DevBuf<unsigned long long> lbeg, lcnt;
    DevBuf<uint32_t> llen;
    unsigned ln = 0;
    unsigned total() const { return n[0] + n[1] + n[2] + n[3] + ln; }
    WordsDev<TokT> dev() const {
        WordsDev<TokT> W{};
        for (int c = 0; c < kNumCls; ++c) W.c[c] = SlotCls<TokT>{slot[c].p, cnt[c].p, n[c], 0, 0, 0};
        W.ltok = ltok.p; W.lbeg = lbeg.p; W.llen = llen.p; W.lcnt = lcnt.p; W.ln = ln;
        return W;
    }
};

template <class TokT>
class MergeLoop {
   public:
    MergeLoop(hipStream_t stream, Comm* comm, const uint8_t* text, int n_rounds, TrainOutput& out)
        : s_(stream), comm_(comm), text_(text), n_rounds_(n_rounds), out_(out) {}
    ~MergeLoop() {
        if (snap_st_) (void)hipHostFree(snap_st_);
        if (snap_ti_) (void)hipHostFree(snap_ti_);
        for (auto e : blk_ev_)
            if (e) (void)hipEventDestroy(e);
    }
    MergeLoop(const MergeLoop&) = delete;
    MergeLoop& operator=(const MergeLoop&) = delete;

    void build_words(const WordCounts& wc, const std::vector<std::string>& specials);
    void run();

   private:
    static constexpr int kBatch = 64;
    static constexpr int kTrips = 32;   // batched mode: at most this many [select][merge][apply] per block
    int trips_ = 8;                     // trips per block (BPE355_TRIPS): a halt leaves at most ~1.5
                                        // blocks of empty trips queued behind it
    static_assert(2 * kTrips <= kBatch, "two blocks' timing events fit the event pool");
    static constexpr int kArgBlocks = 64;
    static constexpr unsigned kCScanBlocks = 64;   // k_apply_argmax workgroups scanning C
    unsigned nparts_ = 0;                          // argmax partials the next k_merge reduces
    static constexpr int kTimingStride = 8;   // k_merge launches timed: one in 8
    static constexpr unsigned long long kTarget = 4096;
    // batched mode: the pair table grows past load 1 / kPairLoadDiv (an insert is an unsuccessful
    // linear-probe search: ~2.5 dependent probes at load 1/2, ~1.4 at 1/4)
    static constexpr size_t kPairLoadDiv = 2;   // 4 measured: no gain (366 vs 364 ms)

    void alloc_pairs(size_t cap);
    void grow_pairs();
    void ensure_pool(unsigned need);
    void push_state() { BPE_HIP(hipMemcpyAsync(st_.p, &hs_, sizeof(hs_), hipMemcpyHostToDevice, s_)); }
    void pull_state() {
        BPE_HIP(hipMemcpyAsync(&hs_, st_.p, sizeof(hs_), hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipStreamSynchronize(s_));
    }
    int rebuild();  // 0 ok, 1 exhausted (only zero-count keys), 2 empty
    void exhaustion();
    void compact();
    void layout_blocks();
    void build_index();
    PairsDev pairs() const { return PairsDev{pkey_.p, pcnt_.p, pflag_.p, pcap_ - 1, C_.p}; }
    ToksDev toks() const {
        return ToksDev{pool_.p, toff_.p, tlen_.p, thash_.p, tpw_.p, tkey8_.p, tmap_.p,
                       (uint32_t)(tmap_.n - 1)};
    }

    hipStream_t s_;
    Comm* comm_;
    // the sharded exchange runs when there are several ranks; BPE355_FORCE_COMM=1 runs it on a
    // 1-rank communicator too (tests the RCCL calls on a single-GPU box)
    bool sharded() const {
        static const bool force = std::getenv("BPE355_FORCE_COMM") != nullptr;
        return comm_ && (comm_->nranks > 1 || force);
    }
    const uint8_t* text_;
    int n_rounds_;
    TrainOutput& out_;

    RoundState hs_{};
    DevBuf<RoundState> st_;
    // words
    unsigned n_words_ = 0, max_len_ = 0;
    HostWords<TokT> words_;
    WordsDev<TokT> wdev_{};
    WordsDev<TokT> wdev_trip_{};    // the slot classes over k_trip's workgroups
    unsigned trip_grid_ = 1;
    unsigned merge_grid_ = 1;
    unsigned merge_grid_cur_ = 0;   // k_merge_batch blocks for the next block of trips (0: merge_grid_)
    double scan_bytes_ = 0, long_bytes_ = 0;
    unsigned long long long_tokens_ = 0;
    unsigned n_live_ = 0;
    DevBuf<unsigned long long> hist_;
    // pairs
    size_t pcap_ = 0;
    DevBuf<unsigned long long> pkey_;
    DevBuf<long long> pcnt_;
    DevBuf<unsigned> pflag_;
    DevBuf<uint4> C_;
    // tokens
    unsigned tok_cap_ = 0;
    size_t lr_member_ = 0;        // cells per member: 2 x tok_cap_, rounded up to whole 64-cell blocks
    DevBuf<unsigned> tb_, tbc_;   // touched-block bitmaps (CellMarks)
    CellMarks cm_{};
    DevBuf<uint8_t> pool_;
    DevBuf<uint32_t> toff_, tlen_;
    DevBuf<unsigned long long> tmap_;
    DevBuf<unsigned long long> thash_, tpw_, tkey8_;
    DevBuf<unsigned long long> LR_;
    DevBuf<Partial> part_;
    DevBuf<uint32_t> m_a_, m_b_, m_new_, m_mode_;
    // batched rounds (single rank): several exact merges per trip (k_select)
    bool batched_ = false;
    bool fused_ = false;         // k_trip (BPE355_FOLD=1), else k_select + k_merge_batch
    int max_batch_ = kMaxBatch;
    long long trips_launched_ = 0, trips_run_ = 0, rounds_batched_ = 0;
    std::unique_ptr<std::vector<int>> trip_log_;   // analysis knob BPE355_TRIP_LOG=path: every trip's record
    DevBuf<BatchState> bs_;
    DevBuf<Batch> batch_;
    DevBuf<unsigned long long> dbg_, sig_;   // BPE355_CHECK_MARKS
    DevBuf<uint32_t> tags_;      // per slot word: the last batch that claimed it
    DevBuf<int> trip_info_;      // per trip of a block: first round, members, scan mode, list entries (2 slots)
    RoundState* snap_st_ = nullptr;   // pinned: the state at the end of each in-flight block
    int* snap_ti_ = nullptr;          // pinned: each block's trip_info
    RoundState* snap_st_dev_ = nullptr;   // (their device-side addresses)
    int* snap_ti_dev_ = nullptr;
    hipEvent_t blk_ev_[2] = {nullptr, nullptr};
    long long slot_base_[2] = {0, 0};   // trips launched before each slot's block
    void launch_block(int slot, bool timing, std::vector<hipEvent_t>& ev);
    unsigned merge_grid() const;
    void finish_block(int slot, bool timing, std::vector<hipEvent_t>& ev, double& k1_ms, double& k1_bytes,
                      long long& k1_launches);
    DevBuf<unsigned long long> probe_;   // BPE355_PROBE stamps
    void report_probe();
    DevBuf<Partial> list_;       // the candidate list (every present key >= T2)
    static constexpr unsigned kApplyBatchBlocks = kApplyGrid;
    void reset_tags();

    DevBuf<long long> m_cnt_;   // BPE355_ROUND_LOG: each round's winning count (else unallocated)
    DevBuf<RebuildStats> rs_;
    // posting index
    DevBuf<uint32_t> ilist_, ibeg_, ilen_;
    DevBuf<uint32_t> ix_cnt_, ix_pos_, ix_keys_, ix_vals_, ix_keys2_;   // its build's scratch
    DevBuf<uint8_t> ix_tmp_;
    HostWords<TokT> spare_;   // the word table's other buffer set (compaction writes into it)
    unsigned cls_cap_[kNumCls] = {};   // words each slot class can ever hold (set by the first compaction)
    bool cls_cap_set_ = false;
    DevBuf<MoveCounts> move_counts_;
    DevBuf<unsigned> move_blk_;
    IndexDev idev_{};
    int next_index_round_ = 256;
};

template <class TokT>
void MergeLoop<TokT>::build_words(const WordCounts& wc, const std::vector<std::string>& specials) {
    // specials -> device (compared once per unique word, not per occurrence)
    std::string spb;
    std::vector<uint32_t> spo, spl;
    for (const auto& s : specials) { spo.push_back((uint32_t)spb.size()); spl.push_back((uint32_t)s.size()); spb += s; }
    DevBuf<uint8_t> d_spb(std::max<size_t>(spb.size(), 1));
    DevBuf<uint32_t> d_spo(std::max<size_t>(spo.size(), 1)), d_spl(std::max<size_t>(spl.size(), 1));
    if (!spb.empty()) BPE_HIP(hipMemcpyAsync(d_spb.p, spb.data(), spb.size(), hipMemcpyHostToDevice, s_));
    if (!spo.empty()) {
        BPE_HIP(hipMemcpyAsync(d_spo.p, spo.data(), spo.size() * 4, hipMemcpyHostToDevice, s_));
        BPE_HIP(hipMemcpyAsync(d_spl.p, spl.data(), spl.size() * 4, hipMemcpyHostToDevice, s_));
    }
    // occupied count-table slots -> (offset, len, count) records
    DevBuf<unsigned> cnts(2);
    BPE_HIP(hipMemsetAsync(cnts.p, 0, 8, s_));
    DevBuf<unsigned long long> w_off(wc.cap), w_cnt(wc.cap);
    DevBuf<uint32_t> w_len(wc.cap);
    hipLaunchKernelGGL(k_collect_words, dim3(ceil_div(wc.cap, (size_t)kCollectThreads * kCollectPer)),
                       dim3(kCollectThreads), 0, s_, wc.kv.p,
                       wc.pos.p, wc.cap, text_, d_spb.p, d_spo.p, d_spl.p, (int)specials.size(),
                       w_off.p, w_len.p, w_cnt.p, cnts.p, cnts.p + 1);
    BPE_HIP(hipGetLastError());
    unsigned h2[2];
    BPE_HIP(hipMemcpyAsync(h2, cnts.p, 8, hipMemcpyDeviceToHost, s_));
    BPE_HIP(hipStreamSynchronize(s_));
    n_words_ = h2[0];
    max_len_ = h2[1];
    const unsigned n = n_words_;
    hist_.alloc((size_t)kHistReplicas * 65536);
    BPE_HIP(hipMemsetAsync(hist_.p, 0, hist_.bytes(), s_));
    // all words start in the CSR side table; compact() then sorts them into slot classes
    HostWords<TokT>& H = words_;
    unsigned long long total_tok = 0;
    H.ln = n;
    H.llen.alloc(std::max(n, 1u));
    H.lbeg.alloc(std::max(n, 1u));
    H.lcnt.alloc(std::max(n, 1u));
    if (n) {
        DevBuf<unsigned long long> len64(n);
        hipLaunchKernelGGL(k_len_u64, dim3(ceil_div(n, 256)), dim3(256), 0, s_, w_len.p, n, len64.p);
        exclusive_sum(len64.p, H.lbeg.p, n, s_);
        unsigned long long last[2];
        BPE_HIP(hipMemcpyAsync(&last[0], H.lbeg.p + n - 1, 8, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipMemcpyAsync(&last[1], len64.p + n - 1, 8, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipStreamSynchronize(s_));
        total_tok = last[0] + last[1];
    }
    H.ltok.alloc(std::max<unsigned long long>(total_tok, 1));
    if (n) {
        BPE_HIP(hipMemcpyAsync(H.llen.p, w_len.p, n * 4ull, hipMemcpyDeviceToDevice, s_));
        BPE_HIP(hipMemcpyAsync(H.lcnt.p, w_cnt.p, n * 8ull, hipMemcpyDeviceToDevice, s_));
        hipLaunchKernelGGL(k_fill_words<TokT>, dim3(ceil_div(n, 256)), dim3(256), 0, s_, text_, w_off.p,
                           w_len.p, H.lbeg.p, n, H.ltok.p);
        hipLaunchKernelGGL(k_hist_words, dim3(ceil_div(n, 256)), dim3(256), 0, s_, w_off.p,
                           w_len.p, w_cnt.p, text_, n, hist_.p);
        BPE_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_hist_reduce, dim3(256), dim3(256), 0, s_, hist_.p);
    out_.stats.n_words = n;
    out_.stats.n_word_tokens = (int64_t)total_tok;
    BPE_HIP(hipStreamSynchronize(s_));
    n_live_ = n;
    compact();
}

// Rewrite the word table: drop words of one id, move every word to the narrowest slot class.
template <class TokT>
void MergeLoop<TokT>::compact() {
    HostWords<TokT>& H = words_;
    const unsigned total = H.total();
    DevBuf<MoveCounts>& mc = move_counts_;
    DevBuf<unsigned>& blk = move_blk_;
    mc.reserve(1);
    blk.reserve((size_t)kMoveBlocks * kMoveK);
    BPE_HIP(hipMemsetAsync(mc.p, 0, sizeof(MoveCounts), s_));
    const WordsDev<TokT> src = H.dev();
    if (total) {
        hipLaunchKernelGGL(k_move_count<TokT>, dim3(kMoveBlocks), dim3(256), 0, s_, src, total, blk.p, mc.p);
        hipLaunchKernelGGL(k_move_scan, dim3(1), dim3(kMoveBlocks), 0, s_, blk.p, mc.p);
    }
    MoveCounts h{};
    BPE_HIP(hipMemcpyAsync(&h, mc.p, sizeof(h), hipMemcpyDeviceToHost, s_));
    BPE_HIP(hipStreamSynchronize(s_));
    // the new table goes into the previous compaction's arrays (grow-only: the table shrinks as
    // words finish, so after the first compactions nothing is allocated or freed here)
    HostWords<TokT> D = std::move(spare_);
    // capacities: a word only ever moves to a narrower class, so class c never holds more words
    // than the first compaction put in classes >= c or in the long-word table -- sized once, the
    // arrays are never reallocated (a reallocation's free synchronised the device and cost up to
    // ~1 ms per halt; r06j: compact+index 12.1 -> 9.6 ms, merge phase 182.1 -> 179.7-180.0 ms)
    if (!cls_cap_set_) {
        unsigned ge = h.n[kNumCls];   // (long words shrink into the slot classes too)
        for (int c = kNumCls - 1; c >= 0; --c) cls_cap_[c] = ge += h.n[c];
        cls_cap_set_ = true;
    }
    for (int c = 0; c < kNumCls; ++c) {
        D.n[c] = h.n[c];
        const size_t cap = std::max(cls_cap_[c], h.n[c]);
        D.slot[c].reserve(std::max<size_t>(cap * slot_w(c), 1));
        D.cnt[c].reserve(std::max<size_t>(cap, 1));
    }
    D.ln = h.n[kNumCls];
    D.ltok.reserve(std::max<unsigned long long>(h.long_tokens, 1));
    D.lbeg.reserve(std::max(D.ln, 1u));
    D.llen.reserve(std::max(D.ln, 1u));
    D.lcnt.reserve(std::max(D.ln, 1u));
    if (total)
        hipLaunchKernelGGL(k_move<TokT>, dim3(kMoveBlocks), dim3(256), 0, s_, src, total, D.dev(), blk.p, mc.p);
    BPE_HIP(hipGetLastError());
    BPE_HIP(hipStreamSynchronize(s_));
    spare_ = std::move(words_);
    words_ = std::move(D);
    long_tokens_ = h.long_tokens;
    n_live_ = words_.total();
    hs_.n_single = 0;
    layout_blocks();
}

// Posting lists token -> words over the current slot table (long words are always scanned).
template <class TokT>
void MergeLoop<TokT>::build_index() {
    const unsigned n = wdev_.off[kNumCls];
    const unsigned tcap = 256u + (unsigned)n_rounds_ + 1u;
    if (!ibeg_.p) {
        ibeg_.alloc(tcap);
        ilen_.alloc(tcap);
    }
    BPE_HIP(hipMemsetAsync(ibeg_.p, 0, ibeg_.bytes(), s_));
    BPE_HIP(hipMemsetAsync(ilen_.p, 0, ilen_.bytes(), s_));
    unsigned long long E = 0;
    // scratch kept across builds (grow-only; the first build is the largest)
    DevBuf<uint32_t>&cnt = ix_cnt_, &pos = ix_pos_, &keys = ix_keys_, &vals = ix_vals_, &keys2 = ix_keys2_;
    DevBuf<uint8_t>& tmp = ix_tmp_;
    cnt.reserve(std::max(n, 1u));
    pos.reserve(std::max(n, 1u));
    if (n) {
        if (BPE355_INDEX_REGS) index_pass<TokT, false>(wdev_, nullptr, cnt.p, nullptr, nullptr, s_);
        else hipLaunchKernelGGL(k_index_count<TokT>, dim3(ceil_div(n, 256)), dim3(256), 0, s_, wdev_, n, cnt.p);
        exclusive_sum(cnt.p, pos.p, n, s_, &tmp);
        uint32_t last[2];
        BPE_HIP(hipMemcpyAsync(&last[0], pos.p + n - 1, 4, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipMemcpyAsync(&last[1], cnt.p + n - 1, 4, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipStreamSynchronize(s_));
        E = (unsigned long long)last[0] + last[1];
    }
    keys.reserve(std::max<unsigned long long>(E, 1));
    vals.reserve(std::max<unsigned long long>(E, 1));
    keys2.reserve(std::max<unsigned long long>(E, 1));
    ilist_.reserve(std::max<unsigned long long>(E, 1));
    if (E) {
        if (BPE355_INDEX_REGS) index_pass<TokT, true>(wdev_, pos.p, nullptr, keys.p, vals.p, s_);
        else hipLaunchKernelGGL(k_index_emit<TokT>, dim3(ceil_div(n, 256)), dim3(256), 0, s_, wdev_, n, pos.p,
                                keys.p, vals.p);
        int bits = 1;
        while ((1u << bits) < tcap) ++bits;
        radix_sort_pairs(keys.p, keys2.p, vals.p, ilist_.p, E, (unsigned)bits, s_, &tmp);
        hipLaunchKernelGGL(k_index_bounds, dim3(ceil_div(E, 256)), dim3(256), 0, s_, keys2.p, E,
                           ibeg_.p, ilen_.p);
        hipLaunchKernelGGL(k_index_lens, dim3(ceil_div(tcap, 256)), dim3(256), 0, s_, ibeg_.p, ilen_.p, tcap);
    }
    BPE_HIP(hipGetLastError());
    BPE_HIP(hipStreamSynchronize(s_));
    static const unsigned full_div = [] {
        const char* e = std::getenv("BPE355_FULL_DIV");   // experiment knob: scan when lists > n / div
        // n / 4 (r03 sweep, profiles/r03/m_full_div_sweep.txt: 2-4 give 258-264 ms of merges,
        // 6 264-268, 9 275, 14 299)
        return e ? (unsigned)std::max(1, std::atoi(e)) : 4u;
    }();
    idev_ = IndexDev{ilist_.p, ibeg_.p, ilen_.p, n / full_div, n};
    out_.stats.n_index_builds++;
}

// blocks of k_merge per slot class: enough waves to cover each class with a few words per
// thread in flight, block-uniform class so the scan has no per-lane class branch
template <class TokT>
void MergeLoop<TokT>::layout_blocks() {
    WordsDev<TokT> W = words_.dev();
    W.off[0] = 0;
    for (int c = 0; c < kNumCls; ++c) W.off[c + 1] = W.off[c] + W.c[c].n;
    // about one resident generation of workgroups (4 per CU): each block's prologue is a
    // chain of dependent loads, so a second generation would pay it again
    static const unsigned kGridBudget = [] {
        const char* e = std::getenv("BPE355_GRID");   // experiment knob
        return e ? (unsigned)std::max(16, std::atoi(e)) : 1024u;
    }();
    double total_b = 0;
    for (int c = 0; c < kNumCls; ++c) total_b += (double)W.c[c].n * slot_w(c);
    unsigned blk = 0;
    for (int c = 0; c < kNumCls; ++c) {
        const unsigned per_thread = c == 0 ? 4 : (c == 1 ? 2 : 1);
        const unsigned need = ceil_div(W.c[c].n, 256u * per_thread);
        const unsigned share = total_b > 0 ? (unsigned)(kGridBudget * (W.c[c].n * (double)slot_w(c)) / total_b) : 0;
        W.c[c].blk0 = blk;
        W.c[c].nblk = W.c[c].n ? std::max(1u, std::min(need, share)) : 0;
        blk += W.c[c].nblk;
    }
    W.lblk0 = blk;
    W.lnblk = std::min(ceil_div(W.ln, 256u), 64u);
    blk += W.lnblk;
    merge_grid_ = std::max(blk, (unsigned)kMaxBatch);   // k_merge_batch: block j registers member j
    wdev_ = W;
    {   // k_trip's layout: the same classes over kTripThreads-thread workgroups
        constexpr unsigned r = kTripThreads / 256;
        WordsDev<TokT> Wb = W;
        unsigned bb = 0;
        for (int c = 0; c < kNumCls; ++c) {
            Wb.c[c].blk0 = bb;
            Wb.c[c].nblk = W.c[c].n ? std::max(1u, ceil_div(W.c[c].nblk, r)) : 0;
            bb += Wb.c[c].nblk;
        }
        Wb.lblk0 = bb;
        Wb.lnblk = std::min(ceil_div(W.ln, kTripThreads), 64u / r);
        bb += Wb.lnblk;
        trip_grid_ = std::max(bb, (unsigned)kMaxBatch);
        wdev_trip_ = Wb;
    }
    if (std::getenv("BPE355_TRACE"))
        std::fprintf(stderr, "[bpe355] words per slot class: %u %u %u %u, long %u (%llu ids); merge grid %u\n", W.c[0].n,
                     W.c[1].n, W.c[2].n, W.c[3].n, W.ln, (unsigned long long)long_tokens_, merge_grid_);
    // algorithmic bytes of one k_merge launch: every slot, and every long word's ids + length
    scan_bytes_ = 0;
    for (int c = 0; c < kNumCls; ++c) scan_bytes_ += (double)W.c[c].n * slot_w(c) * sizeof(TokT);
    long_bytes_ = (double)W.ln * 4 + (double)long_tokens_ * sizeof(TokT);
    scan_bytes_ += long_bytes_;
}

template <class TokT>
void MergeLoop<TokT>::alloc_pairs(size_t cap) {
    pcap_ = cap;
    pkey_.alloc(cap);
    pcnt_.alloc(cap);
    pflag_.alloc(cap);
    C_.alloc(cap);
    BPE_HIP(hipMemsetAsync(pkey_.p, 0, pkey_.bytes(), s_));
    BPE_HIP(hipMemsetAsync(pcnt_.p, 0, pcnt_.bytes(), s_));
    BPE_HIP(hipMemsetAsync(pflag_.p, 0, pflag_.bytes(), s_));
    hs_.capC = (unsigned)cap;
}

template <class TokT>
void MergeLoop<TokT>::grow_pairs() {
    DevBuf<unsigned long long> okey = std::move(pkey_);
    DevBuf<long long> ocnt = std::move(pcnt_);
    DevBuf<unsigned> oflag = std::move(pflag_);
    const size_t ocap = pcap_;
    alloc_pairs(ocap * 2);
    hs_.pair_used = 0;
    push_state();
    hipLaunchKernelGGL(k_rehash, dim3(ceil_div(ocap, 256)), dim3(256), 0, s_, okey.p, ocnt.p,
                       oflag.p, ocap, pairs(), st_.p);
    BPE_HIP(hipGetLastError());
    pull_state();
}

template <class TokT>
void MergeLoop<TokT>::ensure_pool(unsigned need) {
    if (hs_.pool_used + (unsigned long long)need <= hs_.pool_cap) return;
    unsigned long long cap = hs_.pool_cap;
    while (hs_.pool_used + (unsigned long long)need > cap) cap *= 2;
    BPE_REQUIRE(cap < (1ULL << 32), BPE_E_LIMIT, "token byte pool exceeds 4 GiB");
    DevBuf<uint8_t> np(cap);
    BPE_HIP(hipMemcpyAsync(np.p, pool_.p, hs_.pool_used, hipMemcpyDeviceToDevice, s_));
    pool_ = std::move(np);
    hs_.pool_cap = (unsigned)cap;
    push_state();
}

template <class TokT>
int MergeLoop<TokT>::rebuild() {
    out_.stats.n_rebuilds++;
    const int grid = 1024;
    BPE_HIP(hipMemsetAsync(rs_.p, 0, sizeof(RebuildStats), s_));
    hipLaunchKernelGGL(k_rebuild_hist, dim3(grid), dim3(256), 0, s_, pairs(), pcap_, rs_.p);
    BPE_HIP(hipGetLastError());
    RebuildStats h;
    BPE_HIP(hipMemcpyAsync(&h, rs_.p, sizeof(h), hipMemcpyDeviceToHost, s_));
    BPE_HIP(hipStreamSynchronize(s_));
    int top = -1;
    for (int k = 63; k >= 0; --k)
        if (h.bins[k]) { top = k; break; }
    if (top < 0) return h.ghosts ? 1 : 2;
    // the log2 bin where the cumulative count from the top crosses the target
    unsigned long long cum = 0;
    int k = top;
    for (; k >= 0; --k) {
        if (cum + h.bins[k] > kTarget) break;
        cum += h.bins[k];
    }
    long long T;
    if (k < 0) {
        T = 1;
    } else {  // refine inside bin k with 1024 linear sub-bins
        const long long lo = 1LL << k, hi = lo << 1;
        const long long width = std::max(1LL, lo / 1024);
        hipLaunchKernelGGL(k_rebuild_sub, dim3(grid), dim3(256), 0, s_, pairs(), pcap_, lo, hi, width, rs_.p);
        BPE_HIP(hipGetLastError());
        BPE_HIP(hipMemcpyAsync(h.sub, rs_.p->sub, sizeof(h.sub), hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipStreamSynchronize(s_));
        T = hi;  // everything above bin k
        for (int j = 1023; j >= 0; --j) {
            if (!h.sub[j]) continue;
            if (cum + h.sub[j] > kTarget && cum > 0) break;
            cum += h.sub[j];
            T = lo + (long long)j * width;
            if (cum > kTarget) break;
        }
    }
    hs_.T = T;
    hs_.nC = 0;
    hs_.halt = HALT_NONE;
    push_state();
    hipLaunchKernelGGL(k_build_C, dim3(grid), dim3(256), 0, s_, pairs(), pcap_, T, st_.p);
    if (batched_) {   // the rebuilt C's best (partials) and candidate list
        BPE_HIP(hipMemsetAsync(&bs_.p->list_n[0], 0, sizeof(bs_.p->list_n), s_));
        hipLaunchKernelGGL(k_apply_batch, dim3(kApplyBatchBlocks), dim3(kApplyBatchThreads), 0, s_, st_.p, bs_.p,
                           (const Batch*)batch_.p, pairs(), toks(), LR_.p, lr_member_,
                           (size_t)kMaxBatch * lr_member_, tok_cap_, part_.p, list_.p, 1, cm_, 0);
    }
    else
        hipLaunchKernelGGL(k_argmax, dim3(kArgBlocks), dim3(256), 0, s_, st_.p, pairs(), toks(), part_.p);
    nparts_ = kArgBlocks;
    BPE_HIP(hipGetLastError());
    pull_state();
    BPE_REQUIRE(!(hs_.err & ERR_C_FULL), BPE_E_NOMEM, "candidate list overflow");
    // re-threshold when C has grown 4x (or past 16k) by crossings since this rebuild
    hs_.c_limit = (unsigned)std::min<unsigned long long>(
        std::max<unsigned long long>(4ull * hs_.nC, 4 * kTarget), hs_.capC);
    push_state();
    return 0;
}

// posting lists are rebuilt (with a compaction) when the round count has grown by this factor
// since the last build (experiment knob BPE355_INDEX_GROWTH)
static double index_growth() {
    static const double g = [] {
        const char* e = std::getenv("BPE355_INDEX_GROWTH");
        return e ? std::max(1.1, std::atof(e)) : 2.5;
    }();
    return g;
}

template <class TokT>
void MergeLoop<TokT>::run() {
    st_.alloc(1);
    rs_.alloc(1);
    tok_cap_ = 256u + (unsigned)n_rounds_ + 1u;
    part_.alloc(std::max<size_t>(std::max<size_t>(kArgBlocks, kApplyBatchBlocks),
                                 ceil_div(4ull * tok_cap_, 256) + kCScanBlocks));
    // single rank: batched rounds (BPE355_BATCH = members per trip, 1..8; 0 = the per-round
    // kernels); sharded per-round exchange: the per-round kernels
    {
        const char* e = std::getenv("BPE355_BATCH");
        max_batch_ = e ? std::min(std::atoi(e), kMaxBatch) : kMaxBatch;
        batched_ = !sharded() && max_batch_ >= 1;
    }
    // cells: two buffers by round (trip) parity; batched: kMaxBatch members each
    lr_member_ = (2ull * tok_cap_ + 63) / 64 * 64;
    LR_.alloc(2 * (batched_ ? (size_t)kMaxBatch : 1) * lr_member_);
    BPE_HIP(hipMemsetAsync(LR_.p, 0, LR_.bytes(), s_));
    if (batched_) {   // touched blocks: the apply visits the dense token prefix and the marked blocks
        const unsigned dense_tok = [] {   // test knob BPE355_DENSE_TOK (>= 128, a multiple of 32; per call)
            const char* e = std::getenv("BPE355_DENSE_TOK");
            const unsigned v = e ? (unsigned)std::max(0, std::atoi(e)) : 2048u;
            return std::max(128u, v / 32 * 32);
        }();
        const unsigned tbw = ceil_div(tok_cap_, 1024u);
        const bool marks = tbw <= kTBMax && !(std::getenv("BPE355_CELL_MARKS") && std::getenv("BPE355_CELL_MARKS")[0] == '0');
        // the apply lists touched blocks once the tokens pass sparse_from (test knob
        // BPE355_SPARSE_FROM; below, scanning every cell costs less than building the list)
        const unsigned sparse_from = [&] {
            const char* e = std::getenv("BPE355_SPARSE_FROM");
            // 16384 (r06h, merge phase at the bench config, two reps: 181.3-181.9 ms, against 182.6-182.8
            // at 8192, 185.6-186.3 at 2048 and 184.5 with no marks)
            return std::max(dense_tok, e ? (unsigned)std::max(0, std::atoi(e)) : 16384u);
        }();
        cm_ = CellMarks{nullptr, nullptr, marks ? tbw : 0u, dense_tok, sparse_from, nullptr};
        if (marks) {
            tb_.alloc(2ull * kTBRep * kMaxBatch * tbw);
            tbc_.alloc((size_t)kMaxBatch * tbw);
            BPE_HIP(hipMemsetAsync(tb_.p, 0, tb_.bytes(), s_));
            BPE_HIP(hipMemsetAsync(tbc_.p, 0, tbc_.bytes(), s_));
            cm_.tb = tb_.p;
            cm_.tbc = tbc_.p;
        }
    }
    if (batched_) {
        bs_.alloc(1);
        BPE_HIP(hipMemsetAsync(bs_.p, 0, sizeof(BatchState), s_));
        batch_.alloc(1);
        BPE_HIP(hipMemsetAsync(batch_.p, 0, sizeof(Batch), s_));
        trip_info_.alloc(2 * kTI * kTrips);
        if (!snap_st_) {   // coherent pinned memory, written by k_snapshot
            BPE_HIP(hipHostMalloc(reinterpret_cast<void**>(&snap_st_), 2 * sizeof(RoundState), hipHostMallocCoherent));
            BPE_HIP(hipHostMalloc(reinterpret_cast<void**>(&snap_ti_), 2 * kTI * kTrips * sizeof(int),
                                  hipHostMallocCoherent));
            BPE_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&snap_st_dev_), snap_st_, 0));
            BPE_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&snap_ti_dev_), snap_ti_, 0));
            for (auto& e : blk_ev_) BPE_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        if (const char* e = std::getenv("BPE355_TRIPS")) trips_ = std::max(1, std::min(std::atoi(e), kTrips));
        list_.alloc(2 * kListCap);   // by trip parity
        // select and merge of a trip in one launch (k_trip), or k_select + k_merge_batch
        const char* fe = std::getenv("BPE355_FOLD");
        fused_ = fe && fe[0] == '1';
    }
    if (batched_ && std::getenv("BPE355_CHECK_MARKS")) {
        dbg_.alloc(8);
        BPE_HIP(hipMemsetAsync(dbg_.p, 0, dbg_.bytes(), s_));
        sig_.alloc(1 + kApplyBatchBlocks);
        BPE_HIP(hipMemsetAsync(sig_.p, 0, sig_.bytes(), s_));
        cm_.sig = sig_.p;
    }
    const char* trip_log_path = std::getenv("BPE355_TRIP_LOG");   // analysis knob: the trips' records
    if (batched_ && trip_log_path) trip_log_.reset(new std::vector<int>());
    m_a_.alloc(n_rounds_); m_b_.alloc(n_rounds_); m_new_.alloc(n_rounds_); m_mode_.alloc(n_rounds_);
    const char* round_log = std::getenv("BPE355_ROUND_LOG");   // analysis knob: per-round records
    if (round_log) m_cnt_.alloc(n_rounds_);
    toff_.alloc(tok_cap_); tlen_.alloc(tok_cap_);
    thash_.alloc(tok_cap_); tpw_.alloc(tok_cap_); tkey8_.alloc(tok_cap_);
    tmap_.alloc(next_pow2(16ull * tok_cap_));   // load <= 1/16: a miss (a fresh pair) is ~1 probe
    BPE_HIP(hipMemsetAsync(tmap_.p, 0, tmap_.bytes(), s_));
    const unsigned pool_cap = std::max(1u << 16, 64u * std::max(max_len_, 8u));
    pool_.alloc(pool_cap);

    // global initial pair histogram (train.py:35-49): one all-reduce when sharded; plus the
    // longest word over all ranks (a merged token can be as long as any rank's longest word)
    if (sharded()) {
        comm_->allreduce_i64(reinterpret_cast<int64_t*>(hist_.p), 65536, s_);
        std::vector<int64_t> ml(comm_->nranks, 0);
        ml[comm_->rank] = max_len_;
        DevBuf<int64_t> d_ml(ml.size());
        BPE_HIP(hipMemcpyAsync(d_ml.p, ml.data(), ml.size() * 8, hipMemcpyHostToDevice, s_));
        comm_->allreduce_i64(d_ml.p, ml.size(), s_);
        BPE_HIP(hipMemcpyAsync(ml.data(), d_ml.p, ml.size() * 8, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipStreamSynchronize(s_));
        for (int64_t v : ml) max_len_ = std::max<unsigned>(max_len_, (unsigned)v);
    }
    // test knob BPE355_PAIR_CAP_LOG2: a smaller first table (>= 2^18 holds the 65 536 byte pairs
    // at load 1/2), so moderate corpora exercise grow_pairs / k_rehash as the bench corpus does
    // first table: ~2 slots per unique word (the bench corpus peaks at 0.8 keys per word, so the
    // table never grows there; each growth is a rehash plus a rebuild of C)
    int pair_log2 = 22;
    while (pair_log2 < 26 && (1ull << pair_log2) < 2ull * n_words_) ++pair_log2;
    if (const char* e = std::getenv("BPE355_PAIR_CAP_LOG2")) pair_log2 = std::max(18, std::min(30, std::atoi(e)));
    alloc_pairs(size_t(1) << pair_log2);
    const unsigned n_single_keep = hs_.n_single;
    memset(&hs_, 0, sizeof(hs_));
    hs_.n_single = n_single_keep;
    hs_.n_rounds = n_rounds_;
    hs_.ntok = 256;
    hs_.capC = (unsigned)pcap_;
    hs_.c_limit = (unsigned)pcap_;
    hs_.pool_used = 256;
    hs_.pool_cap = pool_cap;
    push_state();
    hipLaunchKernelGGL(k_init_tokens, dim3(1), dim3(256), 0, s_, toks());
    hipLaunchKernelGGL(k_init_pairs, dim3(256), dim3(256), 0, s_, hist_.p, pairs(), st_.p);
    BPE_HIP(hipGetLastError());
    pull_state();
    build_index();
    if (batched_) reset_tags();
    hs_.halt = HALT_REBUILD;
    hs_.max_len = std::max(max_len_, 1u);
    hs_.max_batch = max_batch_;
    {
        const char* e = std::getenv("BPE355_LDS_CELLS");
        hs_.narrow_limit = (e ? e[0] != '0' : BPE355_LDS_CELLS != 0) ? (1ll << 32) : 0;
    }
    if (batched_ && std::getenv("BPE355_PROBE") && !BPE355_PROBE_CODE)
        std::fprintf(stderr, "[bpe355 probe] BPE355_PROBE needs a library built with -DBPE355_PROBE_CODE=1 "
                             "(tools/build_variant.sh): no stamps in this one\n");
    if (batched_ && std::getenv("BPE355_PROBE") && BPE355_PROBE_CODE) {
        probe_.alloc((size_t)kProbeSlots * (n_rounds_ / kProbeTrip + 2));
        BPE_HIP(hipMemsetAsync(probe_.p, 0, probe_.bytes(), s_));
        hs_.probe = probe_.p;
    }

    const bool timing = timing_enabled();
    std::vector<hipEvent_t> ev;
    std::vector<uint32_t> hmode;
    if (timing) {
        ev.resize(2 * kBatch);
        for (auto& e : ev) BPE_HIP(hipEventCreate(&e));
    }
    double k1_ms = 0, k1_bytes = 0;
    long long k1_launches = 0;
    const bool sharded = this->sharded();

    const bool trace = std::getenv("BPE355_TRACE") != nullptr;
    const int rank = comm_ ? comm_->rank : 0;
    // host-side phase clock (trace): rebuilds, table growth, compaction + index, trip blocks
    double h_ms[4] = {0, 0, 0, 0};
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto since = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    for (;;) {
        if (trace)
            std::fprintf(stderr, "[bpe355 r%d] round %d halt %d nC %u T %lld pairs %llu err %u\n", rank,
                         hs_.round, hs_.halt, hs_.nC, hs_.T, hs_.pair_used, hs_.err);
        if (hs_.round >= n_rounds_) break;
        if (hs_.halt == HALT_REBUILD) {
            const auto t0 = now();
            const int r = rebuild();
            h_ms[0] += since(t0);
            if (r == 1) { exhaustion(); break; }
            if (r == 2) break;   // no keys left: `if len(byte_pair_frequencies) == 0: break`
        }
        if (batched_) {
            // k_select checks the pair table, the token pool and the compaction schedule before
            // every trip and hands back to the host (HALT_HOST); here the host makes room
            if (hs_.pair_used + 4ull * (hs_.ntok + kMaxBatch) * kMaxBatch > pcap_ / kPairLoadDiv) {
                const auto t0 = now();
                grow_pairs();
                h_ms[1] += since(t0);
                hs_.halt = HALT_REBUILD;   // C holds slot indices: rebuild it
                continue;
            }
            ensure_pool((unsigned)(4 * kMaxBatch) * std::max(max_len_, 1u));
            if (hs_.halt == HALT_HOST) hs_.halt = HALT_NONE;
            hs_.host_round = next_index_round_;
            hs_.single_limit = n_live_ / 4 + 1024;
            hs_.pair_limit = pcap_ / kPairLoadDiv;
            push_state();
            const auto tb0 = now();
            {   // blocks back to back until one halts; the block behind a halted one is empty
                int slot = 0;
                launch_block(slot, timing, ev);
                for (;;) {
                    launch_block(slot ^ 1, timing, ev);
                    finish_block(slot, timing, ev, k1_ms, k1_bytes, k1_launches);
                    if (hs_.halt != HALT_NONE || hs_.err) break;
                    slot ^= 1;
                }
                finish_block(slot ^ 1, timing, ev, k1_ms, k1_bytes, k1_launches);   // drained
            }
            h_ms[3] += since(tb0);
            BPE_REQUIRE(!(hs_.err & ERR_PAIRS_FULL), BPE_E_NOMEM, "pair table overflow");
            BPE_REQUIRE(!(hs_.err & ERR_C_FULL), BPE_E_NOMEM, "candidate list overflow");
            BPE_REQUIRE(!(hs_.err & ERR_POOL), BPE_E_NOMEM, "token pool overflow");
            if (hs_.halt == HALT_DONE) break;
            if (hs_.n_single > n_live_ / 4 + 1024 || hs_.round >= next_index_round_) {
                const auto t0 = now();
                compact();
                build_index();
                reset_tags();
                push_state();
                h_ms[2] += since(t0);
                next_index_round_ = std::max(hs_.round + 512, (int)(hs_.round * index_growth()));
            }
            continue;
        }
        // capacity headroom for one batch (worst case: 2 new keys per token per round)
        int R = std::min(kBatch, n_rounds_ - hs_.round);
        const unsigned long long per_round = 2ull * (hs_.ntok + R + 1);
        // keep the load <= 1/2: an insert is an unsuccessful linear-probe search, ~2.5 probes at
        // load 1/2 vs ~8.5 at 3/4 -- each probe a dependent load in k_apply
        while (hs_.pair_used + per_round * R > pcap_ / 2) {
            if (R > 8) { R /= 2; continue; }
            grow_pairs();
            hs_.halt = HALT_REBUILD;   // C holds slot indices: rebuild it
            break;
        }
        if (hs_.halt == HALT_REBUILD) continue;
        ensure_pool((unsigned)R * std::max(max_len_, 1u));
        const long long start_round = hs_.round;
        for (int k = 0; k < R; ++k) {
            // rewrite -> [one all-reduce of the delta cells when sharded] -> apply -> argmax.
            // (Applying the deltas inside the merge kernel instead was measured slower: each
            // hit's pair updates serialize on one thread, see DESIGN.md.)  With timing on, one
            // launch in kTimingStride is timed, by events stamped from k_merge's own dispatch
            // packet (events on every launch cost ~8 us of idle per round).
            const bool timed = timing && (start_round + k) % kTimingStride == 0;
            // the round's cells: buffer (round & 1); k_apply_argmax clears the other one
            const long long rnd = start_round + k;
            unsigned long long* LRc = LR_.p + (size_t)(rnd & 1) * 2 * tok_cap_;
            unsigned long long* LRo = LR_.p + (size_t)((rnd + 1) & 1) * 2 * tok_cap_;
            hipExtLaunchKernelGGL(k_merge<TokT>, dim3(merge_grid_), dim3(256), 0, s_,
                                  timed ? ev[2 * k] : nullptr, timed ? ev[2 * k + 1] : nullptr, 0,
                                  st_.p, (const Partial*)part_.p, (int)nparts_, pairs(), toks(),
                                  wdev_, idev_, LRc, m_a_.p, m_b_.p, m_new_.p, m_mode_.p, m_cnt_.p);
            if (sharded) {   // the one collective per merge round
                const size_t ntok_bound = 256 + (size_t)rnd + 1;
                comm_->allreduce_i64(reinterpret_cast<int64_t*>(LRc), 2 * ntok_bound, s_);
            }
            const unsigned ntb = 256u + (unsigned)rnd + 1u;
            const unsigned cell_blocks = ceil_div(4ull * ntb, kApplyThreads);
            const unsigned c_blocks = std::min<unsigned>(kCScanBlocks,
                                                         std::max(1u, ceil_div(hs_.c_limit, kApplyThreads)));
            hipLaunchKernelGGL(k_apply_argmax, dim3(cell_blocks + c_blocks), dim3(kApplyThreads), 0, s_, st_.p,
                               pairs(), toks(), (const unsigned long long*)LRc, LRo, ntb, cell_blocks,
                               part_.p);
            nparts_ = cell_blocks + c_blocks;
        }
        BPE_HIP(hipGetLastError());
        pull_state();
        if (timing) {
            const int done = (int)(hs_.round - start_round);
            hmode.resize(std::max(done, 1));
            if (done)
                BPE_HIP(hipMemcpy(hmode.data(), m_mode_.p + start_round, done * 4ull, hipMemcpyDeviceToHost));
            const double slot_avg = scan_bytes_ / std::max(1u, idev_.n_slot_words + words_.ln);
            for (int k = 0; k < std::min(done, R); ++k) {
                if ((start_round + k) % kTimingStride) continue;
                float t = 0;
                BPE_HIP(hipEventElapsedTime(&t, ev[2 * k], ev[2 * k + 1]));
                k1_ms += t;
                // algorithmic bytes: every slot on a full scan; list entries + their slots
                // (at the table's mean slot size) plus the long words in index mode
                k1_bytes += hmode[k] == 0xffffffffu ? scan_bytes_
                                                    : hmode[k] * (4.0 + slot_avg) + long_bytes_;
                ++k1_launches;
            }
        }
        BPE_REQUIRE(!(hs_.err & ERR_PAIRS_FULL), BPE_E_NOMEM, "pair table overflow");
        BPE_REQUIRE(!(hs_.err & ERR_C_FULL), BPE_E_NOMEM, "candidate list overflow");
        BPE_REQUIRE(!(hs_.err & ERR_POOL), BPE_E_NOMEM, "token pool overflow");
        if (hs_.halt == HALT_DONE) break;
        // compaction (drop finished words, narrower slots) + fresh posting lists: when many
        // words finished, and on a geometric schedule so later tokens get lists of their own
        if (hs_.n_single > n_live_ / 4 + 1024 || hs_.round >= next_index_round_) {
            compact();
            build_index();
            push_state();
            next_index_round_ = std::max(hs_.round + 512, (int)(hs_.round * 2.5));
        }
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    if (trace)
        std::fprintf(stderr, "[bpe355] merge loop host clock: rebuild %.1f ms, grow %.1f, compact+index %.1f, trip blocks %.1f\n",
                     h_ms[0], h_ms[1], h_ms[2], h_ms[3]);
    if (round_log && hs_.round) {   // a, b, new, list length (~0: full scan), count per round
        const int rd = hs_.round;
        std::vector<uint32_t> va(rd), vb(rd), vn(rd), vm(rd);
        std::vector<long long> vc(rd);
        BPE_HIP(hipMemcpy(va.data(), m_a_.p, rd * 4ull, hipMemcpyDeviceToHost));
        BPE_HIP(hipMemcpy(vb.data(), m_b_.p, rd * 4ull, hipMemcpyDeviceToHost));
        BPE_HIP(hipMemcpy(vn.data(), m_new_.p, rd * 4ull, hipMemcpyDeviceToHost));
        BPE_HIP(hipMemcpy(vm.data(), m_mode_.p, rd * 4ull, hipMemcpyDeviceToHost));
        BPE_HIP(hipMemcpy(vc.data(), m_cnt_.p, rd * 8ull, hipMemcpyDeviceToHost));
        if (FILE* f = std::fopen(round_log, "wb")) {
            for (int r = 0; r < rd; ++r) {
                std::fwrite(&va[r], 4, 1, f); std::fwrite(&vb[r], 4, 1, f); std::fwrite(&vn[r], 4, 1, f);
                std::fwrite(&vm[r], 4, 1, f); std::fwrite(&vc[r], 8, 1, f);
            }
            std::fclose(f);
        }
    }
    if (dbg_.p) {
        unsigned long long d[8];
        BPE_HIP(hipMemcpy(d, dbg_.p, sizeof(d), hipMemcpyDeviceToHost));
        std::fprintf(stderr, "[bpe355 check-marks] nonzero cells left after the clear: %llu (first: trip %llu member %llu "
                             "cell %llu); bitmap words left: %llu; apply workgroups with another view: %llu (first: "
                             "trip %llu workgroup %llu)\n", d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7]);
        BPE_REQUIRE(d[0] == 0 && d[4] == 0, BPE_E_HIP, "cell marks: a delta outside the marked blocks");
    }
    if (trip_log_ && !trip_log_->empty()) {   // kTI ints per trip (k > 0: the trips that ran)
        if (FILE* f = std::fopen(trip_log_path, "wb")) {
            std::fwrite(trip_log_->data(), sizeof(int), trip_log_->size(), f);
            std::fclose(f);
        }
    }
    if (probe_.p) report_probe();
    if (batched_) {
        BatchState b{};
        BPE_HIP(hipMemcpy(&b, bs_.p, sizeof(b), hipMemcpyDeviceToHost));
        out_.stats.n_trips = trips_run_;
        out_.stats.n_rounds_batched = rounds_batched_;
        if (BPE355_STATS_CODE && std::getenv("BPE355_TRACE")) {
            std::fprintf(stderr, "[bpe355] trips: list overflow %llu, head miss %llu, short %llu; k:", b.n_overflow,
                         b.n_headmiss, b.n_short);
            for (int i = 0; i <= kMaxBatch; ++i) std::fprintf(stderr, " %llu", b.k_hist[i]);
            std::fprintf(stderr, "; k=1 because: a==b %llu, not fresh %llu, no list %llu, P2 fails %llu, tie %llu\n",
                         b.k1_why[0], b.k1_why[1], b.k1_why[2], b.k1_why[3], b.k1_why[4]);
            std::fprintf(stderr, "[bpe355] batch ended by: cap %llu, list ran out %llu, candidate k failed the token "
                         "rules %llu, count gap / tie %llu, P1 alone %llu\n", b.end_why[0], b.end_why[1],
                         b.end_why[2], b.end_why[3], b.end_why[4]);
        }
    }
    out_.stats.merge_kernel_ms = k1_ms;
    out_.stats.merge_kernel_launches = k1_launches;
    out_.stats.merge_kernel_bytes = k1_bytes;
    out_.stats.n_pairs_final = (int64_t)hs_.pair_used;
    out_.stats.n_rounds_device = hs_.round;

    // pull the device decisions and replay them on the host (token bytes, dedupe check)
    const int rd = hs_.round;
    std::vector<uint32_t> ma(rd), mb(rd), mn(rd);
    if (rd) {
        BPE_HIP(hipMemcpyAsync(ma.data(), m_a_.p, rd * 4ull, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipMemcpyAsync(mb.data(), m_b_.p, rd * 4ull, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipMemcpyAsync(mn.data(), m_new_.p, rd * 4ull, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipStreamSynchronize(s_));
    }
    // (out_.merges may already hold the exhaustion tail: prepend the device rounds)
    std::vector<std::pair<std::string, std::string>> tail = std::move(out_.merges);
    out_.merges.clear();
    auto& tb = out_.tok_bytes;
    tb.clear();
    for (int b = 0; b < 256; ++b) tb.push_back(std::string(1, (char)b));
    for (int r = 0; r < rd; ++r) {
        std::string nb = tb[ma[r]] + tb[mb[r]];
        if (mn[r] == tb.size()) tb.push_back(nb);
        else BPE_REQUIRE(mn[r] < tb.size() && tb[mn[r]] == nb, BPE_E_HIP,
                         "device token dedupe disagrees with host replay");
        out_.merges.emplace_back(tb[ma[r]], tb[mb[r]]);
    }
    for (auto& m : tail) out_.merges.push_back(std::move(m));
}

// BPE355_PROBE summary (stderr): mean phase durations of the sampled trips, us
template <class TokT>
void MergeLoop<TokT>::report_probe() {
    std::vector<unsigned long long> pr(probe_.n);
    BPE_HIP(hipMemcpy(pr.data(), probe_.p, probe_.bytes(), hipMemcpyDeviceToHost));
    const char* names[] = {"sel:issue", "sel:p1+list+meta", "sel:rule", "sel:fill", "gap sel>merge", "merge:pop",
                           "merge:rewrite", "merge:flush", "gap merge>apply", "apply:clear", "apply:items",
                           "apply:blocktop", "apply:end", "gap apply>sel"};
    const int from[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13};
    const int to[] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 16};
    double acc[14] = {};
    int n = 0;
    // the last workgroups: merge flush (block 0) -> last merge workgroup done -> apply start;
    // apply end (block 0) -> last apply workgroup done -> the next trip's select start
    double tails[4] = {};
    int nt4 = 0;
    for (size_t t = 0; t + 1 < pr.size() / kProbeSlots; ++t) {
        const unsigned long long* p = &pr[kProbeSlots * t];
        bool ok = true;
        for (int i = 0; i < 14; ++i) ok &= p[i] != 0;
        if (!ok) continue;
        for (int i = 0; i < 13; ++i) acc[i] += (double)(p[to[i]] - p[from[i]]) * 0.01;
        ++n;
        if (p[14] && p[15] && p[16]) {
            tails[0] += (double)(long long)(p[14] - p[8]) * 0.01;
            tails[1] += (double)(long long)(p[9] - p[14]) * 0.01;
            tails[2] += (double)(long long)(p[15] - p[13]) * 0.01;
            tails[3] += (double)(long long)(p[16] - p[15]) * 0.01;
            ++nt4;
        }
    }
    std::fprintf(stderr, "[bpe355 probe] %d sampled trips, mean us:", n);
    for (int i = 0; i < 13 && n; ++i) std::fprintf(stderr, " %s %.2f |", names[i], acc[i] / n);
    std::fprintf(stderr, "\n");
    {   // inside select's rule: p1 over the waves | list head + metadata | clash + k | strict gap / 4'
        double r[4] = {};
        int nr = 0;
        for (size_t t = 0; t + 1 < pr.size() / kProbeSlots; ++t) {
            const unsigned long long* p = &pr[kProbeSlots * t];
            if (!(p[2] && p[17] && p[18] && p[19] && p[3])) continue;
            r[0] += (double)(p[17] - p[2]) * 0.01; r[1] += (double)(p[18] - p[17]) * 0.01;
            r[2] += (double)(p[19] - p[18]) * 0.01; r[3] += (double)(p[3] - p[19]) * 0.01;
            ++nr;
        }
        if (nr)
            std::fprintf(stderr, "[bpe355 probe] select rule: p1 %.2f | head+meta %.2f | clash+k+gap %.2f | record %.2f\n",
                         r[0] / nr, r[1] / nr, r[2] / nr, r[3] / nr);
        double q[6] = {};
        int nq = 0;
        for (size_t t = 0; t + 1 < pr.size() / kProbeSlots; ++t) {
            const unsigned long long* p = &pr[kProbeSlots * t];
            if (!p[1] || !p[24] || !p[25] || !p[26] || !p[27] || !p[28] || !p[2]) continue;
            q[0] += (double)((long long)p[24] - (long long)p[1]) * 0.01; q[1] += (double)((long long)p[25] - (long long)p[24]) * 0.01;
            q[2] += (double)((long long)p[26] - (long long)p[1]) * 0.01; q[3] += (double)((long long)p[27] - (long long)p[25]) * 0.01;
            q[4] += (double)((long long)p[28] - (long long)p[27]) * 0.01; q[5] += (double)((long long)p[2] - (long long)p[28]) * 0.01;
            ++nq;
        }
        if (nq)
            std::fprintf(stderr, "[bpe355 probe] select phase 1 (list thread 0): list entry %.2f | metadata+dedupe %.2f | "
                                 "(wave 0 partials %.2f) | barrier %.2f | rank %.2f | minima+barrier %.2f (%d trips)\n",
                         q[0] / nq, q[1] / nq, q[2] / nq, q[3] / nq, q[4] / nq, q[5] / nq, nq);
        std::vector<double> nls, rl;
        for (size_t t = 0; t + 1 < pr.size() / kProbeSlots; ++t) {
            const unsigned long long* p = &pr[kProbeSlots * t];
            if (p[30]) nls.push_back((double)p[30] - 1);
            if (p[27] && p[29]) rl.push_back(((long long)p[29] - (long long)p[27]) * 0.01);
        }
        {   // the rank stretch split: count ranks (27 -> 29), the barrier behind them (29 -> 31), the
            // exact ranking and the top entries' stores (31 -> 28)
            double a = 0, b = 0, c = 0;
            int n = 0;
            for (size_t t = 0; t + 1 < pr.size() / kProbeSlots; ++t) {
                const unsigned long long* p = &pr[kProbeSlots * t];
                if (!p[27] || !p[29] || !p[31] || !p[28]) continue;
                a += ((long long)p[29] - (long long)p[27]) * 0.01;
                b += ((long long)p[31] - (long long)p[29]) * 0.01;
                c += ((long long)p[28] - (long long)p[31]) * 0.01;
                ++n;
            }
            if (n)
                std::fprintf(stderr, "[bpe355 probe] select rank: count ranks %.2f | barrier %.2f | exact rank + stores %.2f (%d trips)\n",
                             a / n, b / n, c / n, n);
        }
        std::sort(nls.begin(), nls.end());
        std::sort(rl.begin(), rl.end());
        if (!nls.empty() && !rl.empty())
            std::fprintf(stderr, "[bpe355 probe] select list entries p10 %.0f p50 %.0f p90 %.0f max %.0f | ranking loop us p50 %.2f p90 %.2f\n",
                         nls[nls.size() / 10], nls[nls.size() / 2], nls[nls.size() * 9 / 10], nls.back(),
                         rl[rl.size() / 2], rl[rl.size() * 9 / 10]);
    }
    {   // which workgroup finishes last: merge blocks below k register members; apply's last block
        int nm = 0, nm_reg = 0, na = 0, na_lastblk = 0;
        std::vector<int> mlast, alast;
        for (size_t t = 0; t + 1 < pr.size() / kProbeSlots; ++t) {
            const unsigned long long* p = &pr[kProbeSlots * t];
            if (p[20]) { ++nm; nm_reg += (p[20] - 1) < kMaxBatch; mlast.push_back((int)p[20] - 1); }
            if (p[21]) { ++na; na_lastblk += (p[21] - 1) == kApplyGrid - 1; alast.push_back((int)p[21] - 1); }
        }
        if (nm && na) {
            std::sort(alast.begin(), alast.end());
            std::sort(mlast.begin(), mlast.end());
            std::fprintf(stderr, "[bpe355 probe] last merge wg < %d (registers a member): %d of %d (median wg %d) | "
                         "last apply wg = grid-1: %d of %d (median wg %d)\n", kMaxBatch, nm_reg, nm,
                         mlast[mlast.size() / 2], na_lastblk, na, alast[alast.size() / 2]);
            double wl = 0, wc = 0;
            for (size_t t = 0; t + 1 < pr.size() / kProbeSlots; ++t) {
                wl += (double)pr[kProbeSlots * t + 22];
                wc += (double)pr[kProbeSlots * t + 23];
            }
            std::fprintf(stderr, "[bpe355 probe] apply workgroups per trip reserving list space %.1f, C space %.1f\n",
                         wl / na, wc / na);
        }
    }
    if (nt4)
        std::fprintf(stderr, "[bpe355 probe] %d trips: merge last-workgroup tail %.2f | last merge wg > apply start %.2f | "
                     "apply last-workgroup tail %.2f | last apply wg > next select %.2f\n", nt4, tails[0] / nt4,
                     tails[1] / nt4, tails[2] / nt4, tails[3] / nt4);
    // distribution of whole trips (select start -> apply end) and of the rewrite, by trip decile
    std::vector<double> tot, rw;
    std::vector<double> dec_tot(10, 0.0), dec_rw(10, 0.0);
    std::vector<int> dec_n(10, 0);
    size_t nt = 0;   // sampled trips that ran (the buffer is sized for the worst case)
    for (size_t t = 0; t < pr.size() / kProbeSlots; ++t)
        if (pr[kProbeSlots * t] != 0) nt = t + 1;
    for (size_t t = 0; t < nt; ++t) {
        const unsigned long long* p = &pr[kProbeSlots * t];
        bool ok = true;
        for (int i = 0; i < 14; ++i) ok &= p[i] != 0;
        if (!ok) continue;
        const double a = (double)(p[13] - p[0]) * 0.01, b = (double)(p[7] - p[6]) * 0.01;
        tot.push_back(a); rw.push_back(b);
        const size_t d = t * 10 / nt;
        dec_tot[d] += a; dec_rw[d] += b; dec_n[d]++;
    }
    auto pct = [](std::vector<double> v, double q) {
        if (v.empty()) return 0.0;
        std::sort(v.begin(), v.end());
        return v[std::min(v.size() - 1, (size_t)(q * v.size()))];
    };
    std::fprintf(stderr, "[bpe355 probe] trip us p50 %.1f p90 %.1f p99 %.1f max %.1f | rewrite p50 %.1f p90 %.1f p99 %.1f max %.1f\n",
                 pct(tot, 0.5), pct(tot, 0.9), pct(tot, 0.99), pct(tot, 1.0), pct(rw, 0.5), pct(rw, 0.9), pct(rw, 0.99),
                 pct(rw, 1.0));
    std::fprintf(stderr, "[bpe355 probe] by decile (trip/rewrite us):");
    for (int d = 0; d < 10; ++d)
        if (dec_n[d]) std::fprintf(stderr, " %.1f/%.1f", dec_tot[d] / dec_n[d], dec_rw[d] / dec_n[d]);
    std::fprintf(stderr, "\n");
}

template <class TokT>
void MergeLoop<TokT>::reset_tags() {
    tags_.reserve(std::max(idev_.n_slot_words, 1u));
    BPE_HIP(hipMemsetAsync(tags_.p, 0, std::max(idev_.n_slot_words, 1u) * sizeof(uint32_t), s_));
}

// One block: kTrips x [k_select][k_merge_batch][k_apply_batch], then a snapshot of the state
// and of the trips' records into pinned memory, ordered on the stream, and an event.  Two blocks
// are in flight: the host reads one block's snapshot while the next one runs, so the device does
// not idle at every host check.  A block launched after a halt finds nothing to do (k_select
// sees st->halt).  With timing on, k_merge_batch is event-timed on one trip in kTimingStride
// (events stamped by its own dispatch packet).
template <class TokT>
unsigned MergeLoop<TokT>::merge_grid() const {
    // experiment knob: size the grid from the last block's trips (measured slower at the bench
    // config, 531 vs 365 ms of merges: list sizes vary too much from one block of trips to the
    // next), so the full layout is the default
    static const bool adaptive = std::getenv("BPE355_MERGE_GRID_ADAPTIVE") != nullptr;
    // long words are handled by the blocks past the slot-class layout: those need the full grid
    if (!adaptive || wdev_.ln > 0 || merge_grid_cur_ == 0) return merge_grid_;
    return std::min(merge_grid_cur_, merge_grid_);
}

template <class TokT>
void MergeLoop<TokT>::launch_block(int slot, bool timing, std::vector<hipEvent_t>& ev) {
    const size_t lr_member = lr_member_, lr_parity = (size_t)kMaxBatch * lr_member;
    const unsigned ntb = tok_cap_;
    const unsigned apply_blocks = kApplyBatchBlocks;
    // whether this block's applies may list touched blocks: the tokens may pass cm_.sparse_from
    // within the two blocks in flight (the apply decides from the batch's own count)
    const int sparse_hint = cm_.tbw && (long long)hs_.ntok + 2ll * trips_ * kMaxBatch >= (long long)cm_.sparse_from;
    int* ti = trip_info_.p + (size_t)slot * kTI * kTrips;
    slot_base_[slot] = trips_launched_;
    for (int t = 0; t < trips_; ++t) {
        const bool timed = timing && (trips_launched_ + t) % kTimingStride == 0;
        hipEvent_t* e = &ev[2 * ((size_t)slot * kTrips + t)];
        const SelOut so{m_a_.p, m_b_.p, m_new_.p, m_mode_.p, m_cnt_.p, ti, t};
        if (fused_ && sizeof(TokT) == 2) {   // (u32 ids: k_trip would spill at 1024 threads)
            hipExtLaunchKernelGGL(k_trip<TokT>, dim3(trip_grid_), dim3(kTripThreads), 0, s_,
                                  timed ? e[0] : nullptr, timed ? e[1] : nullptr, 0,
                                  st_.p, bs_.p, pairs(), toks(), wdev_trip_, idev_, batch_.p, (const Partial*)part_.p,
                                  (const Partial*)list_.p, so, LR_.p, lr_member, lr_parity, tags_.p, cm_);
        } else {
            hipLaunchKernelGGL(k_select, dim3(1), dim3(kSelThreads), 0, s_, (const RoundState*)st_.p, bs_.p, toks(),
                               idev_, batch_.p, (const Partial*)part_.p, (const Partial*)list_.p, so);
            hipExtLaunchKernelGGL(k_merge_batch<TokT>, dim3(merge_grid()), dim3(256), 0, s_,
                                  timed ? e[0] : nullptr, timed ? e[1] : nullptr, 0,
                                  st_.p, (const Batch*)batch_.p, pairs(), toks(), wdev_, idev_, LR_.p, lr_member,
                                  lr_parity, tags_.p, cm_);
        }
        if (dbg_.p)
            hipLaunchKernelGGL(k_check_clear, dim3(256), dim3(256), 0, s_, (const Batch*)batch_.p, (const unsigned long long*)LR_.p,
                               lr_member, lr_parity, (const unsigned*)cm_.tb, cm_.tbw, dbg_.p);
        hipLaunchKernelGGL(k_apply_batch, dim3(apply_blocks), dim3(kApplyBatchThreads), 0, s_, st_.p, bs_.p,
                           (const Batch*)batch_.p, pairs(), toks(), LR_.p, lr_member, lr_parity, ntb, part_.p,
                           list_.p, 0, cm_, sparse_hint);
        if (sig_.p)
            hipLaunchKernelGGL(k_check_sig, dim3(1), dim3(256), 0, s_, (const Batch*)batch_.p, sig_.p,
                               (unsigned)kApplyBatchBlocks, dbg_.p);
    }
    static_assert(sizeof(RoundState) % 4 == 0, "k_snapshot copies words");
    // the block's snapshot: one small kernel stores the state and the trip records into pinned
    // host memory (two copy packets cost ~3x as much at every block boundary)
    hipLaunchKernelGGL(k_snapshot, dim3(1), dim3(256), 0, s_, (const uint32_t*)st_.p,
                       (unsigned)(sizeof(RoundState) / 4), (const uint32_t*)ti, (unsigned)(kTI * trips_),
                       (uint32_t*)(snap_st_dev_ + slot), (uint32_t*)(snap_ti_dev_ + (size_t)slot * kTI * kTrips));
    BPE_HIP(hipGetLastError());
    BPE_HIP(hipEventRecord(blk_ev_[slot], s_));
    trips_launched_ += trips_;
}

template <class TokT>
void MergeLoop<TokT>::finish_block(int slot, bool timing, std::vector<hipEvent_t>& ev, double& k1_ms,
                                   double& k1_bytes, long long& k1_launches) {
    BPE_HIP(hipEventSynchronize(blk_ev_[slot]));
    hs_ = snap_st_[slot];
    const int* ti = snap_ti_ + (size_t)slot * kTI * kTrips;
    for (int t = 0; t < trips_; ++t) {
        trips_run_ += ti[kTI * t + 1] > 0;
        rounds_batched_ += ti[kTI * t + 1] > 1 ? ti[kTI * t + 1] : 0;
        if (trip_log_) trip_log_->insert(trip_log_->end(), ti + kTI * t, ti + kTI * (t + 1));
    }
    {   // size the merge grid of the blocks launched from now on by this block's largest trip:
        // the members' list entries at one per thread, twice over for growth; a full scan (or
        // a single member without a list) wants the whole layout.  Any grid is correct.
        unsigned need = kMaxBatch;
        for (int t = 0; t < trips_; ++t) {
            if (ti[kTI * t + 1] <= 0) continue;
            if (ti[kTI * t + 2]) { need = merge_grid_; break; }
            need = std::max(need, 2 * ceil_div((unsigned)ti[kTI * t + 3], 256u));
        }
        merge_grid_cur_ = std::max<unsigned>(64, need);
    }
    if (!timing) return;
    const double slot_avg = scan_bytes_ / std::max(1u, idev_.n_slot_words + words_.ln);
    for (int t = 0; t < trips_; ++t) {
        if ((slot_base_[slot] + t) % kTimingStride || ti[kTI * t + 1] <= 0) continue;
        float ms = 0;
        const hipEvent_t* e = &ev[2 * ((size_t)slot * kTrips + t)];
        BPE_HIP(hipEventElapsedTime(&ms, e[0], e[1]));
        // algorithmic bytes: every slot on a full scan, else the members' list entries and their
        // slots (at the table's mean slot size); every long word once per trip
        const bool full = ti[kTI * t + 2] != 0;
        k1_ms += ms;
        k1_bytes += full ? scan_bytes_ : long_bytes_ + (double)(unsigned)ti[kTI * t + 3] * (4.0 + slot_avg);
        ++k1_launches;
    }
}

// Every word is one token: the reference keeps popping the remaining zero-count keys,
// greatest (bytes a, bytes b) first, until the rounds run out or the dict is empty.
template <class TokT>
void MergeLoop<TokT>::exhaustion() {
    const int rd = hs_.round;
    std::vector<uint32_t> ma(rd), mb(rd), mn(rd);
    if (rd) {
        BPE_HIP(hipMemcpyAsync(ma.data(), m_a_.p, rd * 4ull, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipMemcpyAsync(mb.data(), m_b_.p, rd * 4ull, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipMemcpyAsync(mn.data(), m_new_.p, rd * 4ull, hipMemcpyDeviceToHost, s_));
    }
    DevBuf<unsigned long long> keys(std::max<size_t>(hs_.pair_used, 1));
    DevBuf<unsigned> nk(1);
    BPE_HIP(hipMemsetAsync(nk.p, 0, 4, s_));
    hipLaunchKernelGGL(k_collect_present, dim3(1024), dim3(256), 0, s_, pairs(), pcap_, keys.p, nk.p);
    unsigned hk = 0;
    BPE_HIP(hipMemcpyAsync(&hk, nk.p, 4, hipMemcpyDeviceToHost, s_));
    BPE_HIP(hipStreamSynchronize(s_));
    std::vector<unsigned long long> hkeys(hk);
    if (hk) {
        BPE_HIP(hipMemcpyAsync(hkeys.data(), keys.p, hk * 8ull, hipMemcpyDeviceToHost, s_));
        BPE_HIP(hipStreamSynchronize(s_));
    }
    std::vector<std::string> tb;
    for (int b = 0; b < 256; ++b) tb.push_back(std::string(1, (char)b));
    for (int r = 0; r < rd; ++r) {
        std::string nb = tb[ma[r]] + tb[mb[r]];
        if (mn[r] == tb.size()) tb.push_back(nb);
        else BPE_REQUIRE(mn[r] < tb.size() && tb[mn[r]] == nb, BPE_E_HIP,
                         "device token dedupe disagrees with host replay");
    }
    std::vector<std::pair<std::string, std::string>> ghosts;
    ghosts.reserve(hk);
    for (auto k : hkeys) ghosts.emplace_back(tb[k >> 32], tb[k & 0xffffffffu]);
    std::sort(ghosts.begin(), ghosts.end(), [](const auto& x, const auto& y) { return x > y; });
    const size_t left = (size_t)(n_rounds_ - rd);
    if (ghosts.size() > left) ghosts.resize(left);
    out_.stats.n_rounds_host = (int64_t)ghosts.size();
    out_.merges = std::move(ghosts);   // the tail; run() prepends the device rounds
}

}  // namespace

namespace {

// Several ranks: an error one rank met before the first collective (reading or validating its
// slab) is raised by every rank, so none waits in a collective another never reaches.  The
// error of the earliest slab wins; a UTF-8 position is reported in whole-corpus bytes.
void agree_on_errors(Comm* comm, const Error* mine, hipStream_t stream) {
    const int R = comm->nranks;
    std::vector<int64_t> v(3 * (size_t)R, 0);
    if (mine) {
        v[3 * comm->rank] = mine->code;
        v[3 * comm->rank + 1] = mine->sys_errno;
        const size_t p = mine->msg.find("position ");
        v[3 * comm->rank + 2] = p == std::string::npos ? 0 : std::stoll(mine->msg.substr(p + 9));
    }
    DevBuf<int64_t> d(v.size());
    BPE_HIP(hipMemcpyAsync(d.p, v.data(), v.size() * 8, hipMemcpyHostToDevice, stream));
    comm->allreduce_i64(d.p, v.size(), stream);
    BPE_HIP(hipMemcpyAsync(v.data(), d.p, v.size() * 8, hipMemcpyDeviceToHost, stream));
    BPE_HIP(hipStreamSynchronize(stream));
    for (int r = 0; r < R; ++r) {
        const int code = (int)v[3 * r];
        if (!code) continue;
        if (r == comm->rank && mine) throw *mine;
        if (code == BPE_E_UTF8)
            throw Error{code, "'utf-8' codec can't decode byte at position " + std::to_string(v[3 * r + 2])};
        throw Error{code, "rank " + std::to_string(r) + " failed before training (code " + std::to_string(code) + ")",
                    (int)v[3 * r + 1]};
    }
}

}  // namespace

bool per_round_exchange() {
    const char* ex = std::getenv("BPE355_EXCHANGE");
    return ex && std::string(ex) == "rounds";
}

void train_on_device(const uint8_t* d_raw, size_t n, int vocab_size,
                     const std::vector<std::string>& specials, Comm* comm, hipStream_t stream,
                     TrainOutput& out, const TrainOpts& opt, Prepared* pre) {
    const auto t0 = std::chrono::steady_clock::now();
    out = TrainOutput{};
    DevBuf<uint8_t> scratch;
    size_t tn = 0;
    const uint8_t* text = nullptr;
    const bool several = comm && comm->nranks > 1;
    WordCounts wc;
    float count_ms = 0;
    std::chrono::steady_clock::time_point t1;
    {
        Error err{0, ""};
        bool failed = opt.has_pending;
        if (failed) err = opt.pending;
        if (!failed && pre) {   // validated and counted while the corpus arrived (drive.hip)
            text = pre->text;
            tn = pre->n;
            wc = std::move(pre->wc);
            count_ms = pre->count_kernel_ms;
            out.stats.t_prepare_ms = pre->t_prepare_ms;
            out.stats.n_bytes = (int64_t)tn;
            t1 = std::chrono::steady_clock::now() - std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                                         std::chrono::duration<double, std::milli>(pre->t_count_ms));
        } else if (!failed) {
            try {
                text = prepare_text(d_raw, n, scratch, &tn, stream);
                out.stats.t_prepare_ms = ms_since(t0);
                out.stats.n_bytes = (int64_t)tn;
                t1 = std::chrono::steady_clock::now();
                count_words(text, tn, wc, stream, timing_enabled() ? &count_ms : nullptr);
            } catch (const Error& e) {
                if (!several && !opt.slab_offset) throw;
                err = e;
                failed = true;
            }
        }
        if (failed && err.code == BPE_E_UTF8 && opt.slab_offset) {
            const size_t p = err.msg.find("position ");
            if (p != std::string::npos)
                err.msg = "'utf-8' codec can't decode byte at position " +
                          std::to_string(std::stoull(err.msg.substr(p + 9)) + opt.slab_offset);
        }
        if (several) agree_on_errors(comm, failed ? &err : nullptr, stream);
        else if (failed) throw err;
    }

    // len(vocab) at loop start: Vocab(special_tokens) = specials then the 256 bytes, deduped
    std::set<std::string> base;
    for (const auto& s : specials) base.insert(s);
    for (int b = 0; b < 256; ++b) base.insert(std::string(1, (char)b));
    const long long rounds = (long long)vocab_size - (long long)base.size();

    out.stats.t_count_ms = ms_since(t1);
    out.stats.count_kernel_ms = count_ms;
    out.stats.count_kernel_bytes = (double)tn;
    out.stats.n_pretokens = (int64_t)wc.n_pretokens;
    out.stats.n_count_records = (int64_t)wc.n_records;
    out.stats.count_reduce_ms = wc.reduce_ms;
    out.stats.count_partial_ms = wc.partial_ms;
    out.stats.n_count_batches = (int64_t)wc.batches;
    if (rounds <= 0) {
        out.stats.t_total_ms = ms_since(t0);
        return;
    }
    BPE_REQUIRE(rounds < (1LL << 31) - 512, BPE_E_LIMIT, "vocab_size too large");
    // several ranks: by default exchange the word tables once and train on their union with no
    // per-round collective (exchange.hip); BPE355_EXCHANGE=rounds keeps the slabs' words local and
    // all-reduces the pair deltas every round.  BPE355_FORCE_EXCHANGE=1 runs the word exchange
    // on a 1-rank communicator too (tests the collective on a single-GPU box).
    DevBuf<uint8_t> union_text;
    Comm* loop_comm = comm;
    const bool per_round = per_round_exchange();
    if (comm && !per_round && (comm->nranks > 1 || std::getenv("BPE355_FORCE_EXCHANGE"))) {
        auto te = std::chrono::steady_clock::now();
        uint64_t uw = 0;
        union_word_tables(text, wc, comm, stream, union_text, &uw, &out.stats);
        text = union_text.p;
        loop_comm = nullptr;
        out.stats.t_exchange_ms = ms_since(te);
        out.stats.n_exchanged_words = (int64_t)uw;
    }
    if (!opt.merge_loop) {
        out.stats.t_total_ms = ms_since(t0);
        return;
    }
    auto go = [&](auto tag) {
        using TokT = decltype(tag);
        auto t2 = std::chrono::steady_clock::now();
        MergeLoop<TokT> loop(stream, loop_comm, text, (int)rounds, out);
        loop.build_words(wc, specials);
        { WordCounts drop = std::move(wc); }
        out.stats.t_words_ms = ms_since(t2);
        auto t3 = std::chrono::steady_clock::now();
        loop.run();
        out.stats.t_merge_ms = ms_since(t3);
    };
    if (256 + rounds + 1 < 65535) go(uint16_t{});
    else go(uint32_t{});
    out.stats.t_total_ms = ms_since(t0);
}

}  // namespace bpe
