// Tokenizer.encode on the device -- reference models/tokenizer/tokenizer.py:
//   12-38   construction: vocab_inv (last id wins), specials deduped + longest first,
//           missing specials appended with ids len(vocab), len(vocab)+1, ...
//   63-66   segment: re.split on the specials alternation (leftmost match, longest first)
//   68-90   pretokenize each non-special segment on its own with the GPT-2 pattern; drop
//           matches equal to a special; special segments stay whole
//   92-138  per pretoken: repeatedly merge ALL occurrences of the adjacent pair with the lowest
//           merge rank (ties: leftmost) until no pair is ranked; ids via vocab_inv (KeyError)
//
// Device pipeline (one stream):
//   0. (once per tokenizer) build_dictionary: every vocab entry of 2..16 bytes encoded by
//      k_encode_words into an L2-sized open-addressing table, and the one-byte words' ids.
//   1. k_find_specials marks where a special starts (first-byte bitmap, then compare); the
//      sorted matches become the segment table on the device (k_sp_*), or on the host when
//      matches overlap.
//   2. k_enc_scan4: persistent workgroups stage 16 KiB chunks in LDS, evaluate the token-start
//      predicate per 64-byte block, and write one u32 record per pre-token, each chunk's records
//      one dense run: a direct id (one-byte words, one-id dictionary words, via an LDS word
//      cache), a special, a dictionary entry, or the slot of a word-table entry (the long tail).
//   3. k_collect + k_encode_words: the word table's words get their rank-ordered merges once
//      (after step 4's resolve has inserted them).
//   4. k_enc_resolve_c: the scan's pending words (LDS-cache misses) -> a dictionary word's ids'
//      info, or a word-table slot, in a kernel with registers to spare; k_enc_finalize: the
//      table words' slots -> their ids' info.
//   5. k_enc_emit<count>, an exclusive scan of the chunks' id counts, k_enc_emit<write>: per
//      chunk, ids assembled in LDS and stored with coalesced writes.

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "drive.h"
#include "internal.h"
#include "prims.h"
#include "pretok.h"
#include "stage.h"
#include "stage2.h"

namespace bpe {
namespace {

constexpr unsigned long long kOff40 = (1ULL << 40) - 1;

struct Seg {                 // a piece of the text: normal (special = -1) or one special token
    unsigned long long start, end;
    int special;
    int pad;
};

struct EncTables {
    const unsigned long long* pm_key;  // ((a << 32) | b) + 1
    const uint2* pm_val;               // (rank, product)
    unsigned long long pm_mask;
    const int64_t* tok2vid;            // internal token -> vocab id, -1 if absent
    const uint32_t* byte2tok;          // 256 entries
    const uint8_t* sp_bytes;
    const uint32_t* sp_off;
    const uint32_t* sp_len;
    const int64_t* sp_vid;
    int n_sp;
};

__device__ __forceinline__ bool bytes_eq(const uint8_t* x, const uint8_t* y, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (x[i] != y[i]) return false;
    return true;
}

// bytes [gp, gp + len) of s (len <= 16) packed little-endian, with aligned 8-byte loads (three at
// most) when the text runs on past them, else byte by byte
__device__ __forceinline__ void load_word(const uint8_t* __restrict__ s, size_t n, size_t gp, size_t len,
                                          uint64_t& lo, uint64_t& hi) {
    if (gp + 24 > n) {
        pack_word(s, gp, len, lo, hi);
        return;
    }
    const uintptr_t addr = reinterpret_cast<uintptr_t>(s + gp);
    const uint64_t* a = reinterpret_cast<const uint64_t*>(addr & ~(uintptr_t)7);
    const unsigned sh = (unsigned)(addr & 7) * 8;
    const uint64_t q0 = a[0], q1 = a[1];
    const uint64_t q2 = (addr & 7) + len > 16 ? a[2] : 0;
    lo = sh ? (q0 >> sh) | (q1 << (64 - sh)) : q0;
    hi = sh ? (q1 >> sh) | (q2 << (64 - sh)) : q1;
    if (len < 8) {
        lo &= (1ULL << (8 * len)) - 1;
        hi = 0;
    } else if (len < 16) {
        hi &= (1ULL << (8 * (len - 8))) - 1;
    }
}

// ------------------------------------------------------------------ 1. special candidates
// Matches are appended as position << 16 | special index (sorted on the device afterwards).
constexpr int kSpShift = 16;

constexpr int kSpLds = 64;   // specials whose first 16 bytes k_find_specials keeps in LDS
constexpr unsigned kSpBuf = 2048;   // matches a workgroup of k_find_specials stages in LDS

__global__ void __launch_bounds__(256) k_find_specials(const uint8_t* __restrict__ s, size_t n, EncTables E,
                                                       const unsigned* __restrict__ first_mask,
                                                       unsigned long long* __restrict__ key_out,
                                                       unsigned* __restrict__ n_out, unsigned long long cap) {
    // Every special matching at i is recorded (sorted longest first, the host takes the first
    // that fits): when the longest one straddles a piece cut, re.split on that piece still
    // matches a shorter special that is its prefix (tokenizer.py:63-66).
    // A thread takes 16-byte units (aligned loads, two in flight; the text is streamed once),
    // marks the bytes that may start a special (first-byte bitmap) and compares only those: the
    // 16 bytes at a candidate against the specials' first 16 (LDS), the rest byte by byte.
    // Grid-stride, the trip count uniform over the workgroup (the candidate loop's __any).
    __shared__ unsigned s_fm[8];
    __shared__ uint64_t s_lo[kSpLds], s_hi[kSpLds];
    __shared__ uint32_t s_len[kSpLds];
    // the workgroup's matches, flushed with one global reservation at the end (a device-scope
    // atomic per wave that found one: millions of them on one word would serialise at ~88/us)
    __shared__ unsigned long long s_keys[kSpBuf];
    __shared__ unsigned s_nk, s_base;
    if (threadIdx.x == 0) s_nk = 0;
    if (threadIdx.x < 8) s_fm[threadIdx.x] = first_mask[threadIdx.x];
    const int nsl = E.n_sp < kSpLds ? E.n_sp : kSpLds;
    if ((int)threadIdx.x < nsl) {
        const uint32_t l = E.sp_len[threadIdx.x];
        uint64_t lo = 0, hi = 0;
        const uint8_t* p = E.sp_bytes + E.sp_off[threadIdx.x];
        for (uint32_t j = 0; j < l && j < 16; ++j) {
            if (j < 8) lo |= (uint64_t)p[j] << (8 * j);
            else hi |= (uint64_t)p[j] << (8 * (j - 8));
        }
        s_lo[threadIdx.x] = lo;
        s_hi[threadIdx.x] = hi;
        s_len[threadIdx.x] = l;
    }
    __syncthreads();
    const uint8_t* const a0 = s - (reinterpret_cast<uintptr_t>(s) & 15);   // (global address space kept)
    const size_t lead = (size_t)(s - a0);
    const size_t nv = (n + lead + 15) / 16;   // 16-byte units covering [s, s + n)
    const size_t S = (size_t)gridDim.x * blockDim.x;
    auto unit = [&](size_t v, uint32_t (&w)[4]) -> unsigned {   // candidate bits of unit v
        unsigned cm = 0;
        const long long p0 = (long long)(16 * v) - (long long)lead;   // text position of byte 0
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const long long p = p0 + j;
            const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 0xffu;
            if (p >= 0 && p < (long long)n && ((s_fm[b >> 5] >> (b & 31)) & 1u)) cm |= 1u << j;
        }
        return cm;
    };
    auto load = [&](size_t v, uint32_t (&w)[4]) {
        w[0] = w[1] = w[2] = w[3] = 0;
        if (v >= nv) return;
        const long long p0 = (long long)(16 * v) - (long long)lead;
        if (p0 >= 0 && p0 + 16 <= (long long)n) {
            const uint4 q = *reinterpret_cast<const uint4*>(a0 + 16 * v);
            w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
        } else {
            for (int j = 0; j < 16; ++j) {
                const long long p = p0 + j;
                if (p >= 0 && p < (long long)n) w[j >> 2] |= (uint32_t)s[p] << (8 * (j & 3));
            }
        }
    };
    auto check = [&](size_t v, unsigned cm) {
        for (int j = 0; j < 16; ++j) {
            const bool cand = (cm >> j) & 1u;
            if (!__any(cand)) continue;
            const size_t i = 16 * v + j - lead;
            uint64_t tl = 0, th = 0;
            if (cand) load_word(s, n, i, n - i < 16 ? n - i : 16, tl, th);
            for (int k = 0; k < E.n_sp; ++k) {
                bool hit = false;
                if (cand) {
                    const uint32_t l = k < kSpLds ? s_len[k] : E.sp_len[k];
                    if (i + l <= n) {
                        if (k < kSpLds) {
                            const uint64_t mlo = l >= 8 ? ~0ULL : (1ULL << (8 * l)) - 1;
                            const uint64_t mhi = l >= 16 ? ~0ULL : (l <= 8 ? 0ULL : (1ULL << (8 * (l - 8))) - 1);
                            hit = ((tl ^ s_lo[k]) & mlo) == 0 && ((th ^ s_hi[k]) & mhi) == 0 &&
                                  (l <= 16 || bytes_eq(s + i + 16, E.sp_bytes + E.sp_off[k] + 16, l - 16));
                        } else {
                            hit = bytes_eq(s + i, E.sp_bytes + E.sp_off[k], l);
                        }
                    }
                }
                if (hit) {
                    const unsigned long long key = ((unsigned long long)i << kSpShift) | (unsigned)k;
                    const unsigned li = atomicAdd(&s_nk, 1u);
                    if (li < kSpBuf) {
                        s_keys[li] = key;
                    } else {   // the buffer is full: straight to the global list
                        const unsigned idx = atomicAdd(n_out, 1u);
                        if (idx < cap) key_out[idx] = key;
                    }
                }
            }
        }
    };
    for (size_t v0 = (size_t)blockIdx.x * blockDim.x; v0 < nv; v0 += 2 * S) {
        const size_t va = v0 + threadIdx.x, vb = va + S;
        uint32_t wa[4], wb[4];
        load(va, wa);
        load(vb, wb);
        const unsigned ca = va < nv ? unit(va, wa) : 0u, cb = vb < nv ? unit(vb, wb) : 0u;
        if (__any(ca != 0)) check(va, ca);
        if (__any(cb != 0)) check(vb, cb);
    }
    __syncthreads();
    const unsigned nk = s_nk < kSpBuf ? s_nk : kSpBuf;
    if (threadIdx.x == 0) s_base = nk ? atomicAdd(n_out, nk) : 0u;
    __syncthreads();
    for (unsigned q = threadIdx.x; q < nk; q += blockDim.x)
        if (s_base + q < cap) key_out[s_base + q] = s_keys[q];
}

// ------------------------------------------------------------------ 1'. segments on the device
// The sorted matches (position << 16 | index) become the segment table without a host pass when
// the matches that no piece cut splits (a cut strictly inside a match: re.split on the piece
// cannot see it) do not overlap one another -- then re.split keeps every one of them.  Between
// two kept specials (and before the first, after the last) the cuts split the normal text.
// Overlapping matches (a special that overlaps itself or another) go to the host's
// leftmost-longest resolution instead.
__device__ __forceinline__ size_t cuts_le(const unsigned long long* __restrict__ cuts, size_t nc,
                                          unsigned long long p) {   // how many cuts are <= p
    size_t lo = 0, hi = nc;
    while (lo < hi) {
        const size_t mid = (lo + hi) >> 1;
        if (cuts[mid] <= p) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void k_sp_eligible(const unsigned long long* __restrict__ keys, size_t m, const uint32_t* __restrict__ sp_len,
                              const unsigned long long* __restrict__ cuts, size_t nc, uint8_t* __restrict__ elig) {
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (size_t)gridDim.x * blockDim.x) {
        const unsigned long long p = keys[j] >> kSpShift, e = p + sp_len[keys[j] & 0xffffu];
        const size_t i = cuts_le(cuts, nc, p);   // the first cut > p
        elig[j] = (i == nc || cuts[i] >= e) ? 1 : 0;
    }
}

// entry j <= me: the segments ending with special j (j == me: the tail after the last one)
__global__ void k_sp_count(const unsigned long long* __restrict__ keys, size_t me, const uint32_t* __restrict__ sp_len,
                           const unsigned long long* __restrict__ cuts, size_t nc, unsigned long long n,
                           unsigned long long* __restrict__ cnt, unsigned* __restrict__ conflict) {
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j <= me; j += (size_t)gridDim.x * blockDim.x) {
        unsigned long long prev = 0;
        if (j > 0) prev = (keys[j - 1] >> kSpShift) + sp_len[keys[j - 1] & 0xffffu];
        const unsigned long long p = j < me ? keys[j] >> kSpShift : n;
        if (p < prev) atomicOr(conflict, 1u);
        unsigned long long c = j < me ? 1 : 0;
        if (prev < p) c += 1 + (cuts_le(cuts, nc, p - 1) - cuts_le(cuts, nc, prev));   // cuts in (prev, p)
        cnt[j] = c;
    }
}

__global__ void k_sp_emit(const unsigned long long* __restrict__ keys, size_t me, const uint32_t* __restrict__ sp_len,
                          const unsigned long long* __restrict__ cuts, size_t nc, unsigned long long n,
                          const unsigned long long* __restrict__ off, Seg* __restrict__ segs) {
    for (size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x; j <= me; j += (size_t)gridDim.x * blockDim.x) {
        unsigned long long prev = 0;
        if (j > 0) prev = (keys[j - 1] >> kSpShift) + sp_len[keys[j - 1] & 0xffffu];
        const unsigned long long p = j < me ? keys[j] >> kSpShift : n;
        unsigned long long o = off[j];
        if (prev < p) {
            unsigned long long start = prev;
            for (size_t i = cuts_le(cuts, nc, prev); i < nc && cuts[i] < p; ++i) {
                segs[o++] = Seg{start, cuts[i], -1, 0};
                start = cuts[i];
            }
            segs[o++] = Seg{start, p, -1, 0};
        }
        if (j < me) {
            const unsigned k = (unsigned)(keys[j] & 0xffffu);
            segs[o] = Seg{p, p + sp_len[k], (int)k, 0};
        }
    }
}

// ------------------------------------------------------------------ 2. the scan: one record per pre-token
// Records.  Every pre-token becomes one u32; its top bits say what it names:
//   0 | pw                (scan output only) a word the scan left to k_enc_resolve: pending entry
//                         pw (31 bits), which the resolve overwrites with the word's ids' info
//                         (a dictionary word) or its slot record (resolved_is_rec)
//   kRecDirect | id       11: a word of exactly one vocab id (< 2^30): one-byte words (the byte
//                         table) and the dictionary's one-id words
//   kRecSpecial | k       101: special token k
//   kRecSlot | p          100: p < cap: a word-table slot (a word first met in this text, encoded
//                         after the scan by k_encode_words); cap + s: dictionary slot s (a word of
//                         several ids, or none)
// The dictionary (built once per tokenizer, build_dictionary) holds every vocab entry of 2..16
// bytes with its encoding: a pre-token's ids depend only on its bytes (tokenizer.py:124-136), so
// a word found there needs no word-table entry.  The scan itself touches no global table: a word
// its LDS cache does not hold becomes a pending entry (its position and length, 8 bytes), and a
// separate kernel with registers to spare resolves all of them with many lookups in flight --
// the dictionary (2 MB, L2-resident) first, then the word table.
constexpr uint32_t kRecPendBit = 0x80000000u;   // clear: a pending entry
constexpr uint32_t kRecDirect = 0xC0000000u;
constexpr uint32_t kRecSpecial = 0xA0000000u;
constexpr uint32_t kRecSlot = 0x80000000u;
constexpr uint32_t kRecKind3 = 0xE0000000u;     // the kind of a special / slot record
constexpr uint32_t kRecPayload = 0x3FFFFFFFu;   // direct ids are below this
constexpr uint32_t kRecPayload29 = 0x1FFFFFFFu; // slots and special indices
constexpr uint32_t kRecPendMax = 0x7FFFFFFFu;   // pending entries are below this
constexpr uint32_t kRecNone = 0xFFFFFFFFu;      // byte table / dictionary lookup: no record
constexpr uint32_t kDictMark = 0x40000000u;     // DictEnt.rec of a several-id word: kDictMark | slot
__device__ __forceinline__ bool rec_is_direct(uint32_t r) { return (r & kRecDirect) == kRecDirect; }
// A pending entry after the resolve holds either its word's ids' info (a dictionary word: the
// info format of section 5, never in [2^31, 2^32)) or a record kRecSlot | slot (a word-table
// word, whose ids exist only after k_encode_words; k_enc_finalize swaps it for the info).
__device__ __forceinline__ bool resolved_is_rec(unsigned long long v) { return (v >> 31) == 1; }

// ids' info (section 5): kOneId | id, kTwoIds | id1 << 31 | id0, kThreeIds (ids < 2^20),
// kFourIds (ids < 2^15), else nids << 36 | pool offset
constexpr unsigned long long kOneId = 1ULL << 63;
constexpr unsigned long long kTwoIds = 1ULL << 62;
constexpr unsigned long long kThreeIds = 1ULL << 61;
constexpr unsigned long long kFourIds = 1ULL << 60;
constexpr unsigned long long kInlineIds = kOneId | kTwoIds | kThreeIds | kFourIds;
constexpr int kNidsShift = 36;
constexpr unsigned long long kDictPool = 1ULL << 35;
constexpr unsigned long long kPoolOff = kDictPool - 1;

struct DictEnt {               // 32 bytes: one probe is one aligned 32-byte read
    uint64_t lo, hi;           // packed bytes
    uint32_t len;              // 0: an empty slot
    uint32_t rec;              // the word's record (kRecDirect | id, or kDictMark | this slot)
    unsigned long long info;   // its ids (slot_info format below; the pool is the dictionary's)
};
struct EncDict {
    const DictEnt* ent;
    unsigned long long mask;   // slots - 1
    const uint32_t* pool;
    const uint32_t* byte_rec;  // 256 records of the one-byte words (kRecNone: through the table)
    const uint32_t* filt;      // membership bits: a word whose bit is clear is not in the dictionary
};
// The dictionary's membership filter: one bit per hash value's bits 20..39 (128 KB, which stays
// in every XCD's L2 where the 2 MB of entries do not: the resolve's table words, 63 % of the
// pending words at the bench corpus, mostly skip the dictionary probe that would miss L2)
constexpr int kFiltShift = 20;
constexpr unsigned kFiltBits = 1u << 20;
__host__ __device__ inline unsigned filt_index(uint64_t h) { return (unsigned)(h >> kFiltShift) & (kFiltBits - 1); }
__device__ __forceinline__ bool filt_maybe(const EncDict& D, uint64_t h) {
    const unsigned i = filt_index(h);
    return (D.filt[i >> 5] >> (i & 31)) & 1u;
}

__device__ __forceinline__ uint32_t dict_find(const EncDict& D, uint64_t wl, uint64_t wh, uint32_t len, uint64_t h) {
    if (!filt_maybe(D, h)) return kRecNone;
    size_t sl = h & D.mask;
    for (;;) {
        const DictEnt e = D.ent[sl];
        if (e.len == 0) return kRecNone;
        if (e.len == len && e.lo == wl && e.hi == wh) return e.rec;
        sl = (sl + 1) & D.mask;
    }
}
// the same, answering with the word's ids' info (the resolve stores it in the pending entry, so a
// dictionary word needs nothing more after the resolve)
__device__ __forceinline__ bool dict_find_info(const EncDict& D, uint64_t wl, uint64_t wh, uint32_t len, uint64_t h,
                                               unsigned long long* info) {
    if (!filt_maybe(D, h)) return false;
    size_t sl = h & D.mask;
    for (;;) {
        const DictEnt e = D.ent[sl];
        if (e.len == 0) return false;
        if (e.len == len && e.lo == wl && e.hi == wh) {
            *info = e.info;
            return true;
        }
        sl = (sl + 1) & D.mask;
    }
}

// LDS word cache of the scan (2-way): word -> record (build knob BPE355_ENC_CACHE, a power of 2)
#ifndef BPE355_ENC_CACHE
#define BPE355_ENC_CACHE 512
#endif
constexpr int kEncCache = BPE355_ENC_CACHE;
static_assert((kEncCache & (kEncCache - 1)) == 0, "the scan's cache size is a power of two");
#ifndef BPE355_ENC_EPOCH
#define BPE355_ENC_EPOCH 4
#endif
constexpr int kEncEpoch = BPE355_ENC_EPOCH;   // chunks between the scan cache's evictions
constexpr unsigned kEncKeep = 2;
constexpr int kSegLds = 64;

__device__ __forceinline__ int seg_of(const Seg* __restrict__ segs, int nseg, size_t p) {
    int lo = 0, hi = nseg - 1;  // last segment with start <= p
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].start <= p) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

struct ClipWin {   // one block's window with the bytes before window position lo read as '\n'
    int r0, lo;
    __device__ __forceinline__ uint32_t byte(int j) const { return j < lo ? 0x0Au : g_stage[r0 + j]; }
    __device__ __forceinline__ uint32_t dword(int k) const {
        const uint32_t x = *reinterpret_cast<const uint32_t*>(g_stage + r0 + 4 * k);
        const int q = lo - 4 * k;   // bytes of this dword before the segment start
        if (q <= 0) return x;
        if (q >= 4) return 0x0A0A0A0Au;
        const uint32_t m = (1u << (8 * q)) - 1u;
        return (x & ~m) | (0x0A0A0A0Au & m);
    }
};

// The encoder's word table, over the training table's arrays (kv: 16-byte entries, pos): the
// encoder counts nothing, so an entry's second word holds the word's first 8 bytes and a probe
// is one 16-byte load, with no read of the text to verify a key:
//   words of <= 15 bytes: kv[2s] = kInl | len << 56 | bytes 8..14, kv[2s + 1] = ~(bytes 0..7)
//     (claimed by a CAS on the first word, then the second stored; it is never 0 -- that would
//     take eight 0xFF bytes, which valid UTF-8 never holds -- so 0 means "not stored yet" and
//     matches no word, not even one of NUL bytes.  A reader that sees the first word before the
//     second may miss the word and insert it again further on -- a duplicate slot, which encodes
//     to the same ids);
//   longer words: kv[2s] = len << 40 | (offset + 1) of an occurrence, verified against the text.
// pos[s] = an occurrence's offset (k_collect reads (offset, len) of every slot as before).
constexpr int kEncInline = 15;

__device__ __forceinline__ size_t enc_table_add(const uint8_t* __restrict__ s, size_t gp, size_t len, uint64_t wl,
                                                uint64_t wh, uint64_t h, unsigned long long* __restrict__ kv,
                                                unsigned long long* __restrict__ pos, size_t mask,
                                                unsigned* __restrict__ status, bool* inserted) {
    *inserted = false;
    const bool inl = len <= (size_t)kEncInline;
    const unsigned long long mine = inl ? kInl | ((unsigned long long)len << 56) | wh
                                        : ((unsigned long long)len << 40) | (gp + 1);
    size_t slot = h & mask;
    for (int probe = 0; probe < kMaxProbe; ++probe) {
        const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(kv + 2 * slot);
        unsigned long long k = e.x, k0 = e.y;
        if (k == 0) {
            k = atomicCAS(&kv[2 * slot], 0ULL, mine);
            if (k == 0) {   // claimed
                if (inl) kv[2 * slot + 1] = ~wl;
                pos[slot] = gp;
                *inserted = true;
                return slot;
            }
            k0 = kv[2 * slot + 1];
        }
        if (inl) {
            if (k == mine && k0 == ~wl) return slot;
        } else if (!(k & kInl) && (k >> 40) == len) {
            const size_t q = (k & kOffMask) - 1;
            if (bytes_equal(s, q, gp, len)) return slot;
        }
        slot = (slot + 1) & mask;
    }
    atomicOr(status, 1u);
    return ~(size_t)0;
}


struct ScanArgs {
    const uint8_t* s;
    size_t n, n_chunks;
    const Seg* segs;
    int nseg, use_cache;
    unsigned long long* kv;           // the word table (stage.h)
    unsigned long long* pos;
    size_t mask;
    unsigned long long max_fill;
    unsigned long long* fill;
    uint32_t* recs;                   // records, each chunk's run contiguous
    unsigned long long rec_cap;
    unsigned long long rec_region;    // records a workgroup reserves at a time (>= kChunk)
    unsigned long long* rec_fill;
    unsigned long long* rec_base;     // per chunk: its run in recs
    uint32_t* rec_n;
    unsigned long long* pend;         // pending entries: position << 24 | length
    unsigned pend_blocks;             // blocks of kPendBlock entries in the pool
    unsigned* pend_nblk;              // blocks handed out
    uint32_t* block_used;             // entries used per block
    unsigned* status;
};

// A workgroup appends its pending entries to a block of the pool it holds; a block is
// chunk-sized (a chunk has at most one pre-token per byte), so a chunk that does not fit the
// rest of the block takes a new one before its token phase and the appends never check.
constexpr unsigned kPendBlock = kChunk;
constexpr int kPendShift = 24;        // pending entry: position << 24 | length (< 2^24)

// a dictionary record as the emit reads it: several-id words are cap + their dictionary slot
__device__ __forceinline__ uint32_t dict_rec(uint32_t rec, size_t cap) {
    return (rec & kRecDirect) == kDictMark ? kRecSlot | (uint32_t)(cap + (rec & kRecPayload)) : rec;
}

// Persistent workgroups stream 16 KiB chunks through LDS (stage2.h).  Every thread turns its
// 64-byte block into a token-start mask with tokstart.h's predicate, evaluated once per segment
// that overlaps the block on a window clipped to that segment (bytes before the segment start
// read '\n', the segment end is the text end: each segment is pre-tokenized on its own,
// tokenizer.py:68-90); a special segment is one token.  A block's pre-tokens are the set bits of
// its mask, so the chunk's record count and every thread's offset in the chunk's run are one
// block scan of popcounts, and the records of a chunk are written densely.  Per pre-token: a
// special or a one-byte word is its record; a word of 2..16 bytes is looked up in the LDS cache
// (word -> record); anything else becomes a pending entry, cached as such.  Only when the pool
// of pending entries is spent does the scan resolve words itself (dictionary, word table).
// workgroups per CU the scan's registers are capped for (build knob)
#ifndef BPE355_ENC_SCAN_WG
#define BPE355_ENC_SCAN_WG 4
#endif
// the scan's next-chunk loads before the mask phase: 35 spilled VGPRs instead of 63, but no faster
// (168.6-169.4 vs 168.6-168.7 ms per encode, profiles/r04/y_*), so off
#ifndef BPE355_ENC_EARLY_PREFETCH
#define BPE355_ENC_EARLY_PREFETCH 0
#endif
template <bool kAligned>
__global__ void __launch_bounds__(256, BPE355_ENC_SCAN_WG) k_enc_scan4(ScanArgs A, EncDict D) {
    __shared__ uint64_t s_mask[kWords];
    __shared__ unsigned long long c_key[kEncCache];
    __shared__ uint64_t c_lo[kEncCache], c_hi[kEncCache];
    __shared__ uint32_t c_rec[kEncCache];
    __shared__ uint16_t c_hit[kEncCache];   // hits this epoch
    __shared__ uint32_t s_brec[256];
    __shared__ Seg s_seg[kSegLds];
    __shared__ int s_seg0, s_segn;   // first segment of the chunk window and how many are in LDS (-1: too many)
    __shared__ unsigned long long s_red[4];
    __shared__ uint32_t s_wsum[4];
    __shared__ unsigned long long s_rbase, s_rnext, s_rend;   // the record region the workgroup holds
    __shared__ int s_stop, s_pblk;   // s_pblk: the pending block held (-2: none yet, -1: pool spent)
    __shared__ unsigned s_pused;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint8_t* __restrict__ s = A.s;
    const size_t n = A.n;
    const size_t cap = A.mask + 1;
    for (int i = tid; i < kEncCache; i += blockDim.x) { c_key[i] = 0; c_hit[i] = 0; }
    s_brec[tid] = D.byte_rec[tid];
    if (tid == 0) {
        s_pblk = A.pend ? -2 : -1;
        s_pused = 0;
        s_rnext = s_rend = 0;
    }
    load_cls2(tid, blockDim.x);
    unsigned long long inserted = 0;

    // a word resolved here (the pool is spent): dictionary, then the word table (its slot; 0 when
    // the table is full: the host retries with a larger one)
    auto resolve_here = [&](size_t len, size_t gp, uint64_t wl, uint64_t wh, uint64_t h) -> uint32_t {
        if (len <= (size_t)kInline && len >= 2) {
            const uint32_t rec = dict_find(D, wl, wh, (uint32_t)len, h);
            if (rec != kRecNone) return dict_rec(rec, cap);
        }
        bool ins = false;
        const size_t slot = enc_table_add(s, gp, len, wl, wh, h, A.kv, A.pos, A.mask, A.status, &ins);
        inserted += ins;
        return kRecSlot | (slot == ~(size_t)0 ? 0u : (uint32_t)slot);
    };
    // a word left to k_enc_resolve, or resolved here when the pool is spent
    auto pending = [&](size_t len, size_t gp, uint64_t wl, uint64_t wh, bool packed) -> uint32_t {
        const int pb = s_pblk;
        if (pb >= 0) {
            const unsigned idx = atomicAdd(&s_pused, 1u);   // < kPendBlock: reserved per chunk
            const unsigned long long pw = (unsigned long long)pb * kPendBlock + idx;
            A.pend[pw] = ((unsigned long long)gp << kPendShift) | len;
            return (uint32_t)pw;   // a pending record: bit 31 clear
        }
        if (!packed && len <= (size_t)kInline) pack_word(s, gp, len, wl, wh);
        const uint64_t h = len <= (size_t)kInline ? short_hash(wl, wh, len) : hash_word(s, gp, len);
        return resolve_here(len, gp, wl, wh, h);
    };
    // a pre-token of 2..16 bytes at stage position r (global gp): the LDS cache, else pending
    auto short_rec = [&](uint32_t r, size_t len, size_t gp) -> uint32_t {
        uint64_t wl, wh;
        pack_stage(kPre + (int)r, (int)len, wl, wh);
        const uint64_t h = short_hash(wl, wh, len);
        const unsigned ls = (unsigned)(h >> 40) & (kEncCache - 2);
        if (A.use_cache) {
            for (int way = 0; way < 2; ++way) {
                const unsigned sl = ls + way;
                const unsigned long long k = c_key[sl];
                if (k != 0 && k != kBusy && (k >> 40) == len) {
                    __asm__ volatile("" ::: "memory");
                    if (c_lo[sl] == wl && c_hi[sl] == wh) {
                        c_hit[sl] = (uint16_t)(c_hit[sl] + 1);   // a heuristic: races may drop hits
                        return c_rec[sl];
                    }
                }
            }
        }
        const uint32_t rec = pending(len, gp, wl, wh, true);
        if (A.use_cache) {
            for (int way = 0; way < 2; ++way) {   // cache it if a way is free
                const unsigned sl = ls + way;
                if (c_key[sl] == 0 && atomicCAS(&c_key[sl], 0ULL, kBusy) == 0) {
                    c_lo[sl] = wl;
                    c_hi[sl] = wh;
                    c_rec[sl] = rec;
                    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    atomicExch(&c_key[sl], ((unsigned long long)len << 40) | (gp + 1));
                    break;
                }
            }
        }
        return rec;
    };

    uint4 pre[kSVec];
    if (blockIdx.x < A.n_chunks) fetch2<kAligned>(pre, s, n, (size_t)blockIdx.x * kChunk, tid);
    for (size_t c = blockIdx.x; c < A.n_chunks; c += gridDim.x) {
        __syncthreads();
        store2(pre, tid);
        const size_t base = c * kChunk;
        if (tid < 64) {   // wave 0: the segments that overlap the staged window, into LDS
            const size_t w0 = base >= (size_t)kPre ? base - kPre : 0, w1 = base + kWin + kPost;
            const int k0 = seg_of(A.segs, A.nseg, w0);
            const int i = k0 + tid;
            Seg sg{};
            if (i < A.nseg) sg = A.segs[i];
            const bool in = i < A.nseg && sg.start < w1;
            if (in) s_seg[tid] = sg;
            const unsigned long long b = __ballot(in);
            if (tid == 0) {
                s_seg0 = k0;
                s_segn = (b == ~0ULL && k0 + 64 < A.nseg && A.segs[k0 + 64].start < w1) ? -1 : __popcll(b);
                s_stop = *(volatile unsigned long long*)A.fill > A.max_fill;
            }
        }
        __syncthreads();
        if (s_stop) {
            if (tid == 0) atomicOr(A.status, 1u);
            break;
        }
        // the next chunk's loads: before the mask phase (build knob BPE355_ENC_EARLY_PREFETCH), so
        // that they land during its VALU work instead of stalling the token phase's first wait
        if (BPE355_ENC_EARLY_PREFETCH && c + gridDim.x < A.n_chunks) fetch2<kAligned>(pre, s, n, (c + gridDim.x) * kChunk, tid);
        const int seg0 = s_seg0, segn = s_segn;
        auto seg_at = [&](int i) -> Seg { return segn >= 0 ? s_seg[i - seg0] : A.segs[i]; };
        const int seg_end = segn >= 0 ? seg0 + segn : A.nseg;
        auto seg_find = [&](size_t p) -> int {   // the segment holding position p
            if (segn < 0) return seg_of(A.segs, A.nseg, p);
            int lo = seg0, hi = seg_end - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_seg[mid - seg0].start <= p) lo = mid;
                else hi = mid - 1;
            }
            return lo;
        };

        // ---- token starts of this thread's block, per overlapping segment
        const size_t blk = base + 64 * (size_t)tid;
        uint64_t starts = 0, spec = 0;
        if (blk < n) {
            const long long wstart = (long long)blk - kStartPre;
            const int r0 = kPre + 64 * tid - kStartPre;
            for (int i = seg_find(blk); i < seg_end; ++i) {
                const Seg sg = seg_at(i);
                if (sg.start >= blk + 64) break;
                if (sg.end <= blk) continue;
                if (sg.special >= 0) {
                    if (sg.start >= blk) {
                        starts |= 1ULL << (sg.start - blk);
                        spec |= 1ULL << (sg.start - blk);
                    }
                    continue;
                }
                const long long lo = (long long)sg.start - wstart, hi = (long long)sg.end - wstart;
                uint64_t m = token_starts64<DevTab>(ClipWin{r0, lo > 0 ? (int)lo : 0},
                                                    (int)(hi < kStartWin ? hi : kStartWin));
                const int a = sg.start > blk ? (int)(sg.start - blk) : 0;
                const int e = sg.end < blk + 64 ? (int)(sg.end - blk) : 64;
                m &= (e >= 64 ? ~0ULL : ((1ULL << e) - 1)) & (~0ULL << a);
                if (sg.start >= blk) m |= 1ULL << a;   // the segment starts a token
                starts |= m;
            }
        }
        s_mask[tid] = starts;
        // the thread's offset in the chunk's run: a block scan of the per-block record counts
        const uint32_t cnt = (uint32_t)__popcll(starts);
        uint32_t x = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_wsum[wave] = x;
        if (!BPE355_ENC_EARLY_PREFETCH && c + gridDim.x < A.n_chunks) fetch2<kAligned>(pre, s, n, (c + gridDim.x) * kChunk, tid);
        __syncthreads();
        uint32_t toff = x - cnt;
        for (int w = 0; w < wave; ++w) toff += s_wsum[w];
        if (tid == 0) {
            const uint32_t total = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
            // the chunk's run in the workgroup's region; a new region (one global reservation per
            // rec_region records) when it does not fit
            unsigned long long b = s_rnext;
            if (b + total > s_rend) {
                b = atomicAdd(A.rec_fill, A.rec_region);
                s_rend = b + A.rec_region;
                if (s_rend > A.rec_cap) {   // the record buffer is too small: the host retries
                    atomicOr(A.status, 256u);
                    s_rend = 0;
                    b = ~0ULL;
                }
            }
            if (b != ~0ULL) s_rnext = b + total;
            s_rbase = b;
            A.rec_base[c] = b == ~0ULL ? 0 : b;
            A.rec_n[c] = b == ~0ULL ? 0 : total;
            // room in the pending block for every pre-token of the chunk
            if (s_pblk != -1 && (s_pblk == -2 || s_pused + total > kPendBlock)) {
                if (s_pblk >= 0) A.block_used[s_pblk] = s_pused;
                const unsigned nb = atomicAdd(A.pend_nblk, 1u);
                s_pblk = nb < A.pend_blocks ? (int)nb : -1;
                s_pused = 0;
            }
        }
        __syncthreads();
        const unsigned long long rbase = s_rbase;

        // ---- one record per pre-token that starts in the block
        if (rbase != ~0ULL) {
            uint32_t* const out = A.recs + rbase + toff;
            const size_t rem = n > base ? n - base : 0;
            const uint32_t tend = rem < (size_t)kWin ? (uint32_t)rem : (uint32_t)kWin;
            uint32_t k = 0;
            uint64_t m = starts;
            while (m) {
                const uint32_t j = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
                const uint32_t r = 64u * tid + j;
                const size_t gp = base + r;
                uint32_t rec;
                if ((spec >> j) & 1ULL) {
                    rec = kRecSpecial | (uint32_t)seg_at(seg_find(gp)).special;
                } else {
                    size_t e;   // end (global)
                    if (m) {
                        e = base + 64u * tid + (uint32_t)__builtin_ctzll(m);
                    } else {
                        e = ~(size_t)0;
                        for (int w = tid + 1; w < kWords; ++w) {
                            const uint64_t xw = s_mask[w];
                            if (xw) { e = base + 64u * w + (uint32_t)__builtin_ctzll(xw); break; }
                        }
                        if (e == ~(size_t)0) {   // the chunk's last pre-token: its segment decides
                            const Seg sg = seg_at(seg_find(gp));
                            const size_t lim = sg.end < base + tend ? sg.end : base + tend;
                            e = base + token_end(StageText{}, (uint32_t)(lim - base), r);
                            if (lim != sg.end && e + 4 > lim) e = token_end(s, (size_t)sg.end, gp);
                        }
                    }
                    if (e <= gp) { atomicOr(A.status, 16u); rec = kRecSlot; }
                    else {
                        const size_t len = e - gp;
                        if (len == 1) {
                            rec = s_brec[StageText{}[r]];
                            if (rec == kRecNone) rec = pending(1, gp, 0, 0, false);
                        } else if (len <= (size_t)kInline) {
                            rec = short_rec(r, len, gp);
                        } else if (len >= kMaxPretok) {
                            atomicOr(A.status, 2u);
                            rec = kRecSlot;
                        } else {
                            rec = pending(len, gp, 0, 0, false);
                        }
                    }
                }
                out[k++] = rec;
            }
        }
        if ((c - blockIdx.x) / gridDim.x % kEncEpoch == kEncEpoch - 1) {   // cache eviction
            __syncthreads();
            for (int i = tid; i < kEncCache; i += blockDim.x) {
                const unsigned long long kk = c_key[i];
                if (kk == 0 || kk == kBusy) continue;
                if (c_hit[i] >= kEncKeep) { c_hit[i] = 0; continue; }
                c_key[i] = 0;
                c_hit[i] = 0;
            }
        }
        const unsigned long long ins = wave_sum(inserted);
        inserted = 0;
        if (lane == 0) s_red[wave] = ins;
        __syncthreads();
        if (tid == 0) {
            const unsigned long long b = s_red[0] + s_red[1] + s_red[2] + s_red[3];
            if (b) atomicAdd(A.fill, b);
        }
    }
    __syncthreads();
    if (tid == 0 && s_pblk >= 0) A.block_used[s_pblk] = s_pused;
}

// Every pending entry to its final record, in place: the word's bytes from the text, then the
// dictionary, then the word table.  One entry per thread, no mask work: the lookups of many
// entries are in flight at once.
struct ResolveArgs {
    const uint8_t* s;
    size_t n;
    unsigned long long* pend;
    const uint32_t* block_used;
    unsigned long long n_entries;     // blocks handed out x kPendBlock
    unsigned long long* kv;
    unsigned long long* pos;
    size_t mask;
    unsigned long long max_fill;      // words the table takes (load 1/2) before the host retries
    unsigned long long* fill;
    unsigned* status;
    unsigned long long* stats;        // BPE355_TRACE: LDS-cache hits, dictionary hits, table words; else null
};

// the resolve's counters (trace only): one atomic per wave and counter
__device__ __forceinline__ void resolve_stats(unsigned long long* stats, unsigned long long c0, unsigned long long c1,
                                              unsigned long long c2) {
    if (!stats) return;
    c0 = wave_sum(c0);
    c1 = wave_sum(c1);
    c2 = wave_sum(c2);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&stats[0], c0);
        atomicAdd(&stats[1], c1);
        atomicAdd(&stats[2], c2);
    }
}

__global__ void __launch_bounds__(256) k_enc_resolve(ResolveArgs A, EncDict D) {
    unsigned long long inserted = 0, n_dict = 0, n_table = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.n_entries; i += stride) {
        if ((i & (kPendBlock - 1)) >= A.block_used[i / kPendBlock]) continue;
        const unsigned long long e = A.pend[i];
        const size_t gp = (size_t)(e >> kPendShift), len = (size_t)(e & ((1ULL << kPendShift) - 1));
        unsigned long long val = 0;
        bool found = false;
        uint64_t wl = 0, wh = 0, h;
        if (len <= (size_t)kInline) {
            load_word(A.s, A.n, gp, len, wl, wh);
            h = short_hash(wl, wh, len);
            if (len >= 2) found = dict_find_info(D, wl, wh, (uint32_t)len, h, &val);
        } else {
            h = hash_word(A.s, gp, len);
        }
        n_dict += found;
        if (!found) {   // (a probe chain past kMaxProbe sets status 1: the host retries)
            bool ins = false;
            const size_t slot = enc_table_add(A.s, gp, len, wl, wh, h, A.kv, A.pos, A.mask, A.status, &ins);
            inserted += ins;
            ++n_table;
            val = kRecSlot | (slot == ~(size_t)0 ? 0u : (uint32_t)slot);
        }
        A.pend[i] = val;
    }
    resolve_stats(A.stats, 0, n_dict, n_table);
    inserted = wave_sum(inserted);
    if ((threadIdx.x & 63) == 0 && inserted) atomicAdd(A.fill, inserted);
}

// The same with an LDS word cache: a workgroup takes the scan's blocks one at a time (a block
// holds one scan workgroup's misses over ~16 chunks, where mid-frequency words recur beyond the
// scan's small cache), and a word met again skips the dictionary and the table.
constexpr int kResCache = 1024;
__global__ void __launch_bounds__(256) k_enc_resolve_c(ResolveArgs A, EncDict D, unsigned n_blocks) {
    __shared__ unsigned long long c_key[kResCache];
    __shared__ uint64_t c_lo[kResCache], c_hi[kResCache];
    __shared__ uint32_t c_rec[kResCache];   // kRecDirect | id (a one-id dictionary word) or kRecSlot | slot
    unsigned long long inserted = 0, n_hit = 0, n_dict = 0, n_table = 0;
    for (int i = threadIdx.x; i < kResCache; i += blockDim.x) c_key[i] = 0;
    __syncthreads();
    __shared__ unsigned long long s_ins;
    __shared__ int s_full;
    for (unsigned b = blockIdx.x; b < n_blocks; b += gridDim.x) {
        // the words this workgroup inserted so far go to the fill count; past the table's
        // half-load the resolve stops (the host retries with a 4 x larger table)
        const unsigned long long ins = wave_sum(inserted);
        inserted = 0;
        if (threadIdx.x == 0) { s_ins = 0; s_full = 0; }
        __syncthreads();
        if ((threadIdx.x & 63) == 0 && ins) atomicAdd(&s_ins, ins);
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long f = s_ins ? atomicAdd(A.fill, s_ins) + s_ins : *(volatile unsigned long long*)A.fill;
            if (f > A.max_fill) {
                s_full = 1;
                atomicOr(A.status, 1u);
            }
        }
        __syncthreads();
        if (s_full) return;
        const unsigned used = A.block_used[b];
        const size_t base = (size_t)b * kPendBlock;
        for (unsigned j = threadIdx.x; j < used; j += blockDim.x) {
            const unsigned long long e = A.pend[base + j];
            const size_t gp = (size_t)(e >> kPendShift), len = (size_t)(e & ((1ULL << kPendShift) - 1));
            unsigned long long val = 0;   // the dictionary word's info, or the table word's record
            bool found = false;
            uint64_t wl = 0, wh = 0, h;
            unsigned ls = 0;
            const bool cacheable = len >= 2 && len <= (size_t)kInline;
            if (len <= (size_t)kInline) {
                load_word(A.s, A.n, gp, len, wl, wh);
                h = short_hash(wl, wh, len);
                if (cacheable) {
                    ls = (unsigned)(h >> 40) & (kResCache - 2);
                    for (int way = 0; way < 2 && !found; ++way) {
                        const unsigned sl = ls + way;
                        const unsigned long long k = c_key[sl];
                        if (k != 0 && k != kBusy && (k >> 40) == len) {
                            __asm__ volatile("" ::: "memory");
                            if (c_lo[sl] == wl && c_hi[sl] == wh) {
                                const uint32_t r = c_rec[sl];
                                val = rec_is_direct(r) ? kOneId | (r & kRecPayload) : r;
                                found = true;
                            }
                        }
                    }
                    if (found) {
                        ++n_hit;
                        A.pend[base + j] = val;
                        continue;
                    }
                    found = dict_find_info(D, wl, wh, (uint32_t)len, h, &val);
                    n_dict += found;
                }
            } else {
                h = hash_word(A.s, gp, len);
            }
            if (!found) {   // (a probe chain past kMaxProbe sets status 1: the host retries)
                bool ins = false;
                const size_t slot = enc_table_add(A.s, gp, len, wl, wh, h, A.kv, A.pos, A.mask, A.status, &ins);
                inserted += ins;
                ++n_table;
                val = kRecSlot | (slot == ~(size_t)0 ? 0u : (uint32_t)slot);
            }
            // cache it if a way is free (a table word's slot or a one-id word's id; a dictionary
            // word of several ids, rare, is not cached)
            const bool one = (val & kOneId) && (uint32_t)val < kRecPayload;
            if (cacheable && (one || resolved_is_rec(val))) {
                for (int way = 0; way < 2; ++way) {
                    const unsigned sl = ls + way;
                    if (c_key[sl] == 0 && atomicCAS(&c_key[sl], 0ULL, kBusy) == 0) {
                        c_lo[sl] = wl;
                        c_hi[sl] = wh;
                        c_rec[sl] = one ? kRecDirect | (uint32_t)val : (uint32_t)val;
                        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        atomicExch(&c_key[sl], ((unsigned long long)len << 40) | 1ULL);
                        break;
                    }
                }
            }
            A.pend[base + j] = val;
        }
        if (((b - blockIdx.x) / gridDim.x) % 4 == 3) {   // a fresh cache every 4 blocks
            __syncthreads();
            for (int i = threadIdx.x; i < kResCache; i += blockDim.x) c_key[i] = 0;
            __syncthreads();
        }
    }
    resolve_stats(A.stats, n_hit, n_dict, n_table);
    inserted = wave_sum(inserted);
    if ((threadIdx.x & 63) == 0 && inserted) atomicAdd(A.fill, inserted);
}

// ------------------------------------------------------------------ 3. unique words
// Every word-table slot in use -> (slot, offset, length).  A workgroup takes kCollectPer x 256
// slots (coalesced) and reserves its words' positions with ONE global atomic: one per wave would
// be ~0.26 M returning atomics on one word at a 16 M-slot table, ~3 ms at ~88 per us.
constexpr unsigned kCollectPer = 8;
__global__ void __launch_bounds__(256) k_collect(const unsigned long long* __restrict__ kv,
                                                 const unsigned long long* __restrict__ pos, size_t cap,
                                                 uint32_t* __restrict__ w_slot, unsigned long long* __restrict__ w_off,
                                                 uint32_t* __restrict__ w_len, unsigned* __restrict__ n_words) {
    __shared__ unsigned s_n, s_base;
    if (threadIdx.x == 0) s_n = 0;
    const size_t s0 = (size_t)blockIdx.x * 256 * kCollectPer + threadIdx.x;
    unsigned long long key[kCollectPer];
    unsigned mine = 0;
#pragma unroll
    for (unsigned u = 0; u < kCollectPer; ++u) {
        const size_t sl = s0 + (size_t)u * 256;
        key[u] = sl < cap ? kv[2 * sl] : 0ULL;
        mine += key[u] != 0;
    }
    __syncthreads();   // s_n initialised
    const unsigned at = mine ? atomicAdd(&s_n, mine) : 0u;   // LDS: this thread's first position
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_n ? atomicAdd(n_words, s_n) : 0u;
    __syncthreads();
    unsigned w = s_base + at;
#pragma unroll
    for (unsigned u = 0; u < kCollectPer; ++u) {
        const unsigned long long k = key[u];
        if (!k) continue;
        const size_t sl = s0 + (size_t)u * 256;
        const bool inl = (k >> 63) != 0;   // key format: enc_table_add
        w_slot[w] = (uint32_t)sl;
        w_off[w] = inl ? pos[sl] : (k & kOff40) - 1;
        w_len[w] = inl ? (uint32_t)((k >> 56) & 0x7f) : (uint32_t)(k >> 40);
        ++w;
    }
}

// ------------------------------------------------------------------ 5. ids, in one pass
// slot_info[slot] (k_encode_words) and a dictionary entry's info: a word's ids in one 8-byte
// cell -- kOneId | id for a word of one id, kTwoIds | id1 << 31 | id0 for two (ids < 2^31),
// kThreeIds | id2 << 40 | id1 << 20 | id0 for three (ids < 2^20), kFourIds | id3 << 45 | id2 << 30 |
// id1 << 15 | id0 for four (ids < 2^15: vocabularies up to 32768, the bench's 32000), so most
// occurrences need no read of the id pool when their ids are written; else nids << 36 | offset
// into an id pool (the dictionary's pool when kDictPool is set), 0
// for none (a pre-token equal to a special)

__host__ __device__ inline unsigned long long make_info(uint32_t nids, const uint32_t* ids, unsigned long long off) {
    if (nids == 1) return kOneId | ids[0];
    if (nids == 2 && ids[0] < 0x80000000u && ids[1] < 0x80000000u)
        return kTwoIds | ((unsigned long long)ids[1] << 31) | ids[0];
    if (nids == 3 && (ids[0] | ids[1] | ids[2]) < (1u << 20))
        return kThreeIds | ((unsigned long long)ids[2] << 40) | ((unsigned long long)ids[1] << 20) | ids[0];
    if (nids == 4 && (ids[0] | ids[1] | ids[2] | ids[3]) < (1u << 15))
        return kFourIds | ((unsigned long long)ids[3] << 45) | ((unsigned long long)ids[2] << 30) |
               ((unsigned long long)ids[1] << 15) | ids[0];
    return nids ? ((unsigned long long)nids << kNidsShift) | off : 0ULL;
}
__host__ __device__ inline uint32_t info_nids(unsigned long long info) {
    return (info & kOneId) ? 1u : (info & kTwoIds) ? 2u : (info & kThreeIds) ? 3u : (info & kFourIds) ? 4u
                                                        : (uint32_t)((info >> kNidsShift) & 0xffffffu);
}
// an inline info's ids (1..4 of them; the pool format is not inline)
__host__ __device__ inline uint32_t info_inline_ids(unsigned long long info, uint32_t* ids) {
    if (info & kOneId) { ids[0] = (uint32_t)info; return 1; }
    if (info & kTwoIds) {
        ids[0] = (uint32_t)info & 0x7fffffffu;
        ids[1] = (uint32_t)(info >> 31) & 0x7fffffffu;
        return 2;
    }
    if (info & kThreeIds) {
        for (int j = 0; j < 3; ++j) ids[j] = (uint32_t)(info >> (20 * j)) & 0xfffffu;
        return 3;
    }
    for (int j = 0; j < 4; ++j) ids[j] = (uint32_t)(info >> (15 * j)) & 0x7fffu;
    return 4;
}

// After k_encode_words: every resolved pending entry's record replaced by its ids' info (u64,
// slot_info format), so the emit reads a pending word's ids with one gather instead of two
// dependent ones.  One entry per thread, like the resolve.
__global__ void __launch_bounds__(256) k_enc_finalize(unsigned long long* __restrict__ pend,
                                                      const uint32_t* __restrict__ block_used,
                                                      unsigned long long n_entries,
                                                      const unsigned long long* __restrict__ slot_info, size_t cap,
                                                      EncDict D, size_t dict_slots, unsigned* __restrict__ status) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_entries; i += stride) {
        if ((i & (kPendBlock - 1)) >= block_used[i / kPendBlock]) continue;
        const unsigned long long v = pend[i];
        if (!resolved_is_rec(v)) continue;   // a dictionary word's info already
        const uint32_t rec = (uint32_t)v;
        const uint32_t p = rec & kRecPayload29;
        unsigned long long info = 0;
        if (rec_is_direct(rec)) info = kOneId | (rec & kRecPayload);
        else if ((rec & kRecKind3) == kRecSlot && p < cap) info = slot_info[p];
        else if ((rec & kRecKind3) == kRecSlot && p - cap < dict_slots) info = D.ent[p - cap].info;
        else atomicOr(status, 32u);   // a record naming nothing: a bug
        pend[i] = info;
    }
}

struct EmitArgs {
    const uint32_t* recs;
    const unsigned long long* rec_base;
    const uint32_t* rec_n;
    size_t n_chunks;
    const unsigned long long* slot_info;   // word-table slot -> ids
    const uint32_t* pool;
    size_t cap;                            // word-table slots
    EncDict D;
    size_t dict_slots;
    unsigned long long* pend;              // pending entries: their records, or (finalized) their ids' info
    int finalized;
    int writeback;                         // the count pass stores the infos it resolves (no finalize pass)
    const int64_t* sp_vid;
    unsigned long long* ctot;              // per chunk part: its ids (the count pass)
    const unsigned long long* coff;        // per chunk part: its first id's position (exclusive scan)
    unsigned* status;
};

// a record's ids in slot_info format (a one-id word carries its id)
__device__ __forceinline__ unsigned long long rec_info(const EmitArgs& A, uint32_t rec, bool wb = false) {
    uint32_t pw = ~0u;
    if (!(rec & kRecPendBit)) {
        const unsigned long long v = A.pend[rec];
        if (A.finalized || !resolved_is_rec(v)) return v;   // the ids' info (finalize or the resolve)
        pw = rec;
        rec = (uint32_t)v;                                  // k_enc_resolve: a table word's record
    }
    unsigned long long info = 0;
    const uint32_t p = rec & kRecPayload29;
    if (rec_is_direct(rec)) info = kOneId | (rec & kRecPayload);
    else if ((rec & kRecKind3) == kRecSpecial) info = kOneId | (uint32_t)A.sp_vid[p];
    else if (p < A.cap) info = A.slot_info[p];
    else if (p - A.cap < A.dict_slots) info = A.D.ent[p - A.cap].info;
    else atomicOr(A.status, 32u);   // a record naming nothing: a bug
    // the count pass of the no-finalize mode: the pending entry takes its info (every record
    // naming it stores the same value), so the write pass reads it directly
    if (wb && pw != ~0u) A.pend[pw] = info;
    return info;
}

// the ids of one info through put(position, id), from position o; returns how many
template <class Put>
__device__ __forceinline__ uint32_t put_ids(const EmitArgs& A, unsigned long long info, uint32_t o, const Put& put) {
    if (info & kInlineIds) {
        uint32_t ids[4];
        const uint32_t nm = info_inline_ids(info, ids);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            if (j < nm) put(o + j, ids[j]);
        return nm;
    }
    const uint32_t nm = info_nids(info);
    const uint32_t* src = ((info & kDictPool) ? A.D.pool : A.pool) + (info & kPoolOff);
    for (uint32_t j = 0; j < nm; ++j) put(o + j, src[j]);
    return nm;
}

// exclusive scan of v over the 256 threads: this thread's offset; *total = the sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_ws, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_ws[wave] = x;
    __syncthreads();
    uint32_t off = x - v;
    for (int w = 0; w < wave; ++w) off += s_ws[w];
    *total = s_ws[0] + s_ws[1] + s_ws[2] + s_ws[3];
    __syncthreads();
    return off;
}

// Two passes over the chunks, no dependence between workgroups: kCount sums each chunk's ids
// (its records' infos gathered, all loads issued together) into ctot[c]; after an exclusive scan
// of those (coff), the write pass gathers them again -- the chunk's pending entries were just
// read and sit in a few KB of L2 -- assembles the ids in LDS and stores them with coalesced
// 16-byte writes at coff[c] (a chunk averages ~5 K ids).  (A one-pass form with a decoupled
// look-back over the chunks measured slower: its look-back chains)  OutT
// uint32_t: the ids; uint16_t: np.uint16 as encode.py saves them (encode.py:37), an id past
// 65535 reported in status (bit 128) instead of wrapped.
// The passes work on PARTS of chunks (kEmitParts per chunk, the chunk's records split evenly):
// half the registers and LDS of a whole chunk, so twice the workgroups per CU to hide the
// gathers' latency (the write pass is latency-bound at 3 workgroups per CU).
constexpr unsigned kEmitParts = 2;
constexpr unsigned kEmitIds = 12288 / kEmitParts;   // ids staged per part
constexpr int kEmitR = 16 / (int)kEmitParts;        // records per thread held in registers

template <class OutT, bool kCount>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) k_enc_emit(EmitArgs A, OutT* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[kCount ? 4 : kEmitIds];
    __shared__ uint32_t s_ws[4];
    __shared__ unsigned s_wide;
    const int tid = threadIdx.x;
    constexpr bool kNarrow = sizeof(OutT) == 2;
    bool wide = false;
    if (tid == 0) s_wide = 0;
    for (size_t c = blockIdx.x; c < A.n_chunks * kEmitParts; c += gridDim.x) {   // c: a part
        const size_t ch = c / kEmitParts;
        const unsigned part = (unsigned)(c % kEmitParts);
        const uint32_t mc = A.rec_n[ch];
        const uint32_t r0 = (uint32_t)((unsigned long long)mc * part / kEmitParts);
        const uint32_t m = (uint32_t)((unsigned long long)mc * (part + 1) / kEmitParts) - r0;
        const uint32_t* __restrict__ r = A.recs + A.rec_base[ch] + r0;
        if (m <= 256u * kEmitR) {
            const uint32_t R = (m + 255) >> 8;
            const uint32_t lo = tid * R, hi = lo + R < m ? lo + R : m;
            unsigned long long info[kEmitR];
#pragma unroll
            for (int i = 0; i < kEmitR; ++i) info[i] = lo + i < hi ? rec_info(A, r[lo + i], kCount && A.writeback) : 0ULL;
            uint32_t sum = 0;
#pragma unroll
            for (int i = 0; i < kEmitR; ++i) sum += lo + i < hi ? info_nids(info[i]) : 0u;
            uint32_t T;
            const uint32_t toff = block_excl_scan(sum, s_ws, &T);
            if (kCount) {
                if (tid == 0) A.ctot[c] = T;
            } else if (T <= kEmitIds) {
                const unsigned long long P = A.coff[c];
                uint32_t o = toff;
#pragma unroll
                for (int i = 0; i < kEmitR; ++i)
                    if (lo + i < hi) o += put_ids(A, info[i], o, [&](uint32_t q, uint32_t v) { buf[q] = v; });
                __syncthreads();
                // out + P is OutT-aligned: a scalar head up to 16-byte alignment, then 16-byte stores
                constexpr unsigned kPer = 16 / sizeof(OutT);
                const unsigned head = (unsigned)(((16 - ((uintptr_t)(out + P) & 15)) & 15) / sizeof(OutT));
                const unsigned h = head < T ? head : T;
                if ((unsigned)tid < h) {
                    out[P + tid] = (OutT)buf[tid];
                    wide |= buf[tid] > 0xffffu;
                }
                const unsigned body = (T - h) / kPer;
                uint4* dst = reinterpret_cast<uint4*>(out + P + h);
                for (unsigned i = tid; i < body; i += 256) {
                    const unsigned q = h + kPer * i;
                    if (kNarrow) {
                        uint32_t w[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint32_t a = buf[q + 2 * k], b = buf[q + 2 * k + 1];
                            wide |= (a | b) > 0xffffu;
                            w[k] = (a & 0xffffu) | (b << 16);
                        }
                        dst[i] = make_uint4(w[0], w[1], w[2], w[3]);
                    } else {
                        dst[i] = make_uint4(buf[q], buf[q + 1], buf[q + 2], buf[q + 3]);
                    }
                }
                for (unsigned q = h + kPer * body + tid; q < T; q += 256) {
                    out[P + q] = (OutT)buf[q];
                    wide |= buf[q] > 0xffffu;
                }
                __syncthreads();   // buf is reused by the next chunk
            } else {   // too many ids for LDS: straight to memory
                const unsigned long long P = A.coff[c];
                uint32_t o = toff;
#pragma unroll
                for (int i = 0; i < kEmitR; ++i)
                    if (lo + i < hi)
                        o += put_ids(A, info[i], o, [&](uint32_t q, uint32_t v) {
                            out[P + q] = (OutT)v;
                            wide |= kNarrow && v > 0xffffu;
                        });
            }
        } else if (kCount) {   // many records: rounds of 256
            uint32_t sum = 0;
            for (uint32_t b = 0; b < m; b += 256)
                if (b + tid < m) sum += info_nids(rec_info(A, r[b + tid], A.writeback));
            uint32_t T;
            (void)block_excl_scan(sum, s_ws, &T);
            if (tid == 0) A.ctot[c] = T;
        } else {
            const unsigned long long P = A.coff[c];
            uint32_t run = 0;
            for (uint32_t b = 0; b < m; b += 256) {
                const unsigned long long inf = b + tid < m ? rec_info(A, r[b + tid]) : 0ULL;
                uint32_t rt;
                const uint32_t off = block_excl_scan(b + tid < m ? info_nids(inf) : 0u, s_ws, &rt);
                if (b + tid < m)
                    put_ids(A, inf, run + off, [&](uint32_t q, uint32_t v) {
                        out[P + q] = (OutT)v;
                        wide |= kNarrow && v > 0xffffu;
                    });
                run += rt;
            }
        }
    }
    if (kNarrow && !kCount) {
        if (wide) s_wide = 1;
        __syncthreads();
        if (tid == 0 && s_wide) atomicOr(A.status, 128u);
    }
}

__device__ __forceinline__ uint2 rank_of(const EncTables& E, uint32_t a, uint32_t b) {
    const unsigned long long key = ((((unsigned long long)a) << 32) | b) + 1ULL;
    size_t s = mix64(key) & E.pm_mask;
    for (;;) {
        const unsigned long long k = E.pm_key[s];
        if (k == key) return E.pm_val[s];
        if (k == 0) return make_uint2(0xffffffffu, 0);
        s = (s + 1) & E.pm_mask;
    }
}

// tokenizer.py:124-136 for one unique word; the ids are written once into the word's slot
__global__ void __launch_bounds__(256)
k_encode_words(const uint8_t* __restrict__ s, EncTables E, const unsigned long long* __restrict__ w_off,
               const uint32_t* __restrict__ w_len, const unsigned long long* __restrict__ w_idoff,
               const uint32_t* __restrict__ w_slot, unsigned n_words, uint32_t* __restrict__ pool,
               unsigned long long* __restrict__ slot_info, unsigned* __restrict__ status, size_t n) {
    const unsigned w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n_words) return;
    const uint32_t len = w_len[w];
    unsigned long long* info = slot_info + w_slot[w];
    if (w_off[w] + len > n) { atomicOr(status, 64u); *info = 0; return; }   // a bug: report
    const uint8_t* src = s + w_off[w];
    for (int k = 0; k < E.n_sp; ++k)  // match() drops pre-tokens equal to a special (73)
        if (E.sp_len[k] == len && bytes_eq(src, E.sp_bytes + E.sp_off[k], len)) { *info = 0; return; }
    uint32_t* t = pool + w_idoff[w];
    for (uint32_t i = 0; i < len; ++i) t[i] = E.byte2tok[src[i]];
    uint32_t m = len;
    while (m > 1) {
        uint32_t best = 0xffffffffu, prod = 0, ba = 0, bb = 0;
        for (uint32_t i = 0; i + 1 < m; ++i) {
            const uint2 r = rank_of(E, t[i], t[i + 1]);
            if (r.x < best) { best = r.x; prod = r.y; ba = t[i]; bb = t[i + 1]; }
        }
        if (best == 0xffffffffu) break;
        uint32_t j = 0;  // merge() (92-109): every occurrence, left to right
        for (uint32_t i = 0; i < m;) {
            if (t[i] == ba && i + 1 < m && t[i + 1] == bb) { t[j++] = prod; i += 2; }
            else t[j++] = t[i++];
        }
        m = j;
    }
    for (uint32_t i = 0; i < m; ++i) {
        const int64_t v = E.tok2vid[t[i]];
        if (v < 0) atomicOr(status, 4u);
        t[i] = (uint32_t)v;
    }
    *info = make_info(m, t, w_idoff[w]);
}

__global__ void k_word_len64(const uint32_t* __restrict__ w_len, unsigned n, unsigned long long* __restrict__ o) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = w_len[i];
}

}  // namespace
}  // namespace bpe

// =================================================================== the tokenizer object
struct bpe_tokenizer {
    std::vector<std::string> specials;     // deduped, longest first
    std::vector<int64_t> special_vid;
    hipStream_t stream = nullptr;
    bpe::DevBuf<unsigned long long> pm_key;
    bpe::DevBuf<uint2> pm_val;
    size_t pm_cap = 0;
    bpe::DevBuf<int64_t> tok2vid;
    bpe::DevBuf<uint32_t> byte2tok;
    bpe::DevBuf<uint8_t> sp_bytes;
    bpe::DevBuf<uint32_t> sp_off, sp_len;
    bpe::DevBuf<int64_t> sp_vid;
    bpe::DevBuf<unsigned> first_mask;
    // the encoder's dictionary (build_dictionary): every vocab entry of 2..16 bytes with its ids,
    // the one-byte words' records
    bpe::DevBuf<bpe::DictEnt> dict_ent;
    bpe::DevBuf<uint32_t> dict_pool, byte_rec, dict_filt;
    size_t dict_slots = 0, dict_words = 0;
    // the per-pre-token record buffer, kept for the next call: freeing and re-allocating tens of
    // GB per call costs up to seconds in the driver (measured 0.5 -> 2.8 s for an 11.9 GB
    // encode).  Calls on one handle are serialized on its stream.
    bpe::DevBuf<uint32_t> recs_cache;
    // the other per-call device arrays, kept the same way (grow-only): per chunk, per word-table
    // slot, per unique word, the id pool, the u16 output of the bulk encoder
    struct Scratch {
        bpe::DevBuf<uint32_t> rec_n, w_slot, w_len, pool, block_used;
        bpe::DevBuf<unsigned long long> rec_base, rec_fill, fill, kv, pos, w_off, len64, idoff, slot_info;
        bpe::DevBuf<unsigned> status, d_nw, pend_nblk;
        bpe::DevBuf<unsigned long long> ctot, coff;   // per chunk: ids, first id's position
        bpe::DevBuf<unsigned long long> rstats;       // the resolve's counters (BPE355_TRACE)
        bpe::PieceScratch piece;                      // encode_file's piece-start search
        bpe::DevBuf<unsigned long long> pend;   // the scan's pending entries (resolved in place)
        bpe::DevBuf<bpe::Seg> segs;
        bpe::DevBuf<unsigned long long> sp_key, sp_sorted;   // special matches, (position << 16 | index)
        bpe::DevBuf<unsigned long long> sp_cnt, sp_off, cuts;   // the device segment builder's arrays
        bpe::DevBuf<uint8_t> sp_flag;
        bpe::DevBuf<uint8_t> tmp;
        bpe::DevBuf<uint16_t> ids16;
        bpe::DevBuf<uint8_t> text, text2;   // the bulk encoder's file bytes (and its newline-translated copy)
    } sc;
    // construction inputs, to build the same tables for the other ranks of a multi-device encode
    // (bpe_tok_encode_gpus); those copies own their stream and record buffer
    std::string vblob, mblob;
    std::vector<std::string> sp_in;
    int device = 0;
    std::mutex copies_m;
    std::vector<std::pair<long long, std::unique_ptr<bpe_tokenizer>>> copies;   // (rank << 8 | device)
    ~bpe_tokenizer() {
        if (stream) (void)hipStreamDestroy(stream);
    }
    bpe::EncTables tables() const {
        return bpe::EncTables{pm_key.p, pm_val.p, (unsigned long long)(pm_cap - 1), tok2vid.p,
                              byte2tok.p, sp_bytes.p, sp_off.p, sp_len.p, sp_vid.p,
                              (int)specials.size()};
    }
    bpe::EncDict dict() const {
        return bpe::EncDict{dict_ent.p, (unsigned long long)(dict_slots - 1), dict_pool.p, byte_rec.p, dict_filt.p};
    }
};

namespace bpe {
namespace {

uint32_t rd_u32(const uint8_t*& p, const uint8_t* end) {
    BPE_REQUIRE(p + 4 <= end, BPE_E_ARG, "truncated blob");
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
}

// The encoder's dictionary: every vocab entry of 2..16 bytes, encoded once on the device by
// k_encode_words exactly as a pre-token of those bytes is (tokenizer.py:124-136), in an open-
// addressing table keyed by the packed bytes; plus the record of every one-byte word.  Entries
// whose encoding has an id outside the direct range (or a missing vocab id: the KeyError path)
// are left out, so those words take the word table as before.
void build_dictionary(bpe_tokenizer& T, const std::unordered_map<std::string, uint32_t>& intern,
                      const std::vector<int64_t>& vid, const std::vector<uint32_t>& b2t) {
    std::vector<const std::string*> cand;
    for (const auto& kv : intern)
        if (kv.first.size() >= 2 && kv.first.size() <= (size_t)kInline && vid[kv.second] >= 0)
            cand.push_back(&kv.first);
    std::sort(cand.begin(), cand.end(), [](const std::string* a, const std::string* b) { return *a < *b; });
    const size_t nc = cand.size();
    std::vector<unsigned long long> info(nc);
    std::vector<uint32_t> pool;
    if (nc) {
        std::string text;
        std::vector<unsigned long long> off(nc), idoff(nc);
        std::vector<uint32_t> len(nc), slot(nc);
        for (size_t i = 0; i < nc; ++i) {
            off[i] = text.size();
            idoff[i] = text.size();   // ids <= bytes: the pool mirrors the text
            len[i] = (uint32_t)cand[i]->size();
            slot[i] = (uint32_t)i;
            text += *cand[i];
        }
        DevBuf<uint8_t> d_text(text.size());
        DevBuf<unsigned long long> d_off(nc), d_idoff(nc), d_info(nc);
        DevBuf<uint32_t> d_len(nc), d_slot(nc), d_pool(text.size());
        DevBuf<unsigned> d_status(1);
        to_device(d_text.p, text.data(), text.size(), T.stream);
        to_device(d_off.p, off.data(), nc * 8, T.stream);
        to_device(d_idoff.p, idoff.data(), nc * 8, T.stream);
        to_device(d_len.p, len.data(), nc * 4, T.stream);
        to_device(d_slot.p, slot.data(), nc * 4, T.stream);
        BPE_HIP(hipMemsetAsync(d_status.p, 0, 4, T.stream));
        hipLaunchKernelGGL(k_encode_words, dim3(ceil_div(nc, 256)), dim3(256), 0, T.stream, d_text.p, T.tables(),
                           d_off.p, d_len.p, d_idoff.p, d_slot.p, (unsigned)nc, d_pool.p, d_info.p, d_status.p,
                           text.size());
        BPE_HIP(hipGetLastError());
        pool.resize(text.size());
        to_host(info.data(), d_info.p, nc * 8, T.stream);
        to_host(pool.data(), d_pool.p, text.size() * 4, T.stream);
    }
    T.dict_slots = next_pow2(std::max<size_t>(64, 2 * nc));
    std::vector<DictEnt> ent(T.dict_slots);
    std::memset(ent.data(), 0, ent.size() * sizeof(DictEnt));
    std::vector<uint32_t> dpool;
    size_t words = 0;
    for (size_t i = 0; i < nc; ++i) {
        const unsigned long long inf = info[i];
        std::vector<uint32_t> ids;
        if (inf & kInlineIds) {
            uint32_t x[4];
            ids.assign(x, x + info_inline_ids(inf, x));
        } else if (inf) {
            const uint32_t nm = info_nids(inf);
            const size_t o = (size_t)(inf & kPoolOff);
            ids.assign(pool.begin() + o, pool.begin() + o + nm);
        }
        bool ok = true;
        for (uint32_t x : ids) ok = ok && x < kRecPayload;
        if (!ok) continue;
        const std::string& w = *cand[i];
        uint64_t lo = 0, hi = 0;
        for (size_t j = 0; j < w.size(); ++j) {
            const uint64_t b = (uint8_t)w[j];
            if (j < 8) lo |= b << (8 * j);
            else hi |= b << (8 * (j - 8));
        }
        size_t sl = short_hash(lo, hi, w.size()) & (T.dict_slots - 1);
        while (ent[sl].len) sl = (sl + 1) & (T.dict_slots - 1);
        DictEnt& e = ent[sl];
        e.lo = lo;
        e.hi = hi;
        e.len = (uint32_t)w.size();
        if (ids.size() == 1) {
            e.rec = kRecDirect | ids[0];
            e.info = kOneId | ids[0];
        } else {
            e.rec = kDictMark | (uint32_t)sl;
            e.info = make_info((uint32_t)ids.size(), ids.data(), kDictPool | dpool.size());
            if (!ids.empty() && !(e.info & kInlineIds)) dpool.insert(dpool.end(), ids.begin(), ids.end());
        }
        ++words;
    }
    T.dict_words = words;
    std::vector<uint32_t> brec(256, kRecNone);
    for (int b = 0; b < 256; ++b) {
        const int64_t v = vid[b2t[b]];
        bool special = false;
        for (const auto& sp : T.specials) special = special || (sp.size() == 1 && (uint8_t)sp[0] == b);
        if (v >= 0 && v < (int64_t)kRecPayload && !special) brec[b] = kRecDirect | (uint32_t)v;
    }
    T.dict_ent.alloc(ent.size());
    to_device(T.dict_ent.p, ent.data(), ent.size() * sizeof(DictEnt), T.stream);
    T.dict_pool.alloc(std::max<size_t>(dpool.size(), 1));
    if (!dpool.empty()) to_device(T.dict_pool.p, dpool.data(), dpool.size() * 4, T.stream);
    T.byte_rec.alloc(256);
    to_device(T.byte_rec.p, brec.data(), 256 * 4, T.stream);
    std::vector<uint32_t> filt(kFiltBits / 32, 0u);
    for (const DictEnt& e : ent)
        if (e.len) {
            const unsigned i = filt_index(short_hash(e.lo, e.hi, e.len));
            filt[i >> 5] |= 1u << (i & 31);
        }
    T.dict_filt.alloc(filt.size());
    to_device(T.dict_filt.p, filt.data(), filt.size() * 4, T.stream);
    BPE_HIP(hipStreamSynchronize(T.stream));
}

void build_tokenizer(bpe_tokenizer& T, const uint8_t* vb, size_t vn, const uint8_t* mb, size_t mn,
                     const std::vector<std::string>& sp_in) {
    std::unordered_map<std::string, uint32_t> intern;
    std::vector<int64_t> vid;
    auto tok = [&](const std::string& s) {
        auto it = intern.find(s);
        if (it != intern.end()) return it->second;
        const uint32_t id = (uint32_t)intern.size();
        intern.emplace(s, id);
        vid.push_back(-1);
        return id;
    };
    // vocab_inv = {bytes: id}: last id wins (tokenizer.py:19)
    const uint8_t* p = vb;
    const uint8_t* end = vb + vn;
    const uint32_t nv = rd_u32(p, end);
    for (uint32_t i = 0; i < nv; ++i) {
        BPE_REQUIRE(p + 12 <= end, BPE_E_ARG, "truncated vocab blob");
        int64_t id;
        std::memcpy(&id, p, 8);
        p += 8;
        const uint32_t l = rd_u32(p, end);
        BPE_REQUIRE(p + l <= end, BPE_E_ARG, "truncated vocab blob");
        BPE_REQUIRE(id >= 0 && id < (1LL << 32), BPE_E_ARG, "vocab id outside [0, 2^32)");
        vid[tok(std::string((const char*)p, l))] = id;
        p += l;
    }
    // specials: dedupe (first occurrence), longest first; missing ones get ids len(vocab), ...
    for (const auto& s : sp_in) {
        BPE_REQUIRE(!s.empty(), BPE_E_ARG, "empty special token is not supported");
        if (std::find(T.specials.begin(), T.specials.end(), s) == T.specials.end()) T.specials.push_back(s);
    }
    std::stable_sort(T.specials.begin(), T.specials.end(),
                     [](const std::string& x, const std::string& y) { return x.size() > y.size(); });
    int64_t next_id = (int64_t)nv;
    for (const auto& s : T.specials) {
        const uint32_t t = tok(s);
        if (vid[t] < 0) vid[t] = next_id++;
        T.special_vid.push_back(vid[t]);
    }
    // merges: rank = index, later duplicates overwrite (tokenizer.py:115)
    std::unordered_map<unsigned long long, std::pair<uint32_t, uint32_t>> rank;
    p = mb;
    end = mb + mn;
    const uint32_t nm = rd_u32(p, end);
    for (uint32_t i = 0; i < nm; ++i) {
        const uint32_t la = rd_u32(p, end);
        BPE_REQUIRE(p + la <= end, BPE_E_ARG, "truncated merges blob");
        std::string a((const char*)p, la);
        p += la;
        const uint32_t lb = rd_u32(p, end);
        BPE_REQUIRE(p + lb <= end, BPE_E_ARG, "truncated merges blob");
        std::string b((const char*)p, lb);
        p += lb;
        const uint32_t ta = tok(a), tb = tok(b), tp = tok(a + b);
        rank[((unsigned long long)ta << 32) | tb] = {i, tp};
    }
    std::vector<uint32_t> b2t(256);
    for (int b = 0; b < 256; ++b) b2t[b] = tok(std::string(1, (char)b));

    // device tables
    T.pm_cap = next_pow2(std::max<size_t>(64, rank.size() * 2 + 1));
    std::vector<unsigned long long> hk(T.pm_cap, 0);
    std::vector<uint2> hv(T.pm_cap);
    for (const auto& kv : rank) {
        const unsigned long long key = kv.first + 1ULL;
        size_t s = mix64(key) & (T.pm_cap - 1);
        while (hk[s]) s = (s + 1) & (T.pm_cap - 1);
        hk[s] = key;
        hv[s] = make_uint2(kv.second.first, kv.second.second);
    }
    BPE_HIP(hipStreamCreateWithFlags(&T.stream, hipStreamNonBlocking));
    auto up = [&](auto& buf, const auto& vec) {
        buf.alloc(std::max<size_t>(vec.size(), 1));
        if (!vec.empty())
            BPE_HIP(hipMemcpyAsync(buf.p, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice, T.stream));
    };
    up(T.pm_key, hk);
    up(T.pm_val, hv);
    up(T.tok2vid, vid);
    up(T.byte2tok, b2t);
    std::string spb;
    std::vector<uint32_t> spo, spl;
    std::vector<unsigned> fm(8, 0);
    for (const auto& s : T.specials) {
        spo.push_back((uint32_t)spb.size());
        spl.push_back((uint32_t)s.size());
        spb += s;
        const unsigned char c = (unsigned char)s[0];
        fm[c >> 5] |= 1u << (c & 31);
    }
    std::vector<uint8_t> spbv(spb.begin(), spb.end());
    up(T.sp_bytes, spbv);
    up(T.sp_off, spo);
    up(T.sp_len, spl);
    up(T.sp_vid, T.special_vid);
    up(T.first_mask, fm);
    BPE_HIP(hipStreamSynchronize(T.stream));
    build_dictionary(T, intern, vid, b2t);
}

// encode d_text[0..n) into d_out; returns the id count.  `cuts` (sorted byte offsets) make the
// result that of separate encode() calls on the pieces between them, concatenated: a cut ends
// every segment, and a special token may not straddle one (encode.py's 1 M-character chunks,
// encode_iterable's 2 MiB batches).
template <class OutT>
size_t encode_device(bpe_tokenizer& T, const uint8_t* d_text, size_t n, OutT* d_out,
                     hipStream_t s, const std::vector<unsigned long long>& cuts_in = {}) {
    if (n == 0) return 0;
    std::vector<unsigned long long> cuts;
    for (unsigned long long c : cuts_in)
        if (c > 0 && c < n && (cuts.empty() || c > cuts.back())) cuts.push_back(c);
    EncTables E = T.tables();
    // 1. segments: every special match (k_find_specials), sorted on the device by (position,
    // index) -- by position, longest first (T.specials is longest first) -- then built into the
    // segment table on the device (k_sp_*), or left to right here when matches overlap
    auto& S = T.sc;
    DevBuf<Seg>& d_segs = S.segs;
    int nseg = 0;
    bool on_device = false;
    std::vector<unsigned long long> keys;
    if (!T.specials.empty()) {
        BPE_REQUIRE(T.specials.size() < (1u << kSpShift) && (n >> (64 - kSpShift)) == 0, BPE_E_LIMIT,
                    "too many special tokens or too long a text");
        unsigned long long cap = std::max<unsigned long long>(1024, n / 64);
        S.status.reserve(1);
        unsigned cnt32 = 0;
        for (;;) {
            S.sp_key.reserve(cap);
            BPE_HIP(hipMemsetAsync(S.status.p, 0, 4, s));
            hipLaunchKernelGGL(k_find_specials, dim3(std::min<unsigned>(grid_for((n + 15) / 16 + 1, 256), 4096)), dim3(256), 0, s, d_text, n, E,
                               T.first_mask.p, S.sp_key.p, S.status.p, cap);
            BPE_HIP(hipGetLastError());
            to_host(&cnt32, S.status.p, 4, s);
            if (cnt32 <= cap) break;
            cap = cnt32;
        }
        if (cnt32) {
            S.sp_sorted.reserve(cnt32);
            unsigned bits = kSpShift;
            while (bits < 64 && (n >> (bits - kSpShift)) != 0) ++bits;
            radix_sort_keys(S.sp_key.p, S.sp_sorted.p, cnt32, bits, s, &S.tmp);
            const size_t nc = cuts.size();
            S.cuts.reserve(std::max<size_t>(nc, 1));
            if (nc) to_device(S.cuts.p, cuts.data(), nc * 8, s);
            // the matches no cut splits, in order (into sp_key)
            S.sp_flag.reserve(cnt32);
            S.sp_off.reserve(2);
            hipLaunchKernelGGL(k_sp_eligible, dim3(grid_for(cnt32, 256)), dim3(256), 0, s, S.sp_sorted.p,
                               (size_t)cnt32, E.sp_len, S.cuts.p, nc, S.sp_flag.p);
            select_flagged(S.sp_sorted.p, S.sp_flag.p, S.sp_key.p, S.sp_off.p, cnt32, s);
            unsigned long long me = 0;
            to_host(&me, S.sp_off.p, 8, s);
            // segments per kept special (and the tail), their offsets, overlap check
            S.sp_cnt.reserve(me + 1);
            S.sp_off.reserve(me + 1);
            BPE_HIP(hipMemsetAsync(S.status.p, 0, 4, s));
            hipLaunchKernelGGL(k_sp_count, dim3(grid_for(me + 1, 256)), dim3(256), 0, s, S.sp_key.p, (size_t)me,
                               E.sp_len, S.cuts.p, nc, (unsigned long long)n, S.sp_cnt.p, S.status.p);
            exclusive_sum(S.sp_cnt.p, S.sp_off.p, (size_t)me + 1, s, &S.tmp);
            unsigned conflict = 0;
            unsigned long long last[2];
            to_host(&conflict, S.status.p, 4, s);
            to_host(&last[0], S.sp_off.p + me, 8, s);
            to_host(&last[1], S.sp_cnt.p + me, 8, s);
            if (!conflict) {
                const unsigned long long total = last[0] + last[1];
                BPE_REQUIRE(total < (1ull << 31), BPE_E_LIMIT, "too many segments (special tokens and pieces)");
                nseg = (int)total;
                d_segs.reserve(std::max(nseg, 1));
                hipLaunchKernelGGL(k_sp_emit, dim3(grid_for(me + 1, 256)), dim3(256), 0, s, S.sp_key.p, (size_t)me,
                                   E.sp_len, S.cuts.p, nc, (unsigned long long)n, S.sp_off.p, d_segs.p);
                BPE_HIP(hipGetLastError());
                on_device = true;
            } else {
                keys.resize(cnt32);
                to_host(keys.data(), S.sp_sorted.p, (size_t)cnt32 * 8, s);
            }
        }
    }
    if (!on_device) {   // leftmost, non-overlapping (re.split), cut by the pieces
        std::vector<Seg> segs;
        unsigned long long cur = 0;
        size_t ci = 0;
        auto cut_until = [&](unsigned long long upto) {   // normal segments ended by cuts <= upto
            for (; ci < cuts.size() && cuts[ci] <= upto; ++ci) {
                if (cuts[ci] > cur) segs.push_back(Seg{cur, cuts[ci], -1, 0});
                cur = std::max(cur, cuts[ci]);
            }
        };
        for (const unsigned long long key : keys) {
            const unsigned long long p0 = key >> kSpShift;
            const int sk = (int)(key & ((1u << kSpShift) - 1));
            if (p0 < cur) continue;
            const unsigned long long e = p0 + T.specials[sk].size();
            cut_until(p0);
            if (ci < cuts.size() && cuts[ci] < e) continue;   // straddles a cut: a shorter one at p0 may fit
            if (p0 > cur) segs.push_back(Seg{cur, p0, -1, 0});
            segs.push_back(Seg{p0, e, sk, 0});
            cur = e;
        }
        cut_until(n);
        if (cur < n) segs.push_back(Seg{cur, n, -1, 0});
        BPE_REQUIRE(segs.size() < (1ull << 31), BPE_E_LIMIT, "too many segments (special tokens and pieces)");
        nseg = (int)segs.size();
        d_segs.reserve(std::max(nseg, 1));
        to_device(d_segs.p, segs.data(), nseg * sizeof(Seg), s);
    }

    // 2. one staged pass: unique pre-tokens into the word table, one record per pre-token, each
    // chunk's records one dense run
    const size_t n_chunks = (n + kChunk - 1) / kChunk;
    BPE_REQUIRE(n_chunks < (1ull << 32), BPE_E_LIMIT, "text too long for one encode");
    const bool aligned = (reinterpret_cast<uintptr_t>(d_text) & 15u) == 0;
    auto kern = aligned ? k_enc_scan4<true> : k_enc_scan4<false>;
    int per_cu = 0, dev = 0, n_cu = 0;
    BPE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, kStage));
    BPE_HIP(hipGetDevice(&dev));
    BPE_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    unsigned sgrid = (unsigned)std::min<size_t>(n_chunks, (size_t)std::max(1, per_cu) * std::max(1, n_cu));
    if (const char* e = std::getenv("BPE355_STREAM_WG"))   // test knob (see count_words)
        sgrid = std::max(1u, std::min(sgrid, (unsigned)std::atoi(e)));
    // first guesses: small texts have many more unique words per byte than large corpora; natural
    // text has ~0.15 pre-tokens per byte (at most one per byte: the retry's size)
    // word table: distinct words grow sublinearly with the text (~1.3 M in 64 MB and ~7.5 M in
    // 11.9 GB of the OWT-like bench corpus, about n^0.35); 2.5 x that estimate keeps the load under
    // ~0.4, and a table that fills past 1/2 anyway stops the resolve and is retried 4 x larger
    const double est = 1.32e6 * std::pow(std::max(1.0, (double)n / (double)(1u << 26)), 0.35);
    size_t cap = next_pow2(std::max<size_t>(1 << 16, n < (1u << 26) ? n / 16 : (size_t)(2.5 * est)));
    if (const char* e = std::getenv("BPE355_ENC_TABLE_SLOTS"))   // A/B knob: the first table's slots
        cap = next_pow2(std::max<size_t>(1 << 16, std::strtoull(e, nullptr, 10)));
    unsigned long long rec_cap = n < (1u << 26) ? n + 64 : n / 4 + (1u << 20);
    // records are reserved a region per workgroup at a time: a region holds any chunk, and the
    // regions left part-used (the last of every workgroup, a chunk-sized tail of the others) are
    // slack the buffer carries
    const unsigned long long rec_region =
        std::min<unsigned long long>(1u << 18, std::max<unsigned long long>(kChunk, next_pow2(rec_cap / sgrid / 8)));
    const unsigned long long rec_slack = (unsigned long long)sgrid * rec_region;
    rec_cap += rec_slack + rec_cap / rec_region * kChunk;
    if (const char* e = std::getenv("BPE355_ENC_REC_CAP"))   // test knob: force the record retry
        rec_cap = std::max<unsigned long long>(1, std::strtoull(e, nullptr, 10));
    const unsigned long long rec_cap_max = n + n / 8 + rec_slack + 64;   // one record per byte
    // pending entries: ~0.07 per byte at the bench corpus (the LDS cache's misses); a block per
    // workgroup at least twice over; when the pool is spent the scan resolves words itself
    unsigned long long pend_cap = std::max<unsigned long long>(n / 8, 2ull * sgrid * kPendBlock);
    if (const char* e = std::getenv("BPE355_ENC_PEND_CAP"))   // test knob: a small pool (0: none)
        pend_cap = std::strtoull(e, nullptr, 10);
    pend_cap = std::min<unsigned long long>(pend_cap, (unsigned long long)kRecPendMax + 1 - kPendBlock);
    const unsigned pend_blocks = (unsigned)(pend_cap / kPendBlock);
    DevBuf<unsigned long long>&kv = S.kv, &pos = S.pos;
    DevBuf<unsigned long long>&rec_base = S.rec_base, &rec_fill = S.rec_fill, &fill = S.fill;
    DevBuf<uint32_t>& rec_n = S.rec_n;
    DevBuf<unsigned>& status = S.status;
    rec_base.reserve(n_chunks);
    rec_n.reserve(n_chunks);
    rec_fill.reserve(1);
    fill.reserve(1);
    status.reserve(1);
    S.pend.reserve(std::max<unsigned long long>((unsigned long long)pend_blocks * kPendBlock, 1));
    S.block_used.reserve(std::max(pend_blocks, 1u));
    S.pend_nblk.reserve(1);
    const EncDict D = T.dict();
    const bool tracing = std::getenv("BPE355_TRACE") != nullptr;
    if (tracing) S.rstats.reserve(3);
    unsigned long long pend_entries = 0;   // blocks handed out x kPendBlock (the last attempt's)
    BPE_REQUIRE(T.dict_slots < kRecPayload29 / 2, BPE_E_LIMIT, "vocab too large for the encoder's dictionary");
    for (int attempt = 0;; ++attempt) {
        BPE_REQUIRE(cap + T.dict_slots <= (size_t)kRecPayload29, BPE_E_LIMIT, "too many distinct words for one encode");
        kv.reserve(2 * cap);
        pos.reserve(cap);
        T.recs_cache.reserve(rec_cap);
        BPE_HIP(hipMemsetAsync(kv.p, 0, 2 * cap * sizeof(unsigned long long), s));
        BPE_HIP(hipMemsetAsync(status.p, 0, 4, s));
        BPE_HIP(hipMemsetAsync(fill.p, 0, 8, s));
        BPE_HIP(hipMemsetAsync(rec_fill.p, 0, 8, s));
        BPE_HIP(hipMemsetAsync(S.pend_nblk.p, 0, 4, s));
        ScanArgs A{d_text, n, n_chunks, d_segs.p, nseg, std::getenv("BPE355_NOCACHE") ? 0 : 1, kv.p, pos.p,
                   cap - 1, (unsigned long long)(cap / 2), fill.p, T.recs_cache.p, rec_cap, rec_region, rec_fill.p,
                   rec_base.p, rec_n.p, pend_blocks ? S.pend.p : nullptr, pend_blocks, S.pend_nblk.p,
                   S.block_used.p, status.p};
        hipLaunchKernelGGL(kern, dim3(sgrid), dim3(256), kStage, s, A, D);
        BPE_HIP(hipGetLastError());
        unsigned nblk = 0;
        to_host(&nblk, S.pend_nblk.p, 4, s);
        nblk = std::min(nblk, pend_blocks);
        pend_entries = (unsigned long long)nblk * kPendBlock;
        if (tracing) BPE_HIP(hipMemsetAsync(S.rstats.p, 0, 3 * sizeof(unsigned long long), s));
        if (nblk) {   // the pending words, resolved in place
            int r_cu = 0;
            BPE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&r_cu, k_enc_resolve, 256, 0));
            const unsigned long long ne = (unsigned long long)nblk * kPendBlock;
            const unsigned rgrid = (unsigned)std::min<unsigned long long>(ceil_div(ne, 256),
                                                                         (unsigned long long)std::max(1, r_cu) * std::max(1, n_cu) * 8);
            ResolveArgs RA{d_text, n, S.pend.p, S.block_used.p, ne, kv.p, pos.p, cap - 1, (unsigned long long)(cap / 2),
                           fill.p, status.p, tracing ? S.rstats.p : nullptr};
            // the LDS-cached resolve (default: 195 vs 198 ms at the bench corpus, r04h); the knob's
            // 0 runs the uncached one
            const char* rc_env = std::getenv("BPE355_ENC_RESOLVE_CACHE");
            if (!(rc_env && rc_env[0] == '0')) {
                int c_cu = 0;
                BPE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&c_cu, k_enc_resolve_c, 256, 0));
                const unsigned cgrid = std::min<unsigned>(nblk, (unsigned)(std::max(1, c_cu) * std::max(1, n_cu)));
                hipLaunchKernelGGL(k_enc_resolve_c, dim3(cgrid), dim3(256), 0, s, RA, D, nblk);
            } else {
                hipLaunchKernelGGL(k_enc_resolve, dim3(rgrid), dim3(256), 0, s, RA, D);
            }
            BPE_HIP(hipGetLastError());
        }
        unsigned st = 0;
        to_host(&st, status.p, 4, s);
        if (st & 2u) throw Error{BPE_E_LIMIT, "a pre-token is 8 MiB or longer"};
        BPE_REQUIRE(!(st & 16u), BPE_E_HIP, "internal error: encode scan found an empty pre-token");
        if (st & 1u) {
            BPE_REQUIRE(attempt < 8, BPE_E_NOMEM, "word table overflow");
            cap *= 4;
            continue;
        }
        if (st & 256u) {   // more pre-tokens than guessed: one per byte at most
            BPE_REQUIRE(attempt < 8, BPE_E_HIP, "internal error: encode records overflow (retries)");
            BPE_REQUIRE(rec_cap < rec_cap_max, BPE_E_HIP, "internal error: encode records overflow");
            rec_cap = rec_cap_max;
            continue;
        }
        break;
    }
    DevBuf<uint32_t>&w_slot = S.w_slot, &w_len = S.w_len;
    DevBuf<unsigned long long>& w_off = S.w_off;
    DevBuf<unsigned>& d_nw = S.d_nw;
    w_slot.reserve(cap);
    w_off.reserve(cap);
    w_len.reserve(cap);
    d_nw.reserve(1);
    BPE_HIP(hipMemsetAsync(d_nw.p, 0, 4, s));
    hipLaunchKernelGGL(k_collect, dim3(ceil_div(cap, 256 * kCollectPer)), dim3(256), 0, s, kv.p, pos.p, cap, w_slot.p,
                       w_off.p, w_len.p, d_nw.p);
    unsigned nw = 0;
    to_host(&nw, d_nw.p, 4, s);
    if (tracing) {
        unsigned long long nrec = 0, rs[3];
        to_host(&nrec, rec_fill.p, 8, s);
        to_host(rs, S.rstats.p, sizeof rs, s);
        std::fprintf(stderr, "[bpe355 encode] resolve: %llu LDS-cache hits, %llu dictionary words, %llu table words\n",
                     rs[0], rs[1], rs[2]);
        std::vector<uint32_t> used(pend_entries / kPendBlock);
        if (!used.empty()) to_host(used.data(), S.block_used.p, used.size() * 4, s);
        unsigned long long npend = 0;
        for (uint32_t u : used) npend += u;
        std::fprintf(stderr, "[bpe355 encode] %zu bytes: %llu record slots reserved, %llu pending (%zu blocks), %u table words "
                     "(%zu slots), dictionary %zu words\n", n, nrec, npend, used.size(), nw, cap, T.dict_words);
    }

    // 3. encode each word of the table once
    DevBuf<unsigned long long>&len64 = S.len64, &idoff = S.idoff;
    len64.reserve(std::max(nw, 1u));
    idoff.reserve(std::max(nw, 1u) + 1);
    DevBuf<unsigned long long>& slot_info = S.slot_info;   // every slot a record names is a word's slot
    slot_info.reserve(cap);
    BPE_HIP(hipMemsetAsync(slot_info.p, 0, cap * sizeof(unsigned long long), s));
    unsigned long long pool_n = 0;
    if (nw) {
        hipLaunchKernelGGL(k_word_len64, dim3(ceil_div(nw, 256)), dim3(256), 0, s, w_len.p, nw, len64.p);
        exclusive_sum(len64.p, idoff.p, nw, s, &S.tmp);
        unsigned long long last[2];
        to_host(&last[0], idoff.p + nw - 1, 8, s);
        to_host(&last[1], len64.p + nw - 1, 8, s);
        pool_n = last[0] + last[1];
    }
    BPE_REQUIRE(pool_n < kDictPool, BPE_E_LIMIT, "too many distinct words for one encode");
    DevBuf<uint32_t>& pool = S.pool;
    pool.reserve(std::max<unsigned long long>(pool_n, 1));
    BPE_HIP(hipMemsetAsync(status.p, 0, 4, s));
    if (nw) {
        hipLaunchKernelGGL(k_encode_words, dim3(ceil_div(nw, 256)), dim3(256), 0, s, d_text, E, w_off.p,
                           w_len.p, idoff.p, w_slot.p, nw, pool.p, slot_info.p, status.p, n);
        BPE_HIP(hipGetLastError());
    }
    // A/B knob BPE355_ENC_FINALIZE: 0 the emit reads the resolved records instead, 2 the emit's
    // count pass resolves them and stores the infos for the write pass
    const char* fin_env = std::getenv("BPE355_ENC_FINALIZE");
    const int fin_mode = fin_env ? std::atoi(fin_env) : 1;
    const bool finalize = pend_entries && fin_mode == 1;
    const bool writeback = pend_entries && fin_mode == 2;
    if (finalize) {   // pending entries: record -> ids' info
        int f_cu = 0;
        BPE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&f_cu, k_enc_finalize, 256, 0));
        const unsigned fgrid = (unsigned)std::min<unsigned long long>(ceil_div(pend_entries, 256),
                                                                     (unsigned long long)std::max(1, f_cu) * std::max(1, n_cu) * 8);
        hipLaunchKernelGGL(k_enc_finalize, dim3(fgrid), dim3(256), 0, s, S.pend.p, S.block_used.p, pend_entries,
                           slot_info.p, cap, D, T.dict_slots, status.p);
        BPE_HIP(hipGetLastError());
    }
    // 4. ids: the chunks' id counts, their exclusive scan, then the write pass
    DevBuf<unsigned long long>&ctot = S.ctot, &coff = S.coff;
    const size_t n_parts = n_chunks * kEmitParts;
    ctot.reserve(n_parts);
    coff.reserve(n_parts);
    EmitArgs EA{T.recs_cache.p, rec_base.p, rec_n.p, n_chunks, slot_info.p, pool.p, cap, D, T.dict_slots,
                S.pend.p, finalize ? 1 : 0, writeback ? 1 : 0, E.sp_vid, ctot.p, coff.p, status.p};
    {
        auto ck = k_enc_emit<OutT, true>;
        int c_cu = 0;
        BPE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&c_cu, ck, 256, 0));
        const unsigned cgrid = (unsigned)std::min<size_t>(n_parts, (size_t)std::max(1, c_cu) * std::max(1, n_cu) * 2);
        hipLaunchKernelGGL(ck, dim3(cgrid), dim3(256), 0, s, EA, d_out);
        BPE_HIP(hipGetLastError());
    }
    exclusive_sum(ctot.p, coff.p, n_parts, s, &S.tmp);
    if (writeback) EA.finalized = 1;   // every pending entry holds its info now
    {
        auto wk = k_enc_emit<OutT, false>;
        int w_cu = 0;
        BPE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&w_cu, wk, 256, 0));
        const unsigned wgrid = (unsigned)std::min<size_t>(n_parts, (size_t)std::max(1, w_cu) * std::max(1, n_cu) * 2);
        hipLaunchKernelGGL(wk, dim3(wgrid), dim3(256), 0, s, EA, d_out);
        BPE_HIP(hipGetLastError());
    }
    unsigned long long last[2] = {0, 0};
    unsigned st = 0;
    to_host(&last[0], coff.p + n_parts - 1, 8, s);
    to_host(&last[1], ctot.p + n_parts - 1, 8, s);
    to_host(&st, status.p, 4, s);
    if (st & 4u) throw Error{BPE_E_KEY, "a merged token is not in the vocab"};
    BPE_REQUIRE(!(st & 96u), BPE_E_HIP, "internal error: encode records inconsistent (status " +
                                          std::to_string(st) + ")");
    if (sizeof(OutT) == 2)
        BPE_REQUIRE(!(st & 128u), BPE_E_LIMIT, "a token id does not fit np.uint16 (vocab larger than 65536)");
    const size_t total = last[0] + last[1];
    BPE_REQUIRE(total <= n, BPE_E_HIP, "encode produced more ids than input bytes");
    BPE_HIP(hipStreamSynchronize(s));
    return total;
}

// ------------------------------------------------------------------ several devices
// The tokenizer for rank r on device dev: the handle itself for rank 0 on its own device, else a
// copy built from the same inputs (every rank owns its stream and record buffer, also when
// ranks share a device in tests).  The caller has made `dev` current.
bpe_tokenizer& tok_for_rank(bpe_tokenizer& T, int r, int dev) {
    if (r == 0 && dev == T.device) return T;
    const long long key = ((long long)r << 8) | dev;
    std::lock_guard<std::mutex> g(T.copies_m);
    for (auto& c : T.copies)
        if (c.first == key) return *c.second;
    auto U = std::make_unique<bpe_tokenizer>();
    build_tokenizer(*U, reinterpret_cast<const uint8_t*>(T.vblob.data()), T.vblob.size(),
                    reinterpret_cast<const uint8_t*>(T.mblob.data()), T.mblob.size(), T.sp_in);
    U->device = dev;
    T.copies.emplace_back(key, std::move(U));
    return *T.copies.back().second;
}

// g + 1 cut points of text[0, n) for separate encodes whose ids concatenate to encode(text): safe
// split points (a U+0020 between ASCII non-space bytes: the pre-tokens on both sides are those
// of the whole, pretok.h) that no occurrence of any special token spans, so re.split's leftmost
// matches (tokenizer.py:63-66) are those of the whole text too.  A slab with no such point is
// empty (its neighbour takes the text).
std::vector<size_t> encode_cuts(const uint8_t* t, size_t n, int g, const std::vector<std::string>& sp) {
    std::vector<size_t> cut{0};
    for (int r = 1; r < g; ++r) {
        size_t p = n / (size_t)g * (size_t)r;
        for (;;) {
            p = p >= 1 ? bpe_safe_split(t, n, p) : 0;
            if (p == 0 || p <= cut.back()) { p = cut.back(); break; }
            bool spans = false;
            for (const auto& x : sp) {
                const size_t L = x.size();
                for (size_t q = p + 1 > L ? p + 1 - L : 0; q < p && q + L <= n && !spans; ++q)
                    spans = std::memcmp(t + q, x.data(), L) == 0;
                if (spans) break;
            }
            if (!spans) break;
            --p;   // a special spans it: look further back
        }
        cut.push_back(p);
    }
    cut.push_back(n);
    return cut;
}

size_t encode_gpus(bpe_tokenizer& T, const uint8_t* utf8, size_t n, uint32_t* ids_out, int n_gpus) {
    int cur = 0;
    BPE_HIP(hipGetDevice(&cur));
    const std::vector<int> dev = pick_devices(n_gpus);
    const int g = (int)dev.size();
    const std::vector<size_t> cut = encode_cuts(utf8, n, g, T.specials);
    std::vector<std::vector<uint32_t>> ids(g);
    std::vector<std::exception_ptr> errs(g);
    auto work = [&](int r) {
        try {
            BPE_HIP(hipSetDevice(dev[r]));
            const size_t len = cut[r + 1] - cut[r];
            if (len == 0) return;
            bpe_tokenizer& U = tok_for_rank(T, r, dev[r]);
            DevBuf<uint8_t> d_text(len);
            DevBuf<uint32_t> d_out(len);
            BPE_HIP(hipMemcpyAsync(d_text.p, utf8 + cut[r], len, hipMemcpyHostToDevice, U.stream));
            const size_t m = encode_device(U, d_text.p, len, d_out.p, U.stream);
            ids[r].resize(m);
            if (m) BPE_HIP(hipMemcpyAsync(ids[r].data(), d_out.p, m * 4, hipMemcpyDeviceToHost, U.stream));
            BPE_HIP(hipStreamSynchronize(U.stream));
        } catch (...) {
            errs[r] = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    for (int r = 1; r < g; ++r) th.emplace_back(work, r);
    work(0);
    for (auto& x : th) x.join();
    (void)hipSetDevice(cur);
    for (auto& e : errs)   // the earliest slab's error: the one encode(text) would raise first
        if (e) std::rethrow_exception(e);
    size_t m = 0;
    for (int r = 0; r < g; ++r) {
        if (!ids[r].empty()) std::memcpy(ids_out + m, ids[r].data(), ids[r].size() * 4);
        m += ids[r].size();
    }
    return m;
}

template <class F>
int guarded_enc(F&& f) {
    try {
        f();
        set_error(0, "");
        return BPE_OK;
    } catch (const Error& e) {
        set_error(e.code, e.msg);
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error(BPE_E_NOMEM, "host allocation failed");
        return BPE_E_NOMEM;
    }
}

// ------------------------------------------------------------------ file -> uint16 ids, overlapped
// encode.py:31-37 for a regular file.  A reader thread streams the file into HBM in kReadSlab
// slabs; as they land, the main thread validates the loaded prefix (strict UTF-8, exactly as one
// pass over the whole text), counts its characters to place the piece starts (every
// chars_per_piece-th character, f.read(K)), encodes the pieces that are complete and validated
// straight to uint16 in the tokenizer's kept buffer, and hands their ids to a copier thread that
// moves them into ids_out while the next region is read and encoded.  A text with a carriage
// return (universal newlines move every later piece start) is redone in one serial pass once
// it has been read.  phase_ms: busy time of the reader, of validation + counting, of the encodes
// and of the copier (they overlap).
constexpr size_t kReadSlab = 1ull << 30;        // a multiple of the counting block (64 KiB)
constexpr size_t kMaxRegion = 3ull << 30;       // bytes one encode takes at most
constexpr size_t kLastRegion = 256ull << 20;    // bytes of the last region (the copy tail)
constexpr size_t kMinRegion = 64ull << 20;      // bytes a region takes at least while the file arrives

size_t env_size(const char* name, size_t dflt) {   // test knobs: small slabs and regions
    const char* e = std::getenv(name);
    const long long v = e ? std::atoll(e) : 0;
    return v > 0 ? (size_t)v : dflt;
}

size_t encode_file_pipelined(bpe_tokenizer& T, const Source& src, size_t K, uint16_t* ids_out, size_t cap, int dev,
                             double* ph) {
    using clk = std::chrono::steady_clock;
    auto since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    auto& S = T.sc;
    const hipStream_t s = T.stream;
    const size_t n = src.size;
    if (n == 0) return 0;
    const auto t_call = clk::now();
    const size_t read_slab = std::max<size_t>(1, env_size("BPE355_READ_SLAB", kReadSlab) >> 16) << 16;
    const size_t max_region = env_size("BPE355_ENC_REGION", kMaxRegion);
    const size_t last_region = std::min(max_region, env_size("BPE355_ENC_LAST_REGION", kLastRegion));
    const size_t min_region = std::min(max_region, env_size("BPE355_ENC_MIN_REGION", kMinRegion));
    // per-region lines (range, ids, pieces, ms; then the call's clock in ms at: the slab seen, its
    // validation + counting done, the encode done) appended to the file BPE355_ENC_TRACE names,
    // and one line per slab read and per copy (start, end)
    const char* trace_path = std::getenv("BPE355_ENC_TRACE");
    FILE* const trace = trace_path ? std::fopen(trace_path, "a") : nullptr;
    struct Closer { FILE* f; ~Closer() { if (f) std::fclose(f); } } trace_closer{trace};
    S.text.reserve(n);
    S.ids16.reserve(n);   // ids <= bytes
    uint8_t* const text = S.text.p;

    // reader
    std::mutex m;
    std::condition_variable cv;
    size_t loaded = 0;
    bool read_done = false;
    std::atomic<bool> stop{false};   // an error downstream: read no further
    std::exception_ptr read_err;
    // reader and copier threads, each (measured at 11.9 GB, r04: 8 threads 492-508 ms per call,
    // 4 threads 1.96-2.0 s before the region encode got fast; r03, with a 430 ms encode phase: 4
    // threads 593-648 ms, 8: 713-749, 16: 810-858)
    const int io_n = (int)env_size("BPE355_ENC_IO_THREADS", 8);
    // host threads of each region's copy-out (BPE355_ENC_COPY_THREADS): 4 leave the host cores the
    // encoder's own thread needs while 8 readers run (r04zc, 11.9 GB: 4 threads 358-365 ms per warm
    // call, 8 376-451, 2 442-446)
    const int copy_n = (int)env_size("BPE355_ENC_COPY_THREADS", 4);
    // experiment knob: BPE355_ENC_OVERLAP=0 reads the whole file before the first encode
    const char* ov = std::getenv("BPE355_ENC_OVERLAP");
    const bool overlap_read = !(ov && ov[0] == '0');
    // test knob: the read fails once it reaches this byte offset (an EIO or a file truncated
    // while it is read)
    const size_t fail_at = env_size("BPE355_TEST_READ_FAIL_AT", 0);
    std::thread reader([&] {
        const auto t0 = clk::now();
        try {
            for (size_t off = 0; off < n && !stop.load(); off += read_slab) {
                const size_t len = std::min(read_slab, n - off);
                if (fail_at && off + len >= fail_at)
                    throw Error{BPE_E_IO, "read failed (injected by BPE355_TEST_READ_FAIL_AT)"};
                const double r0 = since(t_call);
                stage_to_device(src, off, len, text + off, dev, io_n);
                if (trace) {
                    std::lock_guard<std::mutex> g(m);
                    std::fprintf(trace, "read %zu %zu at %.1f %.1f\n", off, off + len, r0, since(t_call));
                }
                std::lock_guard<std::mutex> g(m);
                loaded = off + len;
                cv.notify_all();
            }
        } catch (...) {
            std::lock_guard<std::mutex> g(m);
            read_err = std::current_exception();
        }
        std::lock_guard<std::mutex> g(m);
        read_done = true;
        ph[0] = since(t0);
        cv.notify_all();
    });
    // copier: a queue of regions copied out in order by one thread (each copy fans out over io_n
    // threads), so the encoder never waits for one region's copy before it starts the next
    // (r04za timeline: waiting for the previous copy held the encoder 13-40 ms per region)
    std::mutex qm;
    std::condition_variable qcv;
    std::deque<std::pair<size_t, size_t>> cq;
    bool cq_closed = false;
    std::exception_ptr copy_err;
    std::thread copier([&] {
        for (;;) {
            std::pair<size_t, size_t> job;
            {
                std::unique_lock<std::mutex> g(qm);
                qcv.wait(g, [&] { return !cq.empty() || cq_closed; });
                if (cq.empty()) return;
                job = cq.front();
                cq.pop_front();
            }
            if (copy_err || stop.load()) continue;   // after an error: drain without copying
            const auto t0 = clk::now();
            try {
                device_to_host(reinterpret_cast<const uint8_t*>(S.ids16.p + job.first), 2 * job.second,
                               reinterpret_cast<uint8_t*>(ids_out + job.first), dev, copy_n);
            } catch (...) {
                copy_err = std::current_exception();
            }
            ph[3] += since(t0);
            if (trace) {
                std::lock_guard<std::mutex> g(m);
                std::fprintf(trace, "copy %zu ids at %.1f %.1f\n", job.second,
                             std::chrono::duration<double, std::milli>(t0 - t_call).count(), since(t_call));
            }
        }
    });
    auto copy_close = [&] {
        {
            std::lock_guard<std::mutex> g(qm);
            cq_closed = true;
        }
        qcv.notify_all();
        if (copier.joinable()) copier.join();
    };
    auto copy_wait = [&] {   // every queued copy done (then no more can be queued)
        copy_close();
        if (copy_err) std::rethrow_exception(copy_err);
    };
    auto copy_start = [&](size_t at, size_t cnt) {
        {
            std::lock_guard<std::mutex> g(qm);
            cq.emplace_back(at, cnt);
        }
        qcv.notify_one();
    };
    auto finish_threads = [&] {
        stop.store(true);
        {
            std::unique_lock<std::mutex> g(m);
            cv.wait(g, [&] { return read_done; });
        }
        if (reader.joinable()) reader.join();
        copy_close();
    };

    size_t k_done = 0;
    bool serial = false;   // a carriage return: redo in one pass
    try {
        ValidatePass V;
        V.begin(text, n, s);
        std::vector<uint64_t> starts;      // piece starts found so far (global offsets)
        size_t counted = 0, enc_done = 0, next_piece = 1;   // starts[0] == 0
        uint64_t chars = 0;
        size_t seen = 0;
        while (enc_done < n) {
            size_t L;
            {
                std::unique_lock<std::mutex> g(m);
                cv.wait(g, [&] { return (overlap_read && loaded > seen) || read_done; });
                if (read_err) std::rethrow_exception(read_err);
                L = loaded;
            }
            seen = L;
            const auto t1 = clk::now();
            const double t_seen = since(t_call);
            const size_t vend = V.prefix(L);
            const size_t cend = L == n ? n : L / 65536 * 65536;
            if (cend > counted) {
                chars += piece_starts_range(text + counted, cend - counted, K, chars, counted, s, starts, &S.piece);
                counted = cend;
            }
            unsigned long long err = 0;
            bool cr = false;
            V.finish(&err, &cr);
            ph[1] += since(t1);
            const double t_valid = since(t_call);
            if (err != ~0ULL)
                throw Error{BPE_E_UTF8, "'utf-8' codec can't decode byte at position " + std::to_string(err)};
            if (cr) { serial = true; break; }
            // encode the complete pieces inside the validated and counted prefix, at most
            // kMaxRegion at a time, each region ending at a piece start (or the end)
            const size_t ready = std::min(vend, counted);
            auto region_end = [&](size_t from) -> size_t {
                // once the whole text is in, the last region is kept short (at most last_region
                // bytes): its ids' copy is the one step nothing overlaps
                size_t span = max_region;
                if (ready == n) {
                    if (n - from <= last_region) return n;
                    span = std::min(max_region, n - from - last_region);
                }
                size_t lim = from;
                for (size_t i = next_piece; i < starts.size() && starts[i] <= std::min(ready, from + span); ++i)
                    lim = starts[i];
                if (lim == from && ready == n)   // a piece longer than kMaxRegion: whole
                    lim = next_piece < starts.size() ? starts[next_piece] : n;
                // while the file is still arriving, a short leftover (the piece cut by a slab end)
                // waits for the next slab instead of costing an encode call of its own
                if (ready < n && lim - from < min_region) return from;
                return lim;
            };
            for (size_t e_end = region_end(enc_done); e_end > enc_done; e_end = region_end(enc_done)) {
                std::vector<unsigned long long> cuts;
                for (; next_piece < starts.size() && starts[next_piece] < e_end; ++next_piece)
                    cuts.push_back(starts[next_piece] - enc_done);
                if (next_piece < starts.size() && starts[next_piece] == e_end) ++next_piece;
                const auto t2 = clk::now();
                const size_t kk = encode_device(T, text + enc_done, e_end - enc_done, S.ids16.p + k_done, s, cuts);
                const double ems = since(t2);
                ph[2] += ems;
                if (trace) {
                    std::lock_guard<std::mutex> g(m);
                    std::fprintf(trace, "region %zu %zu ids %zu pieces %zu ms %.1f loaded %zu at %.1f %.1f %.1f\n", enc_done,
                                 e_end, kk, cuts.size() + 1, ems, seen, t_seen, t_valid, since(t_call));
                    std::fflush(trace);
                }
                BPE_REQUIRE(k_done + kk <= cap, BPE_E_ARG, "ids_out holds " + std::to_string(cap) +
                                                              " ids, the file encodes to more");
                copy_start(k_done, kk);
                k_done += kk;
                enc_done = e_end;
            }
        }
        copy_wait();
    } catch (...) {
        finish_threads();
        throw;
    }
    if (serial) {   // the rest of the file first; on a read error both threads are joined first
        std::exception_ptr e;
        {
            std::unique_lock<std::mutex> g(m);
            cv.wait(g, [&] { return read_done; });
            e = read_err;
        }
        if (e) {
            finish_threads();
            std::rethrow_exception(e);
        }
    }
    finish_threads();
    if (copy_err) std::rethrow_exception(copy_err);
    if (!serial) return k_done;

    // universal newlines: one pass over the whole text, as read
    const auto t1 = clk::now();
    size_t mlen = 0;
    const uint8_t* t2 = prepare_text(text, n, S.text2, &mlen, s);
    const std::vector<uint64_t> starts = utf8_piece_starts(t2, mlen, K, s);
    ph[1] += since(t1);
    const auto te = clk::now();
    const std::vector<unsigned long long> cuts(starts.begin(), starts.end());
    const size_t kk = mlen ? encode_device(T, t2, mlen, S.ids16.p, s, cuts) : 0;
    ph[2] += since(te);
    BPE_REQUIRE(kk <= cap, BPE_E_ARG, "ids_out holds " + std::to_string(cap) + " ids, the file encodes to " +
                                         std::to_string(kk));
    const auto tc = clk::now();
    if (kk) device_to_host(reinterpret_cast<const uint8_t*>(S.ids16.p), 2 * kk, reinterpret_cast<uint8_t*>(ids_out),
                           dev, io_threads());
    ph[3] += since(tc);
    return kk;
}

}  // namespace
}  // namespace bpe

extern "C" {

int bpe_tok_create(const uint8_t* vocab_blob, size_t vocab_n, const uint8_t* merges_blob, size_t merges_n,
                   const char* const* specials, int n_specials, bpe_tokenizer** out) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(out && vocab_blob && merges_blob, BPE_E_ARG, "NULL argument");
        BPE_REQUIRE(n_specials >= 0 && (n_specials == 0 || specials), BPE_E_ARG, "bad specials");
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            throw bpe::Error{BPE_E_HIP, "no HIP device visible (libbpe355 needs an MI355X / gfx950 GPU)"};
        std::vector<std::string> sp;
        for (int i = 0; i < n_specials; ++i) {
            BPE_REQUIRE(specials[i], BPE_E_ARG, "null special");
            sp.emplace_back(specials[i]);
        }
        auto T = std::make_unique<bpe_tokenizer>();
        bpe::build_tokenizer(*T, vocab_blob, vocab_n, merges_blob, merges_n, sp);
        T->vblob.assign(reinterpret_cast<const char*>(vocab_blob), vocab_n);
        T->mblob.assign(reinterpret_cast<const char*>(merges_blob), merges_n);
        T->sp_in = sp;
        BPE_HIP(hipGetDevice(&T->device));
        *out = T.release();
    });
}

int64_t bpe_tok_special_id(const bpe_tokenizer* tok, int i) {
    if (!tok || i < 0 || i >= (int)tok->special_vid.size()) return -1;
    return tok->special_vid[i];
}

int bpe_tok_encode(bpe_tokenizer* tok, const uint8_t* utf8, size_t n, uint32_t* ids_out, size_t cap,
                   size_t* n_out) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(tok && n_out && (n == 0 || (utf8 && ids_out)), BPE_E_ARG, "NULL argument");
        BPE_REQUIRE(cap >= n, BPE_E_ARG, "ids_out capacity must be >= input bytes");
        *n_out = 0;
        if (n == 0) return;
        bpe::DevBuf<uint8_t> d_text(n);
        bpe::DevBuf<uint32_t> d_out(n);
        BPE_HIP(hipMemcpyAsync(d_text.p, utf8, n, hipMemcpyHostToDevice, tok->stream));
        const size_t m = bpe::encode_device(*tok, d_text.p, n, d_out.p, tok->stream);
        if (m) BPE_HIP(hipMemcpyAsync(ids_out, d_out.p, m * 4, hipMemcpyDeviceToHost, tok->stream));
        BPE_HIP(hipStreamSynchronize(tok->stream));
        *n_out = m;
    });
}

int bpe_tok_encode_device(bpe_tokenizer* tok, const uint8_t* d_utf8, size_t n, uint32_t* d_out,
                          size_t* n_out, void* hip_stream) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(tok && n_out && (n == 0 || (d_utf8 && d_out)), BPE_E_ARG, "NULL argument");
        hipStream_t s = hip_stream ? (hipStream_t)hip_stream : tok->stream;
        *n_out = bpe::encode_device(*tok, d_utf8, n, d_out, s);
    });
}

int bpe_tok_encode_chunks_device(bpe_tokenizer* tok, const uint8_t* d_utf8, size_t n, const uint64_t* starts,
                                 size_t n_starts, uint32_t* d_out, size_t* n_out, void* hip_stream) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(tok && n_out && (n == 0 || (d_utf8 && d_out)), BPE_E_ARG, "NULL argument");
        BPE_REQUIRE(n_starts == 0 || starts, BPE_E_ARG, "NULL starts");
        std::vector<unsigned long long> cuts(starts, starts + n_starts);
        for (size_t i = 1; i < cuts.size(); ++i)
            BPE_REQUIRE(cuts[i] >= cuts[i - 1], BPE_E_ARG, "chunk starts must be sorted");
        hipStream_t s = hip_stream ? (hipStream_t)hip_stream : tok->stream;
        *n_out = bpe::encode_device(*tok, d_utf8, n, d_out, s, cuts);
    });
}

int bpe_tok_encode_file_u16(bpe_tokenizer* tok, const char* path, size_t chars_per_piece, uint16_t* ids_out,
                            size_t cap, size_t* n_out, double* phase_ms) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(tok && path && n_out && chars_per_piece > 0, BPE_E_ARG, "NULL argument");
        *n_out = 0;
        double ph[4] = {0, 0, 0, 0};
        const bpe::Source src = bpe::Source::open_path(path);   // FileNotFoundError etc. before the GPU
        int dev = 0;
        BPE_HIP(hipGetDevice(&dev));
        const size_t k = bpe::encode_file_pipelined(*tok, src, chars_per_piece, ids_out, cap, dev, ph);
        *n_out = k;
        if (phase_ms) std::memcpy(phase_ms, ph, sizeof(ph));
    });
}

int bpe_tok_encode_chunks(bpe_tokenizer* tok, const uint8_t* utf8, size_t n, const uint64_t* starts,
                          size_t n_starts, uint32_t* ids_out, size_t cap, size_t* n_out) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(tok && n_out && (n == 0 || (utf8 && ids_out)), BPE_E_ARG, "NULL argument");
        BPE_REQUIRE(cap >= n, BPE_E_ARG, "ids_out capacity must be >= input bytes");
        BPE_REQUIRE(n_starts == 0 || starts, BPE_E_ARG, "NULL starts");
        *n_out = 0;
        if (n == 0) return;
        std::vector<unsigned long long> cuts(starts, starts + n_starts);
        for (size_t i = 1; i < cuts.size(); ++i)
            BPE_REQUIRE(cuts[i] >= cuts[i - 1], BPE_E_ARG, "chunk starts must be sorted");
        bpe::DevBuf<uint8_t> d_text(n);
        bpe::DevBuf<uint32_t> d_out(n);
        BPE_HIP(hipMemcpyAsync(d_text.p, utf8, n, hipMemcpyHostToDevice, tok->stream));
        const size_t m = bpe::encode_device(*tok, d_text.p, n, d_out.p, tok->stream, cuts);
        if (m) BPE_HIP(hipMemcpyAsync(ids_out, d_out.p, m * 4, hipMemcpyDeviceToHost, tok->stream));
        BPE_HIP(hipStreamSynchronize(tok->stream));
        *n_out = m;
    });
}

int bpe_tok_encode_gpus(bpe_tokenizer* tok, const uint8_t* utf8, size_t n, uint32_t* ids_out, size_t cap,
                        size_t* n_out, int n_gpus) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(tok && n_out && (n == 0 || (utf8 && ids_out)), BPE_E_ARG, "NULL argument");
        BPE_REQUIRE(cap >= n, BPE_E_ARG, "ids_out capacity must be >= input bytes");
        *n_out = 0;
        if (n == 0) return;
        *n_out = bpe::encode_gpus(*tok, utf8, n, ids_out, n_gpus);
    });
}

int bpe_tok_release_buffers(bpe_tokenizer* tok) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(tok, BPE_E_ARG, "NULL argument");
        BPE_HIP(hipStreamSynchronize(tok->stream));
        tok->recs_cache = bpe::DevBuf<uint32_t>();
        tok->sc = bpe_tokenizer::Scratch();
        std::lock_guard<std::mutex> g(tok->copies_m);
        tok->copies.clear();
    });
}

void bpe_tok_free(bpe_tokenizer* tok) { delete tok; }

}  // extern "C"
