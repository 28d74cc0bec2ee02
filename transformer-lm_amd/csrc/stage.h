// Shared by the word counter (text.hip) and the encoder (encode.hip): the global word table's
// entry format and the LDS staging of corpus chunks.
#pragma once

#include <cstddef>
#include <cstdint>

#include "bpe_common.h"
#include "pretok.h"

namespace bpe {

// ------------------------------------------------------------------ word counting
// Global table: open addressing over 16-byte entries {key, count} (one line per probe; the
// table stays small enough to live in the Infinity Cache -- 32-byte entries measured 1.9x
// slower).  Words of <= 7 bytes are stored INLINE: key = kInl | len << 56 | bytes, so a hit
// needs no read of the corpus, and the claimer records an occurrence in the cold `pos` array
// (read only after the kernel).  Longer words are keyed by len << 40 | (offset + 1) of their
// first occurrence and verified against the corpus.  Words of <= 16 bytes hash by their packed
// bytes, longer ones by FNV-1a: a word always takes the same path.
constexpr unsigned long long kOffMask = (1ULL << 40) - 1;
constexpr unsigned long long kInl = 1ULL << 63;
constexpr int kInlineKey = 7;        // longest word stored inline in the key
constexpr int kMaxProbe = 1024;     // at load <= 1/2 a longer chain means the table is full: regrow
constexpr int kInline = 16;          // words up to this length are packed into two u64
constexpr int kChunk = 16384;        // corpus bytes a workgroup scans per iteration
constexpr int kHalo = 1024;          // staged bytes past the chunk (tokens running over its end)
constexpr int kWin = kChunk + kHalo;
constexpr int kPadded = kWin + (kWin / 64) * 4;   // +4 B per 64 B: threads' spans hit distinct banks
constexpr int kVec = (kWin + 16 * 256 - 1) / (16 * 256);   // 16-B loads per thread per chunk
constexpr unsigned long long kBusy = 1ULL << 63;
// Longest pre-token the tables key: len << 40 must stay clear of bit 63 (kInl), so len < 2^23.
// A longer one fails the call with BPE_E_LIMIT (status bit 2), in training and in encoding.
constexpr unsigned long long kMaxPretok = 1ULL << 23;

// Two 64-bit multiplies (the earlier mix64(lo ^ mix64(hi ...)) took four, and on the count and
// encode scans, which hash every pre-token, those quarter-rate v_mul's were the largest VALU cost):
// hi and len folded in through one odd multiply, then a one-multiply finalizer whose xor-shifts
// bring every input bit into the low bits (the table slots) and the high ones (bins, cache sets).
// Checked against the old form on the bench corpus's 934 K distinct words: no full collisions,
// the same bin / cache-set spread and table probe length (tools/hash_quality.py,
// profiles/r05/j_hash_quality.json).
__host__ __device__ inline uint64_t short_hash(uint64_t lo, uint64_t hi, size_t len) {
    uint64_t z = lo ^ ((hi ^ (uint64_t)len) * 0x9E3779B97F4A7C15ULL);
    z ^= z >> 32;
    z *= 0xD6E8FEB86659FD93ULL;
    return z ^ (z >> 32);
}

// The staged window lives in dynamic LDS (kPadded bytes per workgroup), addressed directly:
// a generic pointer to it inside the accessor trips the gfx950 backend.
extern __shared__ __attribute__((aligned(16))) uint8_t g_stage[];

// the staged window, addressed by position relative to the chunk start (32-bit)
struct LdsText {
    __device__ __forceinline__ uint8_t operator[](uint32_t r) const { return g_stage[r + ((r >> 6) << 2)]; }
};
constexpr uint32_t kNotFound = 0xffffffffu;

template <class Src>
__device__ __forceinline__ void pack_word(const Src& t, size_t p, size_t len, uint64_t& lo, uint64_t& hi) {
    lo = 0;
    hi = 0;
    for (size_t i = 0; i < len; ++i) {
        const uint64_t b = t[p + i];
        if (i < 8) lo |= b << (8 * i);
        else hi |= b << (8 * (i - 8));
    }
}

// the word at q of s equals the one at p of t (len > kInline)
template <class Src>
__device__ __forceinline__ bool words_equal(const uint8_t* __restrict__ s, size_t q, const Src& t, size_t p, size_t len) {
    bool eq = true;
    for (size_t i = 0; i < len && eq; ++i) eq = s[q + i] == t[p + i];
    return eq;
}
__device__ __forceinline__ bool words_equal(const uint8_t* __restrict__ s, size_t q, const uint8_t* t, size_t p,
                                            size_t len) {
    return t == s ? bytes_equal(s, q, p, len) : words_equal<const uint8_t*>(s, q, t, p, len);
}

// Add `c` occurrences of a word (c = 0: find or insert only).  Returns its slot, or ~0 when
// the probe limit is hit (status bit 1); *inserted = whether this call created the key.
// wl/wh: the packed bytes (words <= 16 bytes); t/p: the word's bytes for longer ones.
template <class Src>
__device__ __forceinline__ size_t table_add(const uint8_t* __restrict__ s, const Src& t, size_t p, size_t len,
                                            uint64_t wl, uint64_t wh, uint64_t h, unsigned long long c,
                                            unsigned long long* __restrict__ kv,
                                            unsigned long long* __restrict__ pos, size_t mask,
                                            unsigned* __restrict__ status, bool* inserted) {
    *inserted = false;
    const bool inl = len <= (size_t)kInlineKey;
    if (len >= kMaxPretok) {   // its key would read as an inline word
        atomicOr(status, 2u);
        return ~(size_t)0;
    }
    const unsigned long long mine = inl ? kInl | ((unsigned long long)len << 56) | wl
                                        : ((unsigned long long)len << 40) | (p + 1);
    size_t slot = h & mask;
    for (int probe = 0; probe < kMaxProbe; ++probe) {
        unsigned long long k = kv[2 * slot];
        if (k == 0) {
            k = atomicCAS(&kv[2 * slot], 0ULL, mine);
            if (k == 0) {   // claimed
                if (inl) pos[slot] = p;
                if (c) atomicAdd(&kv[2 * slot + 1], c);
                *inserted = true;
                return slot;
            }
        }
        bool eq = false;
        if (inl) {
            eq = k == mine;
        } else if (!(k & kInl) && (k >> 40) == len) {
            const size_t q = (k & kOffMask) - 1;
            if (len <= (size_t)kInline) {
                uint64_t l2, h2;
                pack_word(s, q, len, l2, h2);
                eq = l2 == wl && h2 == wh;
            } else {
                eq = words_equal(s, q, t, p, len);
            }
        }
        if (eq) {
            if (c) atomicAdd(&kv[2 * slot + 1], c);
            return slot;
        }
        slot = (slot + 1) & mask;
    }
    atomicOr(status, 1u);
    return ~(size_t)0;
}

// ------------------------------------------------------------------ chunk staging
// A persistent workgroup stages [base, base + kWin) of the corpus in g_stage: every thread
// holds kVec 16-byte pieces in registers (fetched while the previous chunk is scanned), then
// stores them bank-spread (+4 B per 64 B).
template <bool kAligned>
__device__ __forceinline__ void stage_fetch(uint4 (&pre)[kVec], const uint8_t* __restrict__ s, size_t n,
                                            size_t base, int tid) {
#pragma unroll
    for (int v = 0; v < kVec; ++v) {
        const size_t off = ((size_t)v * 256 + tid) * 16;
        if (off >= (size_t)kWin) continue;
        const size_t g = base + off;
        if (kAligned && g + 16 <= n) {
            pre[v] = *reinterpret_cast<const uint4*>(s + g);
        } else {
            uint8_t tmp[16];
            for (int j = 0; j < 16; ++j) tmp[j] = g + j < n ? s[g + j] : 0;
            __builtin_memcpy(&pre[v], tmp, 16);
        }
    }
}
__device__ __forceinline__ void stage_store(const uint4 (&pre)[kVec], int tid) {
#pragma unroll
    for (int v = 0; v < kVec; ++v) {
        const size_t off = ((size_t)v * 256 + tid) * 16;
        if (off >= (size_t)kWin) continue;
        uint32_t* d = reinterpret_cast<uint32_t*>(g_stage + off + ((off >> 6) << 2));
        d[0] = pre[v].x; d[1] = pre[v].y; d[2] = pre[v].z; d[3] = pre[v].w;
    }
}


}  // namespace bpe
