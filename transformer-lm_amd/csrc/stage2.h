// Chunk staging for the byte-parallel scanners (count.hip, encode.hip): a persistent workgroup
// stages [base - kPre, base + kWin + kPost) of the text in LDS (unpadded), every thread turns one
// 64-byte block into a token-start mask (tokstart.h) read from the stage.
#pragma once

#include <cstddef>
#include <cstdint>

#include "pretok.h"
#include "stage.h"
#include "tokstart.h"

namespace bpe {
namespace {

// classes of the code points below U+0800 (every 2-byte character), 2 bits each, in LDS: the
// corpus's non-ASCII characters are mostly these; the rest go through the global tables
__shared__ uint32_t g_cls2[2048 / 16];

struct DevTab {
    __device__ static unsigned page(unsigned i) { return BPE_UC_PAGE[i]; }
    __device__ static unsigned bits(unsigned pg, unsigned i) { return BPE_UC_BITS[pg][i]; }
    __device__ static int cls(uint32_t cp) {
        return cp < 2048u ? (int)((g_cls2[cp >> 4] >> (2 * (cp & 15u))) & 3u) : uc_class<DevTab>(cp);
    }
};

__device__ __forceinline__ void load_cls2(int tid, int nthreads) {
    for (int i = tid; i < 2048 / 16; i += nthreads) {
        uint32_t x = 0;
        for (int k = 0; k < 16; ++k) x |= (uint32_t)uc_class<DevTab>((uint32_t)(16 * i + k)) << (2 * k);
        g_cls2[i] = x;
    }
}

// the stage as text positions relative to the chunk start (pretok.h's serial scanner)
struct StageText {
    __device__ __forceinline__ uint8_t operator[](uint32_t r) const;
};

constexpr int kPre = 16;                          // staged bytes before the chunk
constexpr int kPost = 16;                         // staged bytes after the halo
constexpr int kStage = kPre + kWin + kPost;       // 17 440
constexpr int kSVec = (kStage + 4095) / 4096;     // 16-B loads per thread per chunk
constexpr int kWords = kChunk / 64;               // mask words of the chunk

__device__ __forceinline__ uint8_t StageText::operator[](uint32_t r) const { return g_stage[kPre + r]; }

// 16 bytes at g that straddle the text start or end (the first and last chunks only)
__device__ __noinline__ uint4 fetch_edge(const uint8_t* __restrict__ s, size_t n, long long g) {
    uint32_t d[4];
    for (int k = 0; k < 4; ++k) {
        uint32_t x = 0;
        for (int j = 0; j < 4; ++j) {
            const long long q = g + 4 * k + j;
            const uint32_t b = q < 0 ? (uint32_t)'\n' : ((size_t)q < n ? (uint32_t)s[q] : 0u);
            x |= b << (8 * j);
        }
        d[k] = x;
    }
    return make_uint4(d[0], d[1], d[2], d[3]);
}

// 16 bytes at p (any alignment) from the two aligned 16-byte words that cover them: every unit
// of a window shares p's misalignment, so the word select is uniform; each aligned word is a
// neighbour's too (an unaligned text, e.g. an encode region starting at a piece start, loads at
// full width instead of byte by byte).  Both words lie in 16-byte units that hold a byte of
// [p, p + 16), so within the allocation.
__device__ __forceinline__ uint4 fetch_shifted(const uint8_t* p) {
    const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
    const unsigned d = (unsigned)(addr & 15);
    const uint4* a = reinterpret_cast<const uint4*>(addr - d);
    const uint4 q0 = a[0];
    if (d == 0) return q0;
    const uint4 q1 = a[1];
    const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    const unsigned k = d >> 2, sh = (d & 3) * 8;
    uint32_t o[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) o[i] = k == 0 ? w[i] : k == 1 ? w[i + 1] : k == 2 ? w[i + 2] : w[i + 3];
    if (sh == 0) return make_uint4(o[0], o[1], o[2], o[3]);
    return make_uint4((o[0] >> sh) | (o[1] << (32 - sh)), (o[1] >> sh) | (o[2] << (32 - sh)),
                      (o[2] >> sh) | (o[3] << (32 - sh)), (o[3] >> sh) | (o[4] << (32 - sh)));
}

// the chunk window [base - kPre, base + kWin + kPost) of s[0, n): bytes before the text read '\n'
// (tokstart.h), bytes past n read 0 (and are flagged past the end by vhi)
template <bool kAligned>
__device__ __forceinline__ void fetch2(uint4 (&pre)[kSVec], const uint8_t* __restrict__ s, size_t n, size_t base,
                                       int tid) {
#pragma unroll
    for (int v = 0; v < kSVec; ++v) {
        const int off = (v * 256 + tid) * 16;
        if (off >= kStage) continue;
        const long long g = (long long)base - kPre + off;
        if (kAligned && g >= 0 && (size_t)g + 16 <= n) pre[v] = *reinterpret_cast<const uint4*>(s + g);
        else if (!kAligned && g >= 0 && (size_t)g + 16 <= n) pre[v] = fetch_shifted(s + g);
        else pre[v] = fetch_edge(s, n, g);
    }
}
__device__ __forceinline__ void store2(const uint4 (&pre)[kSVec], int tid) {
#pragma unroll
    for (int v = 0; v < kSVec; ++v) {
        const int off = (v * 256 + tid) * 16;
        if (off >= kStage) continue;
        *reinterpret_cast<uint4*>(g_stage + off) = pre[v];
    }
}

struct LdsWin {   // one block's 88-byte window in the stage (r0: 8-aligned stage index)
    int r0;
    __device__ __forceinline__ uint32_t byte(int j) const { return g_stage[r0 + j]; }
    __device__ __forceinline__ uint32_t dword(int k) const {
        return *reinterpret_cast<const uint32_t*>(g_stage + r0 + 4 * k);
    }
};

// bytes [r, r + len) of the stage (len <= 16) packed little-endian into two u64
__device__ __forceinline__ void pack_stage(int r, int len, uint64_t& lo, uint64_t& hi) {
    const int a = r & ~7, sh = (r & 7) * 8;
    const uint64_t* q = reinterpret_cast<const uint64_t*>(g_stage + a);
    const uint64_t x0 = q[0], x1 = q[1], x2 = q[2];
    lo = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
    hi = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
    if (len < 8) {
        lo &= (1ULL << (8 * len)) - 1;
        hi = 0;
    } else if (len < 16) {
        hi &= len == 8 ? 0ULL : (1ULL << (8 * (len - 8))) - 1;
    }
}


}  // namespace
}  // namespace bpe
