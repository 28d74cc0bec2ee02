// Shared host/device definitions of libbpe355 (MI355X / gfx950 byte-level BPE).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

#include "../../include/bpe355.h"

namespace bpe {

// ------------------------------------------------------------------ error plumbing
// Every C-ABI entry point returns a BPE_* code and leaves a message for bpe_last_error().
void set_error(int code, const std::string& msg, int sys_errno = 0);
struct Error {
    int code;
    std::string msg;
    int sys_errno = 0;      // for BPE_E_IO: errno, reported by bpe_last_errno on the calling thread
};

#define BPE_HIP(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            throw ::bpe::Error{BPE_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_) + \
                                              " (" __FILE__ ":" + std::to_string(__LINE__) + ")"}; \
    } while (0)

#define BPE_REQUIRE(cond, code, msg)                          \
    do {                                                      \
        if (!(cond)) throw ::bpe::Error{(code), (msg)};       \
    } while (0)

// ------------------------------------------------------------------ device buffers
template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    explicit DevBuf(size_t count) { alloc(count); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
        return *this;
    }
    ~DevBuf() { release(); }
    void alloc(size_t count) {
        release();
        if (!count) return;
        const hipError_t e = hipMalloc(&p, count * sizeof(T));
        if (e == hipErrorOutOfMemory) {
            (void)hipGetLastError();   // clear it: a later launch check must not see this failure
            p = nullptr;
            throw ::bpe::Error{BPE_E_NOMEM, "device allocation of " + std::to_string(count * sizeof(T)) +
                                                " bytes failed (out of memory)"};
        }
        BPE_HIP(e);
        n = count;
    }
    // grow-only: keep the buffer when it already holds count elements (n is then the capacity)
    void reserve(size_t count) {
        if (count > n || !p) alloc(count);
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    size_t bytes() const { return n * sizeof(T); }
};

// ------------------------------------------------------------------ character classes
enum : int { CLS_OTHER = 0, CLS_LETTER = 1, CLS_NUMBER = 2, CLS_SPACE = 3 };

// 64-bit mixers used for hashing on both sides (host copies are only for tables built
// on the host, e.g. the encoder's merge-rank map).
__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ULL;
    z ^= z >> 27; z *= 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// One atomic per wave for a predicate-driven append (same-address atomics serialize on the
// memory side, so per-lane appends to one counter are never used).  Every lane of the wave
// must call it; returns this lane's index, or ~0u when pred is false.
__device__ __forceinline__ unsigned wave_append(bool pred, unsigned* counter) {
    const unsigned long long m = __ballot(pred);
    if (!m) return ~0u;
    const int leader = __ffsll((long long)m) - 1;
    const unsigned lane = threadIdx.x & 63;
    unsigned base = 0;
    if ((int)lane == leader) base = atomicAdd(counter, (unsigned)__popcll(m));
    base = __shfl(base, leader);
    const unsigned below = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    return pred ? base + below : ~0u;
}

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <class T>
__device__ __forceinline__ T wave_max(T v) {
    for (int o = 32; o > 0; o >>= 1) {
        const T w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

inline unsigned ceil_div(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }
// Workgroups for a grid-stride kernel over `items`: a dispatch's grid is at most 2^32 work-items
// (the AQL packet's 32-bit grid size, which a larger launch silently wraps), so a kernel over
// bytes or ids of a multi-GB text strides instead of launching one thread per item.
constexpr size_t kMaxGridBlocks = 1u << 20;
inline unsigned grid_for(size_t items, unsigned block) {
    const size_t b = (items + block - 1) / block;
    return (unsigned)(b < kMaxGridBlocks ? (b ? b : 1) : kMaxGridBlocks);
}
inline size_t next_pow2(size_t x) {
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace bpe
