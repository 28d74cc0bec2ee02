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
void set_error(int code, const std::string& msg);
struct Error {
    int code;
    std::string msg;
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
        n = count;
        if (count) BPE_HIP(hipMalloc(&p, count * sizeof(T)));
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

inline unsigned ceil_div(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }
inline size_t next_pow2(size_t x) {
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace bpe
