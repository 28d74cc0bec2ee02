// Device pre-tokenizer: the GPT-2 pattern of the reference,
//   '(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
// (reference models/tokenizer/train.py:143-146 and tokenizer.py:26, matched with the
// `regex` module's leftmost-first alternation), as a per-thread scanner over UTF-8 bytes.
//
// The regex reduces to a small decision on character classes:
//   * "'" followed by s/d/m/t or ll/ve/re            -> a 2- or 3-byte contraction;
//   * an optional U+0020, then a maximal run of ONE class (letter | number | other);
//   * otherwise a whitespace run, which gives back its last character when a
//     non-space follows (the `\s+(?!\S)` alternative), except a lone one (`\s+`).
// There is no look-behind, so the tokens of a string are a function of (string, start);
// a U+0020 between two ASCII non-space bytes always begins a token, which is what lets the
// corpus be cut into independent pieces (safe points) for threads and for GPUs.
#pragma once

#include <cstddef>
#include <cstdint>

#include "bpe_common.h"

namespace bpe {

#define BPE_UCTAB __device__ const
#include "uniclass_tables.inc"
#undef BPE_UCTAB

// The scanners below read bytes through `Src`: a plain device pointer, or an accessor with
// operator[](size_t) (e.g. a corpus window staged in LDS with a global fallback).

// ASCII classes by arithmetic (no table load on the per-byte critical path); checked against
// the generated table at compile time below.
__host__ __device__ constexpr int ascii_class(uint32_t b) {
    return ((b | 0x20u) - 'a' < 26u) ? CLS_LETTER
         : (b - '0' < 10u)           ? CLS_NUMBER
         : (b == 0x20u || b - 9u < 5u) ? CLS_SPACE
                                      : CLS_OTHER;
}
namespace uctab_check {
#define BPE_UCTAB constexpr
#include "uniclass_tables.inc"
#undef BPE_UCTAB
constexpr bool ascii_ok() {
    for (unsigned b = 0; b < 128; ++b)
        if (ascii_class(b) != BPE_ASCII_CLASS[b]) return false;
    return true;
}
static_assert(ascii_ok(), "ascii_class() disagrees with the generated regex class table");
}  // namespace uctab_check

// class of the code point at s[i] (validated UTF-8); *len = its byte length
template <class Src, class Idx>
__device__ __forceinline__ int class_at(const Src& s, Idx i, int* len) {
    uint32_t b0 = s[i];
    if (b0 < 0x80u) {
        *len = 1;
        return ascii_class(b0);
    }
    uint32_t cp;
    if (b0 < 0xE0u) {
        cp = ((b0 & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu);
        *len = 2;
    } else if (b0 < 0xF0u) {
        cp = ((b0 & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu);
        *len = 3;
    } else {
        cp = ((b0 & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) |
             (s[i + 3] & 0x3Fu);
        *len = 4;
    }
    cp = cp < 0x110000u ? cp : 0x10FFFFu;   // never past the tables, even on unvalidated bytes
    const unsigned pg = BPE_UC_PAGE[cp >> 8];
    return (BPE_UC_BITS[pg][(cp & 255u) >> 2] >> ((cp & 3u) * 2)) & 3;
}

__device__ __forceinline__ bool ascii_nonspace(uint32_t b) {
    return b < 0x80u && b != 0x20u && (b < 0x09u || b > 0x0Du);
}

// A safe point: text[p] == ' ' between two ASCII non-whitespace bytes.  Splitting the text
// there does not change the pre-tokenization of either side.
template <class Src, class Idx>
__device__ __forceinline__ bool is_safe_point(const Src& s, Idx n, Idx p) {
    return p >= 1 && p + 1 < n && s[p] == 0x20 && ascii_nonspace(s[p - 1]) &&
           ascii_nonspace(s[p + 1]);
}

template <class Src, class Idx>
__device__ __forceinline__ Idx next_safe_point(const Src& s, Idx n, Idx p) {
    while (p < n && !is_safe_point(s, n, p)) ++p;
    return p < n ? p : n;
}

// End (exclusive) of the token that starts at byte p of s[0..n).
template <class Src, class Idx>
__device__ __forceinline__ Idx token_end(const Src& s, Idx n, Idx p) {
    const uint32_t b0 = s[p];
    if (b0 == 0x27u && p + 1 < n) {  // contractions
        const uint32_t b1 = s[p + 1];
        if (b1 == 's' || b1 == 'd' || b1 == 'm' || b1 == 't') return p + 2;
        if (p + 2 < n) {
            const uint32_t b2 = s[p + 2];
            if ((b1 == 'l' && b2 == 'l') || (b1 == 'v' && b2 == 'e') || (b1 == 'r' && b2 == 'e'))
                return p + 3;
        }
    }
    int l0;
    int run_cls = class_at(s, p, &l0);
    Idx q = p;
    if (b0 == 0x20u && p + 1 < n) {  // ' ?' prefix: only if a non-space follows
        int l1;
        const int c1 = class_at(s, p + 1, &l1);
        if (c1 != CLS_SPACE) {
            run_cls = c1;
            q = p + 1;
        }
    }
    if (run_cls != CLS_SPACE) {  // ' ?\p{L}+' | ' ?\p{N}+' | ' ?[^\s\p{L}\p{N}]+'
        Idx e = q;
        while (e < n) {
            int l;
            if (class_at(s, e, &l) != run_cls) break;
            e += l;
        }
        return e;
    }
    // '\s+(?!\S)' | '\s+'
    Idx e = p + l0, last = p;
    while (e < n) {
        int l;
        if (class_at(s, e, &l) != CLS_SPACE) break;
        last = e;
        e += l;
    }
    return (e == n || last == p) ? e : last;
}

// Bytes [p, p + len) of s as little-endian 8-byte chunks (the last one zero-padded), read with
// aligned 8-byte loads and funnel shifts: one load per chunk, and never past the aligned word
// that holds byte p + len - 1 (which lies in the same page as that byte).
struct Chunks8 {
    const uint64_t* a;
    unsigned sh;
    size_t left;
    uint64_t cur;
    __device__ __forceinline__ Chunks8(const uint8_t* __restrict__ s, size_t p, size_t len) {
        const uintptr_t x = reinterpret_cast<uintptr_t>(s + p);
        a = reinterpret_cast<const uint64_t*>(x & ~(uintptr_t)7);
        sh = (unsigned)(x & 7) * 8;
        left = len;
        cur = len ? a[0] : 0;
    }
    __device__ __forceinline__ uint64_t next() {   // left > 0
        ++a;
        uint64_t v;
        if (sh == 0) {
            v = cur;
            cur = left > 8 ? *a : 0;
        } else {   // the chunk runs into the next aligned word unless it ends in this one
            const uint64_t nx = sh / 8 + left > 8 ? *a : 0;
            v = (cur >> sh) | (nx << (64 - sh));
            cur = nx;
        }
        if (left < 8) v &= (1ULL << (8 * left)) - 1;
        left = left > 8 ? left - 8 : 0;
        return v;
    }
};

// The hash of a word longer than kInline (the count table's and the encoder's), 8 bytes per step,
// then a final avalanche.  (The r04 form, FNV-1a byte by byte, made one dependent load per byte:
// a wave waited ~25 round trips on any lane holding such a word.)
__device__ __forceinline__ uint64_t hash_word(const uint8_t* __restrict__ s, size_t p, size_t len) {
    Chunks8 c(s, p, len);
    uint64_t h = 0xcbf29ce484222325ULL;
    while (c.left) h = (h ^ c.next()) * 0x9E3779B97F4A7C15ULL;
    return mix64(h ^ len);
}
__device__ __forceinline__ uint64_t hash_word(const uint8_t* __restrict__ s, size_t len) {
    return hash_word(s, 0, len);
}

// bytes [a, a + len) and [b, b + len) of s are equal (8 bytes per step)
__device__ __forceinline__ bool bytes_equal(const uint8_t* __restrict__ s, size_t a, size_t b, size_t len) {
    Chunks8 x(s, a, len), y(s, b, len);
    while (x.left)
        if (x.next() != y.next()) return false;
    return true;
}

}  // namespace bpe
