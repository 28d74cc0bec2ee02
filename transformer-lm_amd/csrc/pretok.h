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

// FNV-1a over the bytes, then a final avalanche: used to place words in the count table.
template <class Src>
__device__ __forceinline__ uint64_t hash_word(const Src& s, size_t p, size_t len) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (size_t i = 0; i < len; ++i) h = (h ^ s[p + i]) * 0x100000001b3ULL;
    return mix64(h ^ len);
}
__device__ __forceinline__ uint64_t hash_word(const uint8_t* __restrict__ s, size_t len) {
    return hash_word(s, 0, len);
}

}  // namespace bpe
