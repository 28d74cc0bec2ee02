// Token starts of the GPT-2 pre-tokenizer as a LOCAL predicate, evaluated 64 bytes at a time on
// bit masks (one bit per byte) -- the byte-parallel form of pretok.h's serial scanner.
//
// Pattern (reference models/tokenizer/train.py:143-146, tokenizer.py:26), matched leftmost-first:
//   '(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
// With K(c) in {L, N, S, O} the class of character c (S = the regex module's \s), SP = U+0020,
// AP = U+0027, a character p of the text begins a token exactly when:
//   * p is inside a contraction: no.  A contraction is an AP at q that begins a token, i.e.
//     q = 0 or (c[q-1] is not SP and K(c[q-1]) != O), followed by s|d|m|t (2 chars) or by
//     ll|ve|re (3 chars); its 2nd/3rd characters are "inside" it;
//   * p directly follows a contraction: yes;
//   * p = 0: yes;
//   * K(c[p]) = S: yes iff K(c[p-1]) != S, or c[p] is the last character of its whitespace run
//     and another character follows (the `\s+(?!\S)` give-back);
//   * otherwise (L, N or O): no if c[p-1] is SP (the ` ?` prefix takes it); yes if
//     K(c[p-1]) = S; else yes iff K(c[p-1]) != K(c[p]).
// Every case looks at characters p-4 .. p+1 only, so the starts of a 64-byte block follow from a
// window of 8 bytes before it and 16 after (a character is at most 4 bytes).  The serial scanner
// (pretok.h token_end, the oracle) and this predicate are checked against each other on CPU
// (tests/test_tokstart.py) and on the device through every parity test.
#pragma once

#include <cstddef>
#include <cstdint>

#include "bpe_common.h"

namespace bpe {

typedef unsigned __int128 u128;

constexpr int kStartPre = 8;                       // window bytes before the 64-byte block
constexpr int kStartWin = kStartPre + 64 + 16;     // 88 bytes: the block and its context

__host__ __device__ __forceinline__ u128 bit128(int j) { return (u128)1 << j; }

// class of a code point through the generated regex tables (Tab::page / Tab::bits); Tab::cls(cp)
// may answer from a faster table first
template <class Tab>
__host__ __device__ __forceinline__ int uc_class(uint32_t cp) {
    cp = cp < 0x110000u ? cp : 0x10FFFFu;
    const unsigned pg = Tab::page(cp >> 8);
    return (Tab::bits(pg, (cp & 255u) >> 2) >> ((cp & 3u) * 2)) & 3;
}

// SWAR helpers on 4 bytes at once: per-byte results are flags in bit 7 of each byte
// bit 7 of each byte of z that is zero (exact per byte: no carry crosses a byte)
__host__ __device__ __forceinline__ uint32_t zero_bytes(uint32_t z) {
    return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;
}
// the four byte flags (bits 7, 15, 23, 31) as a nibble (bit i = byte i): t = m | m << 7 has the
// flags of bytes 2, 3 at bits 30, 31 and those of bytes 0, 1 at 14, 15, which << 14 moves to 28, 29
// (no other set bit of t lands in 28..31); two shift-or ops and a shift
__host__ __device__ __forceinline__ uint32_t flag_nibble(uint32_t m) {
    const uint32_t t = m | (m << 7);
    return (t | (t << 14)) >> 28;
}

__host__ __device__ __forceinline__ int ctz128(u128 x) {
    const uint64_t lo = (uint64_t)x;
    return lo ? __builtin_ctzll(lo) : 64 + __builtin_ctzll((uint64_t)(x >> 64));
}

// Start mask of the block at window positions [kStartPre, kStartPre + 64).  The window `w` holds
// bytes [0, kStartWin) (the block's first byte is byte kStartPre): w.dword(k) = bytes 4k .. 4k+3
// little-endian, w.byte(j) = byte j.  Positions >= vhi are past the end of the text (treated as
// whitespace, never a start).  Bytes before the start of the text must read as '\n' (a
// whitespace other than SP: the text start behaves as after a line break).  Starts before a
// segment's first byte, and at it, are the caller's to clear / force.
template <class Tab, class Win>
__host__ __device__ __forceinline__ uint64_t token_starts64(const Win& w, int vhi) {
    // per-byte flags, built 4 bytes at a time (SWAR: byte-wise range checks by adds that cannot
    // carry out of a byte, flags in bit 7 of each byte, then packed to nibbles) into 32-bit
    // pieces; the rest is derived from these seven.  (The byte-by-byte form it replaces compiled
    // to ~470 instructions per 8 bytes, 40 % of them scalar mask operations, which the CU's one
    // scalar unit serialises over all its waves.)  The rolled loop over the window's dwords keeps
    // the register footprint small: unrolled, all 22 window loads are hoisted and the kernel spills.
    uint32_t fL[3] = {0, 0, 0}, fN[3] = {0, 0, 0}, fS[3] = {0, 0, 0}, fSP[3] = {0, 0, 0};
    uint32_t fAP[3] = {0, 0, 0}, fC[3] = {0, 0, 0}, fNA[3] = {0, 0, 0};
#pragma unroll
    for (int seg = 0; seg < 3; ++seg) {
#pragma unroll 1
      for (int kk = 0; kk < 8; ++kk) {
        const int k = seg * 8 + kk;
        if (k >= kStartWin / 4) break;
        const uint32_t x = w.dword(k);
        const uint32_t hi = x & 0x80808080u;       // non-ASCII bytes
        const uint32_t asc = hi ^ 0x80808080u;     // ASCII bytes
        const uint32_t lo7 = x & 0x7F7F7F7Fu;
        const uint32_t lw = lo7 | 0x20202020u;     // ASCII letters folded to lower case
        // [a-z]: lw >= 0x61 and lw < 0x7B; [0-9]: 0x30 <= lo7 < 0x3A; \t..\r: 0x09 <= lo7 < 0x0E
        const uint32_t l = (lw + 0x1F1F1F1Fu) & ~(lw + 0x05050505u) & asc;
        const uint32_t nn = (lo7 + 0x50505050u) & ~(lo7 + 0x46464646u) & asc;
        const uint32_t spc = zero_bytes(x ^ 0x20202020u);   // U+0020
        const uint32_t sp = ((lo7 + 0x77777777u) & ~(lo7 + 0x72727272u) & asc) | spc;
        const uint32_t ap = zero_bytes(x ^ 0x27272727u);    // U+0027
        const uint32_t ct = hi & ~(x << 1);        // 10xxxxxx: continuation bytes
        const uint32_t na = hi & (x << 1);         // 11xxxxxx: lead bytes of 2..4-byte characters
        const int sh = 4 * kk;
        fL[seg] |= flag_nibble(l) << sh; fN[seg] |= flag_nibble(nn) << sh; fS[seg] |= flag_nibble(sp) << sh;
        fSP[seg] |= flag_nibble(spc) << sh; fAP[seg] |= flag_nibble(ap) << sh;
        fC[seg] |= flag_nibble(ct) << sh; fNA[seg] |= flag_nibble(na) << sh;
      }
    }
    auto join = [](const uint32_t (&f)[3]) -> u128 {
        return (u128)f[0] | ((u128)f[1] << 32) | ((u128)f[2] << 64);
    };
    const u128 VALID = vhi >= 128 ? ~(u128)0 : (vhi <= 0 ? (u128)0 : bit128(vhi) - 1);
    u128 L = join(fL) & VALID, N = join(fN) & VALID;
    u128 S = (join(fS) & VALID) | ~VALID;   // past the end: whitespace (a trailing run keeps its last char)
    const u128 SP = join(fSP) & VALID, AP = join(fAP) & VALID, CONT = join(fC) & VALID;
    // non-ASCII characters: decode (validated UTF-8) and classify through the tables
    for (u128 x = join(fNA) & VALID; x; x &= x - 1) {
        const int j = ctz128(x);
        const uint32_t b = w.byte(j);
        const uint32_t b1 = j + 1 < kStartWin ? (uint32_t)w.byte(j + 1) : 0x80u;
        const uint32_t b2 = j + 2 < kStartWin ? (uint32_t)w.byte(j + 2) : 0x80u;
        const uint32_t b3 = j + 3 < kStartWin ? (uint32_t)w.byte(j + 3) : 0x80u;
        uint32_t cp;
        if (b < 0xE0u) cp = ((b & 0x1Fu) << 6) | (b1 & 0x3Fu);
        else if (b < 0xF0u) cp = ((b & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu);
        else cp = ((b & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | ((b2 & 0x3Fu) << 6) | (b3 & 0x3Fu);
        const int c = Tab::cls(cp);
        const u128 m = bit128(j);
        if (c == CLS_LETTER) L |= m;
        else if (c == CLS_NUMBER) N |= m;
        else if (c == CLS_SPACE) S |= m;
    }
    // continuation bytes take the class of their character
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        L |= (L << 1) & CONT;
        N |= (N << 1) & CONT;
        S |= (S << 1) & CONT;
    }
    const u128 LEAD = VALID & ~CONT;
    const u128 O = VALID & ~(L | N | S);
    // whitespace: the character whose last byte is followed by a non-whitespace byte
    const u128 Send = S & ~(S >> 1);
    const u128 C1 = CONT >> 1, C2 = C1 & (CONT >> 2), C3 = C2 & (CONT >> 3);
    const u128 SendLead = Send | ((Send >> 1) & C1) | ((Send >> 2) & C2) | ((Send >> 3) & C3);
    const u128 startS = S & ((~S << 1) | SendLead);
    const u128 change = (L ^ (L << 1)) | (N ^ (N << 1)) | (O ^ (O << 1));
    const u128 startX = ~S & ~(SP << 1) & ((S << 1) | change);
    u128 start = startS | startX;
    // contractions: an apostrophe that begins a token (not after SP or O), then s|d|m|t or
    // ll|ve|re -- its other characters are no starts, the character after it is one
    for (u128 x = AP & ~(SP << 1) & ~(O << 1); x; x &= x - 1) {
        const int j = ctz128(x);
        const uint32_t b1 = j + 1 < vhi ? (uint32_t)w.byte(j + 1) : 0u;
        const uint32_t b2 = j + 2 < vhi ? (uint32_t)w.byte(j + 2) : 0u;
        int len = 0;
        if (b1 == 's' || b1 == 'd' || b1 == 'm' || b1 == 't') len = 2;
        else if ((b1 == 'l' && b2 == 'l') || (b1 == 'v' && b2 == 'e') || (b1 == 'r' && b2 == 'e')) len = 3;
        if (!len) continue;
        start &= ~(bit128(j + 1) | (len == 3 ? bit128(j + 2) : (u128)0));
        if (j + len < 128) start |= bit128(j + len);
    }
    return (uint64_t)((start & LEAD) >> kStartPre);
}

}  // namespace bpe
