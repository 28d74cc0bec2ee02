// Deterministic synthetic corpora for the bench and the large parity tests (not part of the
// reference: its configs name OpenWebText / TinyStoriesV2, which are not available offline).
//
// The text is cut into independent 4 KiB blocks; block b is produced from a splitmix64 stream
// seeded with (seed, b), integer arithmetic only, so a corpus is a pure function of
// (seed, size, flavour).  Every function here is __host__ __device__: the GPU writes the bench
// corpus straight into HBM (k_synth) and the host writes the very same bytes for the oracle
// (bpe_synth_corpus_host), so the large parity checks compare both trainers on one input.
//
// Words come from a seeded lexicon of 2^21 entries drawn log-uniformly by rank (Zipf exponent
// ~1, like natural text); the mix has capitalisation, digits, punctuation, contractions,
// newlines, a little non-ASCII, and an <|endoftext|> document separator every ~4 KB (OWT-like,
// flavour 0) or ~800 B with a 2^14-word lexicon (TinyStories-like, flavour 1).
#pragma once

#include "bpe_common.h"

namespace bpe {
namespace synth {

constexpr size_t kBlock = 4096;

struct Rng {
    unsigned long long s;
    __host__ __device__ unsigned long long next() {
        s += 0x9E3779B97F4A7C15ULL;
        return mix64(s);
    }
    __host__ __device__ unsigned below(unsigned n) { return (unsigned)(next() % n); }
};

struct Out {
    uint8_t* p;
    size_t left;
    __host__ __device__ bool put(uint8_t c) {
        if (!left) return false;
        *p++ = c;
        --left;
        return true;
    }
    // two bytes of a UTF-8 sequence, or nothing when they do not both fit
    __host__ __device__ void put2(const char* two) {
        if (left < 2) return;
        put((uint8_t)two[0]);
        put((uint8_t)two[1]);
    }
    __host__ __device__ void str(const char* s) {
        while (*s) put((uint8_t)*s++);
    }
};

// English-ish letter frequencies (per 64); 2-byte Latin-1 and Cyrillic letters
__host__ __device__ inline char letter(unsigned i) {
    return "eeeeeeetttttaaaaooooiiiinnnnssshhhrrrddllccuumwfgypbvketaoinjxqz"[i & 63];
}
__host__ __device__ inline const char* latin2(unsigned i) {
    return &"\xC3\xA9\xC3\xA0\xC3\xBC\xC3\xB6\xC3\xB1\xC3\xA7\xC3\x9F\xC3\xA4"[2 * (i & 7)];
}
__host__ __device__ inline const char* cyr2(unsigned i) {
    return &"\xD0\xB0\xD0\xB5\xD0\xB8\xD0\xBE\xD1\x81\xD1\x82\xD1\x80\xD0\xBD"[2 * (i & 7)];
}

// lexicon word `rank`: frequent words are short
__host__ __device__ inline void emit_word(Out& o, unsigned long long lex_seed, unsigned rank, int bucket,
                                          bool cap) {
    unsigned long long h = mix64(lex_seed ^ (0xD1B54A32D192ED03ULL * (rank + 1)));
    const int len = 1 + (bucket >> 1) + (int)(h % 4);
    const unsigned kind = (unsigned)((h >> 32) % 256);
    for (int i = 0; i < len; ++i) {
        h = mix64(h + i);
        if (kind == 0) { o.put2(cyr2((unsigned)h)); continue; }
        if (kind < 6 && i == len / 2) { o.put2(latin2((unsigned)h)); continue; }
        char c = letter((unsigned)h);
        if (i == 0 && cap) c = (char)(c - 32);
        o.put((uint8_t)c);
    }
}

// Block `b` of the corpus: `len` (<= kBlock) bytes at `dst`.
__host__ __device__ inline void block(uint8_t* dst, size_t len, unsigned long long seed, int flavour,
                                      unsigned long long b) {
    Rng r{mix64(seed * 0x9E3779B97F4A7C15ULL + b + 1)};
    const unsigned long long lex_seed = mix64(seed ^ 0x5bd1e995ULL);
    const int lex_bits = flavour == 1 ? 14 : 21;
    const unsigned eot_per = flavour == 1 ? 160 : 800;
    Out o{dst, len};
    bool sentence_start = false;
    // every block starts " The" and ends with a letter run, so every block boundary is a
    // safe split point: a rank's slab [r*B, (r+1)*B) blocks is exactly its share of the corpus
    if (len >= 8) o.str(" The");
    while (o.left > 32) {  // no piece is longer than 30 bytes: nothing is ever truncated
        const unsigned k = r.below(1000);
        if (r.below(eot_per) == 0) {
            o.str(".<|endoftext|>");
            o.str(r.below(2) ? "\n" : "\n\n");
            sentence_start = true;
            continue;
        }
        if (k < 760) {  // a lexicon word, log-uniform rank (~Zipf 1)
            const int bucket = (int)r.below((unsigned)lex_bits);
            const unsigned rank = ((1u << bucket) - 1) + r.below(1u << bucket);
            const bool cap = sentence_start || r.below(20) == 0;
            if (!sentence_start || r.below(4)) o.put(' ');
            emit_word(o, lex_seed, rank, bucket, cap);
            sentence_start = false;
        } else if (k < 830) {
            const unsigned i = r.below(11);
            switch (i) {
                case 0: case 2: o.str(","); break;
                case 1: case 3: o.str("."); break;
                case 4: o.str("!"); break;
                case 5: o.str("?"); break;
                case 6: o.str(";"); break;
                case 7: o.str(":"); break;
                case 8: o.str("..."); break;
                case 9: o.str(" -"); break;
                default: o.str("\""); break;
            }
            sentence_start = i == 1 || i == 3 || i == 4 || i == 5;
        } else if (k < 870) {
            o.put(' ');
            const unsigned d = 1 + r.below(flavour == 1 ? 2 : 6);
            for (unsigned i = 0; i < d; ++i) o.put((uint8_t)('0' + r.below(10)));
        } else if (k < 905) {
            const unsigned i = r.below(8);
            const char* c = i == 0 ? "'s" : i == 1 ? "'t" : i == 2 ? "'re" : i == 3 ? "'ve"
                          : i == 4 ? "'ll" : i == 5 ? "'d" : i == 6 ? "'m" : "'S";
            o.str(c);
        } else if (k < 945) {
            o.str(r.below(3) ? ".\n" : ".\n\n");
            sentence_start = true;
        } else if (k < 965) {
            const unsigned i = r.below(6);
            const char* q = i == 0 ? " (" : i == 1 ? ")" : i == 2 ? " \"" : i == 3 ? "\"" : i == 4 ? " '" : "'";
            o.str(q);
        } else if (k < 975) {
            o.str(r.below(2) ? "  " : " \t");
        } else if (k < 980 && flavour != 1) {
            if (r.below(2)) o.put2("\xC2\xA0");
            else { o.put(0xE2); o.put(0x80); o.put(0x94); }
        } else if (k < 983 && flavour != 1) {
            o.str(" \xF0\x9F\x99\x82");
        } else {
            o.put(' ');
            emit_word(o, lex_seed, r.below(64), 0, false);
        }
    }
    // pad the block to its exact size with " zzz..." (one pre-token), ending on a letter
    if (o.left >= 2) o.put(' ');
    while (o.left) o.put('z');
}

}  // namespace synth
}  // namespace bpe
