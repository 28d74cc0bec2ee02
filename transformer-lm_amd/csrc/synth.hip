// Deterministic synthetic corpora for the bench and the large parity tests (not part of the
// reference: its configs name OpenWebText / TinyStoriesV2, which are not available offline).
//
// The text is cut into independent 4 KiB blocks; block b is produced by one thread from a
// splitmix64 stream seeded with (seed, b), integer arithmetic only, so a corpus is a pure
// function of (seed, size, flavour) on any device.  Words come from a seeded lexicon of
// 2^21 entries drawn log-uniformly by rank (Zipf exponent ~1, like natural text); the
// mix has capitalisation, digits, punctuation, contractions, newlines, a little non-ASCII,
// and an <|endoftext|> document separator every ~4 KB (OWT-like, flavour 0) or ~800 B with
// a 2^14-word lexicon (TinyStories-like, flavour 1).
#include "internal.h"

namespace bpe {
namespace {

constexpr size_t kBlock = 4096;

struct Rng {
    unsigned long long s;
    __device__ unsigned long long next() {
        s += 0x9E3779B97F4A7C15ULL;
        return mix64(s);
    }
    __device__ unsigned below(unsigned n) { return (unsigned)(next() % n); }
};

// English-ish letter frequencies (per 64)
__device__ const char kLetters[64] = {
    'e','e','e','e','e','e','e','t','t','t','t','t','a','a','a','a','o','o','o','o','i','i','i','i',
    'n','n','n','n','s','s','s','h','h','h','r','r','r','d','d','l','l','c','c','u','u','m','w','f',
    'g','y','p','b','v','k','e','t','a','o','i','n','j','x','q','z'};
__device__ const unsigned short kLatin2[8] = {0xA9C3, 0xA0C3, 0xBCC3, 0xB6C3, 0xB1C3, 0xA7C3, 0x9FC3, 0xA4C3};
__device__ const unsigned short kCyr2[8] = {0xB0D0, 0xB5D0, 0xB8D0, 0xBED0, 0x81D1, 0x82D1, 0x80D1, 0xBDD0};

struct Out {
    uint8_t* p;
    size_t left;
    __device__ bool put(uint8_t c) {
        if (!left) return false;
        *p++ = c;
        --left;
        return true;
    }
    __device__ bool put2(unsigned short v) {
        if (left < 2) return false;
        put((uint8_t)(v & 0xff));
        put((uint8_t)(v >> 8));
        return true;
    }
    __device__ void str(const char* s) {
        while (*s) put((uint8_t)*s++);
    }
};

// lexicon word `rank`: frequent words are short
__device__ void emit_word(Out& o, unsigned long long lex_seed, unsigned rank, int bucket, bool cap) {
    unsigned long long h = mix64(lex_seed ^ (0xD1B54A32D192ED03ULL * (rank + 1)));
    const int len = 1 + (bucket >> 1) + (int)(h % 4);
    const unsigned kind = (unsigned)((h >> 32) % 256);
    for (int i = 0; i < len; ++i) {
        h = mix64(h + i);
        if (kind == 0) { o.put2(kCyr2[h & 7]); continue; }
        if (kind < 6 && i == len / 2) { o.put2(kLatin2[h & 7]); continue; }
        char c = kLetters[h & 63];
        if (i == 0 && cap) c = (char)(c - 32);
        o.put((uint8_t)c);
    }
}

__global__ void k_synth(uint8_t* __restrict__ out, size_t n, unsigned long long seed, int flavour,
                        unsigned long long first_block) {
    const size_t lb = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t lo = lb * kBlock;
    const size_t b = lb + first_block;
    if (lo >= n) return;
    const size_t len = (n - lo < kBlock) ? n - lo : kBlock;
    Rng r{mix64(seed * 0x9E3779B97F4A7C15ULL + b + 1)};
    const unsigned long long lex_seed = mix64(seed ^ 0x5bd1e995ULL);
    const int lex_bits = flavour == 1 ? 14 : 21;
    const unsigned eot_per = flavour == 1 ? 160 : 800;
    Out o{out + lo, len};
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
            const char* p[] = {",", ".", ",", ".", "!", "?", ";", ":", "...", " -", "\""};
            const unsigned i = r.below(11);
            o.str(p[i]);
            sentence_start = i == 1 || i == 3 || i == 4 || i == 5;
        } else if (k < 870) {
            o.put(' ');
            const unsigned d = 1 + r.below(flavour == 1 ? 2 : 6);
            for (unsigned i = 0; i < d; ++i) o.put((uint8_t)('0' + r.below(10)));
        } else if (k < 905) {
            const char* c[] = {"'s", "'t", "'re", "'ve", "'ll", "'d", "'m", "'S"};
            o.str(c[r.below(8)]);
        } else if (k < 945) {
            o.str(r.below(3) ? ".\n" : ".\n\n");
            sentence_start = true;
        } else if (k < 965) {
            const char* q[] = {" (", ")", " \"", "\"", " '", "'"};
            o.str(q[r.below(6)]);
        } else if (k < 975) {
            o.str(r.below(2) ? "  " : " \t");
        } else if (k < 980 && flavour != 1) {
            const unsigned short u[] = {0xA0C2, 0x94E2 /*—*/};
            if (r.below(2)) o.put2(u[0]);
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

}  // namespace
}  // namespace bpe

extern "C" int bpe_synth_corpus_device(uint8_t* d_out, size_t n, uint64_t seed, int flavour,
                                       uint64_t first_block, void* hip_stream) {
    if (!d_out && n) return BPE_E_ARG;
    if (n == 0) return BPE_OK;
    hipStream_t s = (hipStream_t)hip_stream;
    const size_t blocks = (n + bpe::kBlock - 1) / bpe::kBlock;
    hipLaunchKernelGGL(bpe::k_synth, dim3(bpe::ceil_div(blocks, 128)), dim3(128), 0, s, d_out, n,
                       (unsigned long long)seed, flavour, (unsigned long long)first_block);
    if (hipGetLastError() != hipSuccess) return BPE_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return BPE_E_HIP;
    return BPE_OK;
}
