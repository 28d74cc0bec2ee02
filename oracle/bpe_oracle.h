/* ORACLE -- TEST INFRASTRUCTURE ONLY (see bpe_oracle.c).  CPU restatement of the
 * reference BPE path; used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg as the checker, never by the product library. */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_OK = 0, OR_E_IO = -1, OR_E_UTF8 = -2, OR_E_KEY = -3, OR_E_ARG = -5 };

typedef struct { uint8_t* data; size_t n; } oracle_blob;

/* specials blob: u32 count, then (u32 len, bytes) per special token (UTF-8) */

/* strict UTF-8 check + universal newlines; caller frees *out with free() */
int oracle_decode_text(const uint8_t* raw, size_t n, uint8_t** out, size_t* out_n,
                       size_t* err_pos);
/* train_bpe on raw file bytes (decoded as the reference's text-mode read) / on decoded text.
 * out blob: u32 nmerges, (u32 la, a, u32 lb, b)*, u32 nvocab, (u32 len, bytes)* in id order */
int oracle_train_raw(const uint8_t* raw, size_t n, int vocab_size, const uint8_t* specials,
                     size_t specials_n, oracle_blob* out, size_t* err_pos);
int oracle_train_text(const uint8_t* text, size_t n, int vocab_size, const uint8_t* specials,
                      size_t specials_n, oracle_blob* out);
/* pretoken -> count table: u32 n, (u32 len, bytes, u64 count)* */
int oracle_word_counts(const uint8_t* text, size_t n, const uint8_t* specials, size_t specials_n,
                       oracle_blob* out);
/* pretoken spans: (u64 start, u64 len)* */
int oracle_pretokenize(const uint8_t* text, size_t n, oracle_blob* out);
/* Tokenizer(vocab, merges, specials).encode(text): out = u32 ids.
 * vocab blob: u32 n, (i64 id, u32 len, bytes)* in dict order; merges blob as train output */
int oracle_encode(const uint8_t* vocab, size_t vocab_n, const uint8_t* merges, size_t merges_n,
                  const uint8_t* specials, size_t specials_n, int specials_is_none,
                  const uint8_t* text, size_t n, oracle_blob* out);
/* encode.py:31-36: each piece [starts[i-1], starts[i]) (starts sorted byte offsets, 0 implied)
 * encoded on its own, ids concatenated */
int oracle_encode_pieces(const uint8_t* vocab, size_t vocab_n, const uint8_t* merges, size_t merges_n,
                         const uint8_t* specials, size_t specials_n, const uint8_t* text, size_t n,
                         const uint64_t* starts, size_t n_starts, oracle_blob* out);
/* Chunked word counting + training (large corpora that do not fit in memory twice).  Each
 * fed piece must end at a safe split point (see bpe_oracle.c).  _train consumes the counts;
 * _words returns them as oracle_word_counts does. */
typedef struct oracle_counter oracle_counter;
oracle_counter* oracle_counter_new(const uint8_t* specials, size_t specials_n);
int oracle_counter_feed(oracle_counter* c, const uint8_t* raw, size_t n, size_t* err_pos);
int oracle_counter_absorb(oracle_counter* dst, const oracle_counter* src);
int oracle_counter_words(const oracle_counter* c, oracle_blob* out);
int oracle_counter_train(oracle_counter* c, int vocab_size, oracle_blob* out);
void oracle_counter_free(oracle_counter* c);
void oracle_free(oracle_blob* b);

#ifdef __cplusplus
}
#endif
