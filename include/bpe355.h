/*
 * libbpe355 -- MI355X (gfx950) byte-level BPE trainer and encoder, C ABI.
 *
 * The drop-in boundary for gashon/transformer-lm's tokenizer path.  The reference has no
 * FFI (it is pure Python); these entry points are what its two Python APIs bind to through
 * ctypes (binding: transformer-lm_amd/bpe_amd/_lib.py):
 *
 *   bpe_train_file / bpe_train_buffer   <- train_bpe(input_path, vocab_size, special_tokens)
 *                                          reference models/tokenizer/train.py:142-231 (its
 *                                          OWT caller, perf/bpe/util.py:16, is one process:
 *                                          n_gpus spreads that one call over the node's GPUs)
 *   bpe_tok_create                      <- Tokenizer.__init__(vocab, merges, special_tokens)
 *                                          reference models/tokenizer/tokenizer.py:12-38
 *   bpe_tok_encode                      <- Tokenizer.encode(text)
 *                                          reference models/tokenizer/tokenizer.py:111-138
 *
 * Conventions
 *  - Every function returns 0 (BPE_OK) or a negative BPE_E_* code; bpe_last_error() gives the
 *    message of the calling thread's last failure.  The Python binding maps BPE_E_IO to
 *    OSError/FileNotFoundError, BPE_E_UTF8 to UnicodeDecodeError and BPE_E_KEY to KeyError,
 *    the exception types the reference raises (train.py:22, tokenizer.py:135).
 *  - Plain pointers and sizes only.  The library owns result objects until *_free().
 *  - Byte-string lists cross the boundary as blobs: a sequence of (u32 little-endian length,
 *    bytes) records.  Merges: (len a, a, len b, b) per merge, in creation order.  Vocab:
 *    (len, bytes) per id, ids 0..n-1 in order (reference Vocab ids are dense, vocab.py:32).
 *  - There is no CPU fallback: without a usable gfx950 device every compute call fails with
 *    BPE_E_HIP.
 */
#ifndef BPE355_H
#define BPE355_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BPE355_ABI_VERSION 2

enum {
    BPE_OK = 0,
    BPE_E_IO = -1,       /* file could not be read (errno in bpe_last_errno()) */
    BPE_E_UTF8 = -2,     /* input is not valid UTF-8 (reference: UnicodeDecodeError) */
    BPE_E_KEY = -3,      /* a merged token is missing from the vocab (reference: KeyError) */
    BPE_E_HIP = -4,      /* HIP runtime / device failure, or no gfx950 device */
    BPE_E_ARG = -5,      /* invalid argument */
    BPE_E_NOMEM = -6,    /* device or host allocation failed */
    BPE_E_RCCL = -7,     /* collective failure */
    BPE_E_LIMIT = -8     /* input exceeds a documented limit (pre-token >= 8 MiB, corpus > 1 TiB) */
};

typedef struct bpe_result bpe_result;
typedef struct bpe_tokenizer bpe_tokenizer;
typedef struct bpe_comm bpe_comm;

int bpe_abi_version(void);
/* The HIP runtime this process bound the library to.  The library is compiled against the ROCm
 * headers of the build image (HIP_VERSION, *compiled); the libamdhip64.so.7 that serves it is
 * whichever copy of that soname the process loaded first -- inside a PyTorch-ROCm process,
 * torch's bundled one (*runtime, hipRuntimeGetVersion; runtime_path: the file, via dladdr).
 * The Python binding refuses a runtime of a different major version. */
int bpe_runtime_info(int* compiled_hip_version, int* runtime_hip_version, char* runtime_path, size_t cap);
const char* bpe_last_error(void);
int bpe_last_errno(void);
/* number of visible gfx950 devices (0 if none); never fails */
int bpe_device_count(void);

/* ---------------------------------------------------------------- multi-GPU (RCCL) */
/* One process per GPU.  Rank 0 creates the id, the caller broadcasts its 128 bytes (e.g. with
 * torch.distributed), every rank calls bpe_comm_init.  A NULL comm means single GPU. */
int bpe_comm_unique_id(uint8_t id_out[128]);
int bpe_comm_init(const uint8_t id[128], int nranks, int rank, int device, bpe_comm** out);
/* A host-staged communicator for testing the sharded path without RCCL: the library calls
 * fn(ctx, buf, count) to all-reduce `count` int64 values in place (sum) on the host. */
typedef int (*bpe_host_allreduce_fn)(void* ctx, int64_t* buf, size_t count);
int bpe_comm_init_host(bpe_host_allreduce_fn fn, void* ctx, int nranks, int rank, int device,
                       bpe_comm** out);
void bpe_comm_free(bpe_comm* comm);

/* ---------------------------------------------------------------- training */
/* train_bpe(input_path, vocab_size, special_tokens) (reference train.py:142-231): reads the
 * file like the reference's open(path, "r", encoding="utf-8").read() (train.py:22: strict
 * UTF-8, universal newlines; a pipe or FIFO is read to EOF).  The file is read by a pool of
 * host threads into pinned staging and copied to HBM while the next piece is read.
 * n_gpus: devices of THIS process to use (<= 0: every visible device).  With more than one,
 * each device takes one slab of the file cut at safe split points, counts its words, one RCCL
 * all-gather merges the word tables and the first device trains on the union.  The result is
 * identical for every n_gpus.  Errors: BPE_E_IO (errno: ENOENT, EISDIR, ...), BPE_E_UTF8. */
int bpe_train_file(const char* path, int vocab_size, const char* const* specials, int n_specials,
                   int n_gpus, bpe_result** out);
/* One rank of a multi-process job (one process per GPU, comm from bpe_comm_init):
 * split = 0: the file is this rank's slab (slabs cut at pre-token boundaries, bpe_safe_split);
 * split = 1: the file is the whole corpus and this rank reads its share of it.
 * All ranks obtain the identical, global result. */
int bpe_train_file_comm(const char* path, int vocab_size, const char* const* specials,
                        int n_specials, bpe_comm* comm, int split, bpe_result** out);
/* train_bpe on raw file bytes in host memory (this rank's slab when comm is set) */
int bpe_train_buffer(const uint8_t* data, size_t n, int vocab_size, const char* const* specials,
                     int n_specials, bpe_comm* comm, bpe_result** out);
/* same, spread over n_gpus devices of this process as bpe_train_file does */
int bpe_train_buffer_gpus(const uint8_t* data, size_t n, int vocab_size,
                          const char* const* specials, int n_specials, int n_gpus,
                          bpe_result** out);
/* same, raw bytes already resident in device memory (d_data on the current device; it is not
 * modified).  stream may be NULL (the library's own stream). */
int bpe_train_device(const uint8_t* d_data, size_t n, int vocab_size, const char* const* specials,
                     int n_specials, bpe_comm* comm, void* hip_stream, bpe_result** out);

/* extract_subword_frequencies (reference train.py:16-28) on the device, for checking the
 * pre-tokenizer + counter on its own: the multi-byte pre-tokens of the text-mode-decoded
 * bytes and their counts (1-byte words carry no pairs and are not counted; pre-tokens equal to
 * a special are skipped, train.py:25).  *blob: (u32 len, bytes, u64 count) records in no
 * particular order, malloc'ed; release with bpe_blob_free. */
int bpe_word_counts(const uint8_t* data, size_t n, const char* const* specials, int n_specials,
                    uint8_t** blob, size_t* blob_n);
void bpe_blob_free(uint8_t* blob);

int64_t bpe_result_n_merges(const bpe_result* r);
int64_t bpe_result_n_vocab(const bpe_result* r);
/* blob views owned by the result */
size_t bpe_result_merges_blob(const bpe_result* r, const uint8_t** data);
size_t bpe_result_vocab_blob(const bpe_result* r, const uint8_t** data);
/* The same records flat: which = 0 merges (a0, b0, a1, b1, ...), 1 vocab in id order; *lens gets
 * one length per record, *bytes their concatenation (*n_bytes long); returns the record count.
 * (Host-side plumbing for the Python shim: one buffer sliced, not one parse per record.) */
size_t bpe_result_flat(const bpe_result* r, int which, const uint32_t** lens, const uint8_t** bytes,
                       size_t* n_bytes);
/* The merges as vocab ids: *ids gets (a0, b0, a1, b1, ...), the ids of flat record order 1 whose
 * bytes each merge joins; returns the merge count (0: not available, use bpe_result_flat 0).  The
 * Python shim then builds merges from the vocab's own bytes objects, as the reference does when it
 * appends (vocab[a], vocab[b]) (train.py:191-196), instead of one new bytes object per part. */
size_t bpe_result_merge_ids(const bpe_result* r, const uint32_t** ids);

typedef struct {
    double t_total_ms;        /* whole call, host wall clock */
    double t_prepare_ms;      /* UTF-8 check + newline translation */
    double t_count_ms;        /* pre-tokenize + unique-word count */
    double t_words_ms;        /* word table + initial pair histogram */
    double t_merge_ms;        /* merge loop */
    double merge_kernel_ms;   /* summed device time of the merge-apply kernel (event-timed) */
    int64_t merge_kernel_launches;
    double merge_kernel_bytes; /* algorithmic bytes moved by those launches */
    double count_kernel_ms;   /* device time of the pre-tokenize/count kernel */
    double count_kernel_bytes;
    int64_t n_bytes;          /* corpus bytes after newline translation (this rank) */
    int64_t n_pretokens;      /* pre-tokens counted (this rank, excl. 1-byte and specials) */
    int64_t n_words;          /* unique multi-byte words (this rank) */
    int64_t n_word_tokens;    /* initial token slots over those words */
    int64_t n_pairs_final;    /* pair-table keys at the end */
    int64_t n_rebuilds;       /* candidate-set rebuilds */
    int64_t n_rounds_device;  /* merges decided on the device */
    int64_t n_rounds_host;    /* zero-count merges emitted after exhaustion */
    int64_t n_index_builds;   /* word-table compactions + posting-list builds */
    int64_t n_trips;          /* merge-loop round trips (several exact merges each when batched) */
    int64_t n_rounds_batched; /* rounds taken in trips of more than one merge */
    double t_exchange_ms;     /* multi-GPU word-table exchange (0 on one rank) */
    int64_t n_exchanged_words; /* local unique words of all ranks gathered (before dedupe) */
    double t_load_ms;         /* file / host buffer -> HBM (0 when the corpus starts in HBM) */
    int64_t n_gpus;           /* devices (ranks) that took part */
    double count_reduce_ms;   /* device time aggregating the counter's spilled records */
    int64_t n_count_records;  /* pre-tokens (or cache entries) spilled as records by the counter */
    double count_partial_ms;  /* device time of the aggregations done while the file was loading */
    int64_t n_count_batches;  /* aggregation batches (1 + those done during the load) */
    double t_gather_ms;       /* multi-GPU word exchange: the all-gather of the segments */
    double t_union_ms;        /* multi-GPU word exchange: the union-table inserts */
    int64_t exchange_seg_bytes; /* multi-GPU word exchange: one rank's segment (all ranks' equal) */
    double t_alltoall_ms;     /* multi-GPU word exchange: the all-to-all of the words by owner */
    double t_owner_ms;        /* multi-GPU word exchange: the owner-table inserts */
    int64_t exchange_a2a_bytes; /* multi-GPU word exchange: the bytes this rank sent in the all-to-all */
} bpe_train_stats;
int bpe_result_stats(const bpe_result* r, bpe_train_stats* out);
void bpe_result_free(bpe_result* r);

/* Hands back the device memory the trainer keeps between calls so that a repeated train_bpe
 * does not pay for fresh allocations: the corpus buffer (drive.hip), the counter's record pool
 * and aggregation bins (count.hip; about 2 x 2 bytes per corpus byte), for `device` (< 0: every
 * device).  The reference keeps nothing after train_bpe returns (train.py:231) and its caller
 * trains an LM on the same GPU next (train.py:230-232), so the Python train_bpe calls this after
 * every call unless keep_device_buffers=True.  Buffers held by a call in flight are not touched,
 * and the cached copy streams (no HBM to speak of) stay for the process, so a transfer of
 * another thread is never cut off.  Tokenizer buffers: bpe_tok_release_buffers.  *freed_bytes (may be
 * NULL): device bytes handed back. */
int bpe_release_device_memory(int device, size_t* freed_bytes);

/* Enable per-launch event timing of the hot kernels (bench / profiling); default off. */
void bpe_set_timing(int enable);

/* ---------------------------------------------------------------- tokenizer */
/* Tokenizer(vocab, merges, special_tokens).  vocab blob: u32 count, then per entry
 * (i64 id, u32 len, bytes) in the caller's dict order (the reverse map keeps the LAST id of a
 * duplicated byte string, tokenizer.py:19).  merges blob: u32 count + merge records.
 * specials: NULL/0 for none.  Missing specials are appended with ids len(vocab), ...
 * (tokenizer.py:35-38); their ids are reported by bpe_tok_special_id. */
int bpe_tok_create(const uint8_t* vocab_blob, size_t vocab_n, const uint8_t* merges_blob,
                   size_t merges_n, const char* const* specials, int n_specials,
                   bpe_tokenizer** out);
int64_t bpe_tok_special_id(const bpe_tokenizer* tok, int i);
/* encode(text): UTF-8 bytes in host memory -> ids.  cap >= n always suffices.
 * Limits of one call (BPE_E_LIMIT): a pre-token under 8 MiB; at most 2^28 word-table slots,
 * i.e. about 134 M distinct pre-tokens at the table's half load (an 11.9 GB OWT-like text has
 * 7.5 M).  A text past that is encoded in pieces cut at safe points (bpe_tok_encode_gpus cuts
 * them that way on one device too), whose concatenated ids are the whole text's. */
int bpe_tok_encode(bpe_tokenizer* tok, const uint8_t* utf8, size_t n, uint32_t* ids_out,
                   size_t cap, size_t* n_out);
/* same, device-resident text and output (d_out holds >= n ids) */
int bpe_tok_encode_device(bpe_tokenizer* tok, const uint8_t* d_utf8, size_t n, uint32_t* d_out,
                          size_t* n_out, void* hip_stream);
/* Chunked encode: the ids of encode(text[starts[i] : starts[i+1]]) for every piece, concatenated
 * (starts sorted byte offsets; the last piece runs to n).  A piece boundary ends every
 * pre-token and no special token may straddle it -- exactly separate encode() calls, as the
 * reference's encode_iterable (tokenizer.py:140-150: 2 MiB-character batches) and dataset
 * encoder (encode.py:31-36: 1 M-character reads) make them. */
int bpe_tok_encode_chunks(bpe_tokenizer* tok, const uint8_t* utf8, size_t n, const uint64_t* starts,
                          size_t n_starts, uint32_t* ids_out, size_t cap, size_t* n_out);
int bpe_tok_encode_chunks_device(bpe_tokenizer* tok, const uint8_t* d_utf8, size_t n, const uint64_t* starts,
                                 size_t n_starts, uint32_t* d_out, size_t* n_out, void* hip_stream);
/* The reference's dataset encoder (encode.py:18-38) on one file: the file is read by the library's
 * pinned multi-threaded reader into HBM, decoded as open(path, "r", encoding="utf-8") reads it
 * (strict UTF-8, universal newlines), cut into chars_per_piece-character pieces (f.read(1024*1024)),
 * each piece encoded on its own, and the ids written as np.uint16 (encode.py:37; an id past
 * 65535 fails with BPE_E_LIMIT instead of wrapping) into ids_out (host memory, cap ids; the
 * file's byte count always suffices).  The device buffers are kept by the tokenizer across
 * calls (about 3 bytes of HBM per file byte: the text and its uint16 ids, on top of the
 * encoder's per-call arrays) until bpe_tok_release_buffers or bpe_tok_free.  The stages overlap:
 * the file streams in by 1 GiB slabs while the pieces already read
 * are validated, encoded and copied out (a text with a carriage return is redone in one pass
 * once read).  phase_ms (NULL or 4 doubles): busy milliseconds of the reader, of validation +
 * piece starts, of the encodes and of the copy to host. */
int bpe_tok_encode_file_u16(bpe_tokenizer* tok, const char* path, size_t chars_per_piece, uint16_t* ids_out,
                            size_t cap, size_t* n_out, double* phase_ms);
/* encode(text) on n_gpus devices of this process (<= 0: every visible one; SURVEY.md 8b's n_gpus):
 * the text is cut at safe split points that no special token spans, each device encodes its
 * piece, the ids are concatenated -- identical to bpe_tok_encode (tokenizer.py:111-138). */
int bpe_tok_encode_gpus(bpe_tokenizer* tok, const uint8_t* utf8, size_t n, uint32_t* ids_out, size_t cap,
                        size_t* n_out, int n_gpus);
/* Frees the device buffers the tokenizer keeps across calls (the encoder's record and scratch
 * arrays, the bulk encoder's text and uint16 ids, the other devices' copies); the next call
 * allocates them again.  The tables of the tokenizer itself stay. */
int bpe_tok_release_buffers(bpe_tokenizer* tok);
void bpe_tok_free(bpe_tokenizer* tok);

/* ---------------------------------------------------------------- decode */
/* Tokenizer.decode (tokenizer.py:155-157): b"".join(vocab[i] for i in ids) on the device; the
 * caller applies .decode("utf-8", errors="replace").  vocab blob: u32 count, then (i64 id,
 * u32 len, bytes) per entry -- the int-keyed entries of Tokenizer.vocab.  An id without an
 * entry fails with BPE_E_KEY (message: the id), as vocab[i] raises KeyError. */
typedef struct bpe_decoder bpe_decoder;
int bpe_dec_create(const uint8_t* vocab_blob, size_t vocab_n, bpe_decoder** out);
/* host ids -> host bytes; *n_out = byte count (also set when cap is too small: BPE_E_ARG) */
int bpe_dec_decode(bpe_decoder* dec, const uint32_t* ids, size_t n, uint8_t* out, size_t cap, size_t* n_out);
/* device ids -> device bytes */
int bpe_dec_decode_device(bpe_decoder* dec, const uint32_t* d_ids, size_t n, uint8_t* d_out, size_t cap,
                          size_t* n_out, void* hip_stream);
void bpe_dec_free(bpe_decoder* dec);

/* ---------------------------------------------------------------- bulk encode plumbing */
/* The raw bytes of a regular file -> device memory d_dst (cap bytes): pread by a pool of host
 * threads into pinned staging buffers, each DMA'd to HBM while the next is read (the file read
 * of encode.py:31-33 / tokenizer.py:111, without a pageable host copy).  d_dst == NULL: size
 * query (*n_out = file size).  BPE_E_IO (errno) on a missing file, a directory, or a file that
 * is not regular (the caller reads a pipe itself); BPE_E_ARG if cap is too small. */
int bpe_read_file_device(const char* path, uint8_t* d_dst, size_t cap, size_t* n_out);
/* n bytes of device memory -> pageable host memory h_dst (e.g. the np.uint16 array encode.py
 * saves), through pinned staging buffers, several copier threads; waits for the device first. */
int bpe_copy_to_host(const void* d_src, size_t n, void* h_dst);
/* open(path, "r", encoding="utf-8").read() on device bytes: strict UTF-8 (BPE_E_UTF8) and
 * universal newlines.  d_out holds n bytes (may be d_in); *n_out = resulting length. */
int bpe_text_prepare_device(const uint8_t* d_in, size_t n, uint8_t* d_out, size_t* n_out, void* hip_stream);
/* Byte offsets of characters 0, K, 2K, ... of valid UTF-8 (K = chars_per_chunk): the pieces
 * successive f.read(K) calls return (encode.py:31-33).  starts == NULL: count only. */
int bpe_utf8_chunk_starts_device(const uint8_t* d_text, size_t n, size_t chars_per_chunk, uint64_t* starts,
                                 size_t cap, size_t* n_starts, void* hip_stream);
/* np.array(token_ids, dtype=np.uint16) (encode.py:37), on the device; BPE_E_LIMIT if an id
 * does not fit (the reference would silently wrap it). */
int bpe_ids_to_u16_device(const uint32_t* d_ids, size_t n, uint16_t* d_out, void* hip_stream);

/* ---------------------------------------------------------------- helpers */
/* Largest p <= pos such that splitting the text at p does not change its pre-tokenization
 * (a U+0020 between two ASCII non-space bytes), or 0. Used to shard a corpus into slabs. */
size_t bpe_safe_split(const uint8_t* data, size_t n, size_t pos);
/* Deterministic synthetic corpus (bench/tests): bytes [first_block*4096, first_block*4096 + n)
 * of corpus (seed, flavour) into device memory; flavour 0 = OWT-like, 1 = TinyStories-like.
 * Every 4096-byte block boundary is a safe split point, so slabs of whole blocks shard it. */
int bpe_synth_corpus_device(uint8_t* d_out, size_t n, uint64_t seed, int flavour,
                            uint64_t first_block, void* hip_stream);
/* The same bytes written by the host (n_threads CPU threads), for the oracle side of the
 * large parity checks; needs no device. */
int bpe_synth_corpus_host(uint8_t* out, size_t n, uint64_t seed, int flavour,
                          uint64_t first_block, int n_threads);

#ifdef __cplusplus
}
#endif
#endif /* BPE355_H */
