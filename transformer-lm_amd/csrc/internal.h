// Host-side interfaces shared by the libbpe355 translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "bpe_common.h"

namespace bpe {

// ---------------------------------------------------------------- communicator
// Sum-all-reduce of int64 buffers across the ranks that each own one corpus slab.
struct Comm {
    int nranks = 1, rank = 0, device = 0;
    virtual ~Comm() = default;
    // in-place sum over ranks of d_buf[0..count) (device memory), ordered on `stream`
    virtual void allreduce_i64(int64_t* d_buf, size_t count, hipStream_t stream) = 0;
    // d_recv[r * bytes .. (r + 1) * bytes) = rank r's d_send[0 .. bytes) (default: through
    // allreduce_i64; RCCL overrides it with ncclAllGather)
    virtual void allgather_bytes(const void* d_send, size_t bytes, void* d_recv, hipStream_t stream);
    // all-to-all of variable sizes: rank p receives scnt[p] bytes from d_send + soff[p] of this
    // rank, and this rank's d_recv + roff[q] gets rcnt[q] bytes from rank q (default: through
    // allgather_bytes, every rank's whole send buffer; RCCL and the in-process ranks override it
    // with point-to-point copies)
    virtual void alltoallv_bytes(const void* d_send, const size_t* soff, const size_t* scnt, void* d_recv,
                                 const size_t* roff, const size_t* rcnt, hipStream_t stream);
};

// ---------------------------------------------------------------- small transfers (hostio.hip)
// host <- device and device <- host through a pinned device-mapped buffer moved by a kernel (no
// copy-engine queue, so they do not wait behind bulk DMA); return once the bytes have arrived
void to_host(void* dst, const void* d_src, size_t bytes, hipStream_t stream);
void to_device(void* d_dst, const void* src, size_t bytes, hipStream_t stream);

// ---------------------------------------------------------------- text preparation
// Validates strict UTF-8 and applies universal newlines (reference train.py:22 text-mode
// read).  Returns the device pointer to use (d_in itself when no \r is present, else
// `scratch`) and the resulting length.  Throws Error{BPE_E_UTF8} on bad input.
const uint8_t* prepare_text(const uint8_t* d_in, size_t n, DevBuf<uint8_t>& scratch,
                            size_t* n_out, hipStream_t stream);

// Byte offsets of characters 0, k, 2k, ... of the UTF-8 text d_text[0, n) (io.hip): where the
// pieces f.read(k) returns begin (reference encode.py:31-33).
std::vector<uint64_t> utf8_piece_starts(const uint8_t* d_text, size_t n, size_t k, hipStream_t stream);
// The same over a range of a longer text whose first character is character c_base: appends the
// starts found (plus `offset`) to out, returns the range's character count.  scratch (optional)
// keeps the device arrays across calls: a freed device buffer synchronises the whole device, which
// in the overlapped encode_file would wait for the copies other threads have in flight.
struct PieceScratch {
    DevBuf<unsigned long long> cnt, first, marks;
    DevBuf<uint8_t> tmp;
};
uint64_t piece_starts_range(const uint8_t* d_text, size_t n, size_t k, uint64_t c_base, uint64_t offset,
                            hipStream_t stream, std::vector<uint64_t>& out, PieceScratch* scratch = nullptr);

// ---------------------------------------------------------------- unique-word count
struct WordCounts {
    DevBuf<unsigned long long> kv;    // cap x {key, count} (layout: text.hip), key 0 = empty
    DevBuf<unsigned long long> pos;   // cap: an occurrence of each inline-keyed word
    size_t cap = 0;
    uint64_t n_pretokens = 0;         // multi-byte pre-tokens seen
    uint64_t n_records = 0;           // cache misses spilled as records (count.hip)
    double reduce_ms = 0;             // device time of their aggregation after the last launch (when timed)
    double partial_ms = 0;            // ... and of the batches aggregated between launches (file path)
    unsigned batches = 0;             // aggregation batches
};
// Pre-tokenize text[0..n) with the GPT-2 pattern and count the multi-byte words.
// (Single-byte words carry no pairs and cannot affect training.)
void count_words(const uint8_t* d_text, size_t n, WordCounts& wc, hipStream_t stream,
                 float* kernel_ms);

// The same count over a text that arrives in segments [lo, hi) cut at safe split points
// (text.hip): range() enqueues one launch per segment into one table; finish() returns false
// when the table overflowed (then recount everything with a larger table).
struct RecPoolOwner;
struct CountPass {
    WordCounts wc;
    bool v2 = true;                       // the byte-parallel counter (count.hip); BPE355_COUNT_V1: the serial one
    std::unique_ptr<RecPoolOwner> rec;    // its record pool (large texts)
    bool pool_fallback = false;           // the pool did not fit in device memory: misses go to the table
    unsigned grid2 = 0;
    DevBuf<unsigned> status;
    DevBuf<unsigned long long> ntok, fill;
    const uint8_t* text = nullptr;
    size_t total = 0;
    hipStream_t s = nullptr;
    bool timed = false;
    const unsigned long long* gate = nullptr;   // device flag: skip the launches unless ~0
    double kernel_ms = 0;        // summed device time of the launches (when timed)
    std::vector<hipEvent_t> ev, pev;   // count launches, partial aggregations
    static size_t initial_cap(size_t n);
    void begin(const uint8_t* d_text, size_t n, size_t cap, hipStream_t stream, bool timing);
    void range(size_t lo, size_t hi);
    // aggregate the records of the pages completed so far (the file path calls it between
    // segments, while the next ones arrive); finish() does the rest
    void partial();
    bool finish();
    CountPass();
    ~CountPass();
};

// Strict UTF-8 validation by segment (the first bad byte, and whether any \r is present).
struct ValidatePass {
    DevBuf<unsigned long long> flags;
    const uint8_t* text = nullptr;
    size_t total = 0;
    hipStream_t s = nullptr;
    void begin(const uint8_t* d_text, size_t n, hipStream_t stream);
    void range(size_t lo, size_t hi);
    // the units not yet validated whose windows lie inside the loaded prefix [0, loaded) of a
    // text that ends at `total` (all of them once loaded == total); returns the validated end
    size_t prefix(size_t loaded);
    size_t done_units = 0;
    void finish(unsigned long long* err_pos, bool* has_cr);   // err_pos ~0: none
};

// A corpus already validated and counted (the overlapped file path, drive.hip)
struct Prepared {
    const uint8_t* text = nullptr;
    size_t n = 0;
    WordCounts wc;
    double t_prepare_ms = 0, t_count_ms = 0, load_ms = 0;
    float count_kernel_ms = 0;
};

// ---------------------------------------------------------------- multi-GPU word exchange
// Replace this rank's word table by the union of every rank's (counts summed), whose words'
// bytes live in `all` (exchange.hip).  One all-gather; afterwards no rank needs the others.
// stats (may be null): t_gather_ms, t_union_ms and exchange_seg_bytes are filled in.
void union_word_tables(const uint8_t* text, WordCounts& wc, Comm* comm, hipStream_t stream,
                       DevBuf<uint8_t>& all, uint64_t* union_words, bpe_train_stats* stats = nullptr);

// ---------------------------------------------------------------- training driver
struct TrainOutput {
    std::vector<std::pair<uint32_t, uint32_t>> merges_internal;  // (a, b) internal ids
    std::vector<std::string> tok_bytes;                          // internal id -> bytes
    std::vector<std::pair<std::string, std::string>> merges;     // byte pairs, in order
    bpe_train_stats stats{};
};
struct TrainOpts {
    size_t slab_offset = 0;     // this slab's first byte in the whole corpus (error positions)
    bool merge_loop = true;     // false: stop after the word exchange (another rank trains)
    bool has_pending = false;   // an error this rank hit before training (e.g. reading its
    Error pending{0, ""};       // slab); raised by every rank together, before any collective
};
std::unique_ptr<Comm> make_rccl_comm(const uint8_t id[128], int nranks, int rank, int device);
// ranks that are threads of one process, possibly sharing a device (tests; comm.hip)
std::shared_ptr<void> make_inproc_group();
std::unique_ptr<Comm> make_inproc_comm(const std::shared_ptr<void>& group, int nranks, int rank, int device);
// BPE355_EXCHANGE=rounds: several ranks keep their slabs' words and all-reduce the pair deltas
// every round, so every rank runs the merge loop (default: one word-table exchange)
bool per_round_exchange();
void train_on_device(const uint8_t* d_raw, size_t n, int vocab_size,
                     const std::vector<std::string>& specials, Comm* comm, hipStream_t stream,
                     TrainOutput& out, const TrainOpts& opt = TrainOpts{}, Prepared* pre = nullptr);

bool timing_enabled();

}  // namespace bpe
