// The byte-parallel counter (count.hip) and its record pool, used by CountPass (text.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>

#include "internal.h"

namespace bpe {

constexpr int kPageRecs = 65536;   // records per pool page (one workgroup appends to a page)

// Device view of the record pool: SoA records {packed bytes lo, hi, len | offset << 5 | count
// << 45}, in pages owned one at a time by a counting workgroup.
struct RecPool {
    uint64_t* lo;
    uint64_t* hi;
    uint64_t* meta;
    unsigned* page_used;   // records in each page (written when a workgroup leaves the page)
    unsigned* n_pages;     // pages handed out
    unsigned max_pages;
    int* wg_page;          // per counting workgroup: its current page (-2 none yet, -1 pool spent)
    unsigned* wg_used;
    unsigned* page_ch;     // per page: records per coarse bin (kCoarse), written with page_used
    unsigned* wg_ch;       // per counting workgroup: its current page's coarse histogram
    // words longer than kInline (their bytes are not in a record): per counting workgroup a
    // segment of lw_per_wg entries {offset | len << 40}, added to the table by k_count_long after
    // each k_count2 launch (lw == nullptr: k_count2 adds them itself)
    unsigned long long* lw;
    unsigned* lw_n;
    unsigned lw_per_wg;
    int on;
};

constexpr int kCoarseBits = 6;   // first partition level: the top 6 bits of the word hash
constexpr int kCoarse = 1 << kCoarseBits;

// Three parallel u64 arrays of one capacity, on one device.  Large record arrays are kept across
// training calls (ScratchArrays::take / give): freeing and re-allocating tens of GB per call
// stalls the host for hundreds of ms (the driver clears fresh VRAM).
struct Arrays3 {
    DevBuf<uint64_t> a, b, c;
    DevBuf<uint8_t> d;   // the level-1 destination's fine bins (allocated on first use as one)
    size_t cap = 0;
    int dev = -1;
    size_t bytes() const { return 3 * cap * sizeof(uint64_t) + d.n; }
};
std::unique_ptr<Arrays3> scratch_take(size_t cap);   // exclusive until given back
void scratch_give(std::unique_ptr<Arrays3> x);
size_t scratch_cached_bytes(int dev);   // free sets of this device held by the cache
size_t scratch_release(int dev);        // hand them back to the device allocator (dev < 0: all); bytes

// a level-2 work item of the record aggregation: a tile of one coarse bin's run
struct L2Tile {
    unsigned long long start;
    unsigned len, coarse;
};

struct RecPoolOwner {
    std::unique_ptr<Arrays3> rec;    // the pool: lo, hi, meta
    DevBuf<unsigned> page_used, n_pages, wg_used, page_ch, wg_ch, lw_n;
    DevBuf<unsigned long long> lw;
    unsigned lw_per_wg = 0;
    DevBuf<unsigned> held, done, list, list_n;   // page selection of the incremental aggregation
    std::unique_ptr<Arrays3> B;                   // level-1 destination
    DevBuf<unsigned> coff, d_t0, fhist, n_tiles;
    DevBuf<unsigned long long> ctot, cbase, ftot, fbase, d_records;
    DevBuf<L2Tile> d_tl;
    unsigned max_tiles = 0;
    DevBuf<int> wg_page;
    unsigned max_pages = 0, n_wg = 0, pages_used = 0;
    unsigned long long records = 0;
    unsigned batches = 0;
    void init(size_t n_bytes, unsigned grid, hipStream_t s);
    ~RecPoolOwner();
    RecPool dev() const;
    // aggregate the complete pages not aggregated yet into the word table (one global add per
    // distinct word per bin); final: every page (the workgroups have finished appending)
    void aggregate(bool final, const uint8_t* text, const WordCounts& wc, unsigned long long* fill, unsigned* status,
                   hipStream_t s);
};

unsigned count2_grid(size_t n_chunks);
// the long words k_count2 listed (R.lw) into the table; enqueued behind each k_count2 launch
void count_long_launch(const uint8_t* text, const WordCounts& wc, unsigned long long* fill, unsigned* status,
                       const RecPool& R, unsigned grid, hipStream_t s);
void count2_launch(const uint8_t* text, size_t lo, size_t hi, size_t c0, size_t nc, unsigned grid,
                   const WordCounts& wc, unsigned long long* fill, unsigned* status, unsigned long long* ntok,
                   const RecPool& R, const unsigned long long* gate, hipStream_t s, hipEvent_t e0, hipEvent_t e1);

}  // namespace bpe
