// Unique-word counting, byte-parallel (reference models/tokenizer/train.py:16-28: finditer with
// the GPT-2 pattern, then a dict count of the matches).
//
// k_count2: persistent workgroups stream 16 KiB chunks (+1 KiB halo) through LDS.  For every
// 64-byte block a thread evaluates the token-start predicate of tokstart.h on bit masks (no
// per-byte serial walk), so the chunk's pre-tokens are read off the masks: a token runs from one
// set bit to the next.  Each pre-token of >= 2 bytes is counted in a per-workgroup LDS cache of
// short words; a cache miss becomes a 24-byte RECORD {bytes lo, bytes hi, len | offset | count}
// appended to the workgroup's page of a record pool (no global atomics, no dependent loads).
// Words longer than 16 bytes, and records that find no pool space, go to the global table
// directly (stage.h table_add) as before.
//
// The records are then aggregated without random global traffic:
//   k_rec_hist    per page: histogram of the records over 4096 bins (top bits of the word hash);
//   k_rec_binscan per bin: exclusive scan over the pages (bin-major), bin totals;
//   k_rec_binbase one workgroup: bin bases;
//   k_rec_scatter per page: every record to its bin's run (LDS cursors);
//   k_rec_reduce  per bin: an LDS hash table sums the bin's records (a bin holds ~1/4096 of the
//                 distinct words), then one global table_add per distinct word.
// The global table is the same {key, count} table as before, so everything downstream (word
// collection, the multi-GPU exchange) is unchanged.
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "count.h"
#include "pretok.h"
#include "prims.h"
#include "stage.h"
#include "stage2.h"
#include "tokstart.h"

// the next chunk's loads issued before the mask phase (1, the default: 14 spilled VGPRs instead of
// 20, k_count2 58.2 vs 59.0 ms in two paired runs, profiles/r04/y_*) or after it (0)
#ifndef BPE355_COUNT_EARLY_PREFETCH
#define BPE355_COUNT_EARLY_PREFETCH 1
#endif

namespace bpe {

namespace {

// LDS word-cache entries (2-way sets).  512 entries keep the workgroup's LDS under 40 KB, so 4
// workgroups fit a CU, with k_count2 held to 128 VGPRs (4 waves/SIMD): 59.0 vs 65.5 ms at
// 11.9 GB for 5 % more records than 1024 entries at 3 waves/SIMD (tools/ab_count.sh; 256
// entries at 5 waves: 55.9 ms but 12 % more records and the same count phase)
constexpr int kCache2 = 512;
constexpr int kEpoch2 = 4;                        // chunks between cache evictions
constexpr unsigned kKeep2 = 2;                    // an entry stays if hit this often per epoch
constexpr unsigned kCntBits = 19;                 // record count field
// worst case of records a workgroup appends per chunk: every pre-token of >= 2 bytes that starts
// in it, plus one eviction of the whole cache and the final flush
constexpr unsigned kRecReserve = kChunk / 2 + 1 + 2 * kCache2;
constexpr int kBinBits = 12;
constexpr int kBins = 1 << kBinBits;

__device__ __forceinline__ unsigned rec_bin(uint64_t h) { return (unsigned)(h >> (64 - kBinBits)); }

template <bool kAligned>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_count2(const uint8_t* __restrict__ s, size_t lo, size_t n, size_t chunk0,
                                                size_t n_chunks, unsigned long long* __restrict__ kv,
                                                unsigned long long* __restrict__ pos, size_t mask,
                                                unsigned long long max_fill, unsigned long long* __restrict__ fill,
                                                unsigned* __restrict__ status, unsigned long long* __restrict__ n_tok,
                                                RecPool R, const unsigned long long* __restrict__ gate, int mode) {
    // a segment is counted only behind a clean validation of everything before it
    if (gate && *gate != ~0ULL) return;
    __shared__ uint64_t s_mask[kWords];
    __shared__ unsigned long long c_key[kCache2];
    __shared__ uint64_t c_lo[kCache2], c_hi[kCache2];
    __shared__ unsigned c_cnt[kCache2];
    __shared__ uint16_t c_mark[kCache2];
    __shared__ unsigned long long s_red[4];
    __shared__ int s_stop, s_page, s_old;
    __shared__ unsigned s_used;
    __shared__ unsigned s_ch[kCoarse];   // the current page's records per coarse bin
    __shared__ unsigned s_nlong;         // entries in this workgroup's long-word segment
    const int tid = threadIdx.x;
    for (int i = tid; i < kCache2; i += blockDim.x) { c_key[i] = 0; c_cnt[i] = 0; c_mark[i] = 0; }
    load_cls2(tid, blockDim.x);
    if (tid == 0) {
        s_page = R.on ? R.wg_page[blockIdx.x] : -1;
        s_used = R.on ? R.wg_used[blockIdx.x] : 0u;
        s_nlong = R.lw ? R.lw_n[blockIdx.x] : 0u;
    }
    if (tid < kCoarse) s_ch[tid] = R.on ? R.wg_ch[(size_t)blockIdx.x * kCoarse + tid] : 0u;
    unsigned long long ntok = 0, inserted = 0, n_miss = 0, n_long = 0;

    // a miss (or an evicted / flushed cache entry): a record in this workgroup's page, else the
    // global table
    auto spill = [&](uint64_t wl, uint64_t wh, size_t len, size_t gpos, unsigned long long c, uint64_t h) {
        const int pg = s_page;
        if (pg >= 0 && c < (1ULL << kCntBits)) {
            atomicAdd(&s_ch[h >> (64 - kCoarseBits)], 1u);
            const unsigned idx = atomicAdd(&s_used, 1u);
            const size_t gi = (size_t)pg * kPageRecs + idx;
            R.lo[gi] = wl;
            R.hi[gi] = wh;
            R.meta[gi] = (unsigned long long)len | ((unsigned long long)gpos << 5) | (c << 45);
            return;
        }
        bool ins;
        table_add(s, s, gpos, len, wl, wh, h, c, kv, pos, mask, status, &ins);
        inserted += ins;
    };

    uint4 pre[kSVec];
    if (blockIdx.x < n_chunks) fetch2<kAligned>(pre, s, n, (chunk0 + blockIdx.x) * kChunk, tid);
    for (size_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        __syncthreads();   // the previous chunk is done with the stage, the masks and the page
        store2(pre, tid);
        if (tid == 0) {
            s_stop = *(volatile unsigned long long*)fill > max_fill;
            s_old = -3;
            if (R.on && s_page != -1 && (s_page == -2 || s_used + kRecReserve > (unsigned)kPageRecs)) {
                if (s_page >= 0) R.page_used[s_page] = s_used;
                s_old = s_page;
                const unsigned pg = atomicAdd(R.n_pages, 1u);
                s_page = pg < R.max_pages ? (int)pg : -1;   // -1: the pool is spent
                s_used = 0;
            }
        }
        __syncthreads();
        if (s_old != -3 && tid < kCoarse) {   // the page left behind: its coarse histogram
            if (s_old >= 0) R.page_ch[(size_t)s_old * kCoarse + tid] = s_ch[tid];
            s_ch[tid] = 0;   // (ordered before this chunk's spills by the mask phase's barrier)
        }
        if (s_stop) {
            if (tid == 0) atomicOr(status, 1u);
            break;
        }
        const size_t base = (chunk0 + c) * kChunk;
        // build knob BPE355_COUNT_EARLY_PREFETCH: the next chunk's loads before the mask phase
        if (BPE355_COUNT_EARLY_PREFETCH && c + gridDim.x < n_chunks)
            fetch2<kAligned>(pre, s, n, (chunk0 + c + gridDim.x) * kChunk, tid);

        // ---- token-start masks: word w covers chunk bytes [64 w, 64 w + 64)
        auto mask_word = [&](int w) -> uint64_t {
            const int r0 = kPre + 64 * w - kStartPre;   // stage index of window byte 0
            const size_t blk = base + 64 * (size_t)w;
            const long long vhi = (long long)n - ((long long)blk - kStartPre);
            uint64_t m = token_starts64<DevTab>(LdsWin{r0}, (int)(vhi < kStartWin ? (vhi > 0 ? vhi : 0) : kStartWin));
            if (blk + 64 <= lo) {
                m = 0;                              // before the text (segment) start
            } else if (blk <= lo) {
                const int k = (int)(lo - blk);      // the text starts here
                m = (m & (~0ULL << k)) | (1ULL << k);
            }
            return m;
        };
        s_mask[tid] = mask_word(tid);
        // (knob 0: the next chunk's loads fly during the token phase only)
        if (!BPE355_COUNT_EARLY_PREFETCH && c + gridDim.x < n_chunks)
            fetch2<kAligned>(pre, s, n, (chunk0 + c + gridDim.x) * kChunk, tid);
        __syncthreads();

        // ---- the pre-tokens that start in this thread's 64 bytes
        // (analysis knob BPE355_COUNT_MODE, timing only -- counts are then incomplete: 1 masks
        // only, 2 + token bounds, 3 + packing and hashing, 4 + the LDS cache, misses dropped; 5 all
        // but the words longer than kInline)
        if (mode == 1) continue;
        const size_t rem = n > base ? n - base : 0;
        const uint32_t tend = rem < (size_t)kWin ? (uint32_t)rem : (uint32_t)kWin;   // staged text end
        uint64_t m = s_mask[tid];
        while (m) {
            const uint32_t r = 64u * tid + (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            size_t e;   // end, relative to base
            if (m) {
                e = 64u * tid + (uint32_t)__builtin_ctzll(m);
            } else {
                e = ~(size_t)0;
                for (int w = tid + 1; w < kWords; ++w) {
                    const uint64_t x = s_mask[w];
                    if (x) { e = 64u * w + (uint32_t)__builtin_ctzll(x); break; }
                }
                if (e == ~(size_t)0) {
                    // the chunk's last pre-token: the serial scanner over the staged halo, trusted
                    // when it stops clear of the staged end (it looks one character ahead), else
                    // over the text itself
                    e = token_end(StageText{}, tend, r);
                    if (e + 4 > tend && tend < rem) e = token_end(s, n, base + r) - base;
                }
            }
            const size_t len = e - r;
            if (len < 2) continue;
            ++ntok;
            if (mode == 2) continue;
            const size_t gpos = base + r;
            if (len > (size_t)kInline) {
                ++n_long;
                if (mode == 5) continue;
                // listed for k_count_long: hashing it here (byte loads from HBM, a byte-wise
                // compare in the table) stalled the whole wave on one lane -- 12 of 47.5 ms of
                // this kernel at 11.9 GB for 0.3 % of the pre-tokens (BPE355_COUNT_MODE=5)
                if (R.lw && len < kMaxPretok) {
                    const unsigned li = atomicAdd(&s_nlong, 1u);
                    if (li < R.lw_per_wg) {
                        R.lw[(size_t)blockIdx.x * R.lw_per_wg + li] = (unsigned long long)gpos | ((unsigned long long)len << 40);
                        continue;
                    }
                }
                bool ins;
                table_add(s, s, gpos, len, 0, 0, hash_word(s, gpos, len), 1, kv, pos, mask, status, &ins);
                inserted += ins;
                continue;
            }
            uint64_t wl, wh;
            pack_stage(kPre + (int)r, (int)len, wl, wh);
            const uint64_t h = short_hash(wl, wh, len);
            if (mode == 3) { n_miss += h & 1; continue; }
            const unsigned ls = (unsigned)(h >> 40) & (kCache2 - 2);
            const unsigned long long mine = ((unsigned long long)len << 40) | (gpos + 1);
            bool done = false;
            for (int way = 0; way < 2 && !done; ++way) {
                const unsigned sl = ls + way;
                unsigned long long k = c_key[sl];
                if (k == 0) {
                    k = atomicCAS(&c_key[sl], 0ULL, kBusy);
                    if (k == 0) {   // claimed: bytes first (drained), then publish the key
                        c_lo[sl] = wl;
                        c_hi[sl] = wh;
                        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        atomicExch(&c_key[sl], mine);
                        atomicAdd(&c_cnt[sl], 1u);
                        done = true;
                        break;
                    }
                }
                if (k != kBusy && (k >> 40) == len) {
                    __asm__ volatile("" ::: "memory");
                    if (c_lo[sl] == wl && c_hi[sl] == wh) {
                        atomicAdd(&c_cnt[sl], 1u);
                        done = true;
                    }
                }
            }
            if (!done) {
                ++n_miss;
                if (mode != 4) spill(wl, wh, len, gpos, 1, h);
            }
        }
        // epoch end: entries hit fewer than kKeep2 times since the last epoch leave the cache
        if ((c - blockIdx.x) / gridDim.x % kEpoch2 == kEpoch2 - 1) {
            __syncthreads();
            for (int i = tid; i < kCache2; i += blockDim.x) {
                const unsigned long long k = c_key[i];
                if (k == 0 || k == kBusy) continue;
                const unsigned cc = c_cnt[i];
                if ((uint16_t)(cc - c_mark[i]) >= kKeep2) {
                    c_mark[i] = (uint16_t)cc;
                    continue;
                }
                spill(c_lo[i], c_hi[i], (size_t)(k >> 40), (size_t)(k & kOffMask) - 1, cc,
                      short_hash(c_lo[i], c_hi[i], (size_t)(k >> 40)));
                c_key[i] = 0;
                c_cnt[i] = 0;
                c_mark[i] = 0;
            }
        }
        const unsigned long long ins = wave_sum(inserted);   // this chunk's new keys
        inserted = 0;
        if ((tid & 63) == 0) s_red[tid >> 6] = ins;
        __syncthreads();
        if (tid == 0) {
            const unsigned long long b = s_red[0] + s_red[1] + s_red[2] + s_red[3];
            if (b) atomicAdd(fill, b);
        }
    }
    __syncthreads();
    for (int i = tid; i < kCache2; i += blockDim.x) {   // flush the cache
        const unsigned long long k = c_key[i];
        if (k == 0 || k == kBusy) continue;
        spill(c_lo[i], c_hi[i], (size_t)(k >> 40), (size_t)(k & kOffMask) - 1, c_cnt[i],
              short_hash(c_lo[i], c_hi[i], (size_t)(k >> 40)));
    }
    __syncthreads();
    if (tid == 0 && R.on) {   // the next launch's workgroup continues this page
        R.wg_page[blockIdx.x] = s_page;
        R.wg_used[blockIdx.x] = s_used;
    }
    if (tid == 0 && R.lw) R.lw_n[blockIdx.x] = s_nlong < R.lw_per_wg ? s_nlong : R.lw_per_wg;
    if (tid < kCoarse && R.on) R.wg_ch[(size_t)blockIdx.x * kCoarse + tid] = s_ch[tid];
    ntok = wave_sum(ntok);
    inserted = wave_sum(inserted);
    n_miss = wave_sum(n_miss);
    n_long = wave_sum(n_long);
    if ((tid & 63) == 0) {
        if (ntok) atomicAdd(n_tok, ntok);
        if (n_miss) atomicAdd(n_tok + 1, n_miss);   // diagnostics (BPE355_TRACE)
        if (n_long) atomicAdd(n_tok + 2, n_long);
        if (inserted) atomicAdd(fill, inserted);
    }
}

constexpr int kLongSlots = 2048;   // k_count_long's LDS table (a segment holds ~1-3 K distinct words)
constexpr int kLongProbe = 16;

// The long words of counting workgroup b's segment into the table.  The frequent ones are
// whitespace runs (at 2 GB of the bench corpus twelve words of 21-32 bytes make 480 K of the 855 K
// long pre-tokens), so adding them one by one serialises on a few table slots (same-address
// atomics): they are summed per segment first in an LDS table keyed by (hash, length), an
// occurrence joining an entry only when its bytes equal the entry's first occurrence.  Then one
// table add per entry.  The segment is emptied for the next k_count2 launch.
__global__ void __launch_bounds__(256) k_count_long(const uint8_t* __restrict__ s, RecPool R,
                                                    unsigned long long* __restrict__ kv,
                                                    unsigned long long* __restrict__ pos, size_t mask,
                                                    unsigned long long* __restrict__ fill, unsigned* __restrict__ status) {
    __shared__ unsigned long long t_h[kLongSlots];   // the word hash (0: free, ~0: being claimed)
    __shared__ unsigned long long t_pos[kLongSlots];
    __shared__ unsigned t_len[kLongSlots], t_cnt[kLongSlots];
    constexpr unsigned long long kClaim = ~0ULL;
    for (int i = threadIdx.x; i < kLongSlots; i += blockDim.x) { t_h[i] = 0; t_cnt[i] = 0; }
    __syncthreads();
    const unsigned b = blockIdx.x;
    const unsigned n = R.lw_n[b];
    unsigned long long inserted = 0;
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long e = R.lw[(size_t)b * R.lw_per_wg + i];
        const size_t gpos = (size_t)(e & kOffMask), len = (size_t)(e >> 40);
        const uint64_t h = hash_word(s, gpos, len);
        bool done = false;
        if (h != 0 && h != kClaim) {
            unsigned sl = (unsigned)(h >> 24) & (kLongSlots - 1);
            for (int probe = 0; probe < kLongProbe && !done; ++probe, sl = (sl + 1) & (kLongSlots - 1)) {
                unsigned long long k = t_h[sl];
                if (k == 0) {
                    k = atomicCAS(&t_h[sl], 0ULL, kClaim);
                    if (k == 0) {   // claimed: position and length first (drained), then the hash
                        t_pos[sl] = gpos;
                        t_len[sl] = (unsigned)len;
                        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        atomicExch(&t_h[sl], h);
                        atomicAdd(&t_cnt[sl], 1u);
                        done = true;
                        break;
                    }
                }
                // (a slot being claimed is passed over: the word may then sit twice; the table merges)
                if (k == h && t_len[sl] == (unsigned)len && bytes_equal(s, t_pos[sl], gpos, len)) {
                    atomicAdd(&t_cnt[sl], 1u);
                    done = true;
                }
            }
        }
        if (!done) {
            bool ins;
            table_add(s, s, gpos, len, 0, 0, h, 1, kv, pos, mask, status, &ins);
            inserted += ins;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kLongSlots; i += blockDim.x) {
        const unsigned long long h = t_h[i];
        if (h == 0 || h == kClaim) continue;
        bool ins;
        table_add(s, s, (size_t)t_pos[i], (size_t)t_len[i], 0, 0, h, t_cnt[i], kv, pos, mask, status, &ins);
        inserted += ins;
    }
    inserted = wave_sum(inserted);
    if ((threadIdx.x & 63) == 0 && inserted) atomicAdd(fill, inserted);
    if (threadIdx.x == 0) R.lw_n[b] = 0u;   // (n was read by every thread before the first barrier)
}

// ------------------------------------------------------------------ record aggregation
__device__ __forceinline__ uint64_t rec_hash(uint64_t lo, uint64_t hi, uint64_t meta) {
    return short_hash(lo, hi, (size_t)(meta & 31u));
}

// the pages' last fill levels (each workgroup's current page)
__global__ void k_rec_retire(RecPool R, unsigned n_wg) {
    const unsigned b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_wg) return;
    const int pg = R.wg_page[b];
    if (pg < 0) return;
    R.page_used[pg] = R.wg_used[b];
    for (int c = 0; c < kCoarse; ++c) R.page_ch[(size_t)pg * kCoarse + c] = R.wg_ch[(size_t)b * kCoarse + c];
}

// pages a counting workgroup still appends to (not complete yet)
__global__ void k_rec_hold(RecPool R, unsigned n_wg, unsigned* __restrict__ held) {
    const unsigned b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_wg) return;
    const int pg = R.wg_page[b];
    if (pg >= 0) held[pg] = 1u;
}

// complete pages not aggregated yet -> list (and marked done); held flags cleared behind
__global__ void k_rec_pick(RecPool R, unsigned* __restrict__ held, unsigned* __restrict__ done,
                           unsigned* __restrict__ list, unsigned* __restrict__ list_n) {
    const unsigned p = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned np = *R.n_pages < R.max_pages ? *R.n_pages : R.max_pages;
    bool take = false;
    if (p < np) {
        take = !held[p] && !done[p];
        held[p] = 0u;
        if (take) done[p] = 1u;
    }
    const unsigned i = wave_append(take, list_n);
    if (take) list[i] = p;
}

// ---- two-level partition of the records by bin (the top 12 bits of the word hash)
// Level 1 splits the pool's pages by the top 6 bits (the per-page histogram came from k_count2),
// level 2 splits each coarse bin's run, in tiles, by the next 6.  Both move records through an
// LDS-sorted tile of kPartTile records, so each bin's share of a tile (~64 records) leaves as
// one contiguous run: whole lines, not the scattered 8-byte writes of a direct per-record scatter.
constexpr int kPartTile = 4096;
constexpr int kL2Tile = 65536;   // records per level-2 work item

// per coarse bin c: exclusive scan of its per-page counts over the pages (offsets within the bin)
__global__ void __launch_bounds__(1024) k_rec_cscan(const unsigned* __restrict__ page_ch,
                                                    const unsigned* __restrict__ list,
                                                    const unsigned* __restrict__ list_n,
                                                    unsigned* __restrict__ coff, unsigned long long* __restrict__ ctot) {
    typedef rocprim::block_scan<unsigned, 1024> Scan;
    __shared__ typename Scan::storage_type tmp;
    __shared__ unsigned carry;
    const unsigned c = blockIdx.x;
    const unsigned n_pages = *list_n;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (unsigned b0 = 0; b0 < n_pages; b0 += 1024) {
        const unsigned i = b0 + threadIdx.x;
        const unsigned v = i < n_pages ? page_ch[(size_t)list[i] * kCoarse + c] : 0u;
        unsigned ex, agg;
        Scan().exclusive_scan(v, ex, 0u, agg, tmp);
        const unsigned cb = carry;
        if (i < n_pages) coff[(size_t)i * kCoarse + c] = cb + ex;
        __syncthreads();
        if (threadIdx.x == 0) carry = cb + agg;
        __syncthreads();
    }
    if (threadIdx.x == 0) ctot[c] = carry;
}

// exclusive scan of n <= 4096 totals (one workgroup); base[n] = their sum
__global__ void __launch_bounds__(1024) k_rec_base(const unsigned long long* __restrict__ tot, int n,
                                                   unsigned long long* __restrict__ base) {
    typedef rocprim::block_scan<unsigned long long, 1024> Scan;
    __shared__ typename Scan::storage_type tmp;
    constexpr int per = 4;
    unsigned long long v[per], ex[per], agg;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        const int i = threadIdx.x * per + k;
        v[k] = i < n ? tot[i] : 0ULL;
    }
    Scan().exclusive_scan(v, ex, 0ULL, agg, tmp);
#pragma unroll
    for (int k = 0; k < per; ++k) {
        const int i = threadIdx.x * per + k;
        if (i < n) base[i] = ex[k];
    }
    if (threadIdx.x == 0) base[n] = agg;
}

// position g of a run laid over pool pages (dpage: the pages in order), or of a flat array
__device__ __forceinline__ size_t paged(unsigned long long g, const unsigned* __restrict__ dpage) {
    static_assert(kPageRecs == 1 << 16, "page-indirect positions");
    return dpage ? (size_t)dpage[g >> 16] * kPageRecs + (size_t)(g & (kPageRecs - 1)) : (size_t)g;
}

// one wave: the batch's coarse-bin bases (cbase[kCoarse] = its records), the level-2 tiles over
// each bin's run (tile0[c]: bin c's first tile; n_tiles) -- built on the device, so a batch needs
// no host round trip
__global__ void __launch_bounds__(64) k_rec_tiles(const unsigned long long* __restrict__ ctot,
                                                  unsigned long long* __restrict__ cbase, L2Tile* __restrict__ tiles,
                                                  unsigned* __restrict__ tile0, unsigned* __restrict__ n_tiles,
                                                  unsigned long long* __restrict__ records) {
    const unsigned c = threadIdx.x;
    const unsigned long long cnt = ctot[c];
    const unsigned nt = (unsigned)((cnt + kL2Tile - 1) / kL2Tile);
    unsigned long long x = cnt;
    unsigned y = nt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long xu = __shfl_up(x, o);
        const unsigned yu = __shfl_up(y, o);
        if (c >= (unsigned)o) { x += xu; y += yu; }
    }
    const unsigned long long b = x - cnt;
    const unsigned t = y - nt;
    cbase[c] = b;
    tile0[c] = t;
    if (c == 63) {
        cbase[kCoarse] = x;
        tile0[kCoarse] = y;
        *n_tiles = y;
        *records += x;
    }
    for (unsigned j = 0; j < nt; ++j) {
        const unsigned long long a = (unsigned long long)j * kL2Tile;
        tiles[t + j] = L2Tile{b + a, (unsigned)(cnt - a < (unsigned long long)kL2Tile ? cnt - a : kL2Tile), c};
    }
}

// records [s0, s0 + len) of (slo, shi, sme) to dest + cur[bin] (cur: LDS, advanced), bin = the 6
// bits of the hash at `shift`, one LDS-sorted tile at a time
// dfine (level 1): each record's next 6 hash bits, its level-2 bin, into a byte array beside the
// destination, so the level-2 histogram reads one byte per record instead of 24
__device__ __forceinline__ void part_tiles(const uint64_t* __restrict__ slo, const uint64_t* __restrict__ shi,
                                           const uint64_t* __restrict__ sme, size_t s0, size_t len, int shift,
                                           unsigned long long* cur, uint64_t* __restrict__ dlo,
                                           uint64_t* __restrict__ dhi, uint64_t* __restrict__ dme,
                                           const unsigned* __restrict__ dpage = nullptr,
                                           uint8_t* __restrict__ dfine = nullptr) {
    __shared__ uint64_t st_lo[kPartTile], st_hi[kPartTile], st_me[kPartTile];
    __shared__ uint8_t st_bin[kPartTile], st_fine[kPartTile];
    __shared__ unsigned t_cnt[kCoarse], t_off[kCoarse], t_cur[kCoarse];
    const int tid = threadIdx.x;
    constexpr int U = kPartTile / 1024;
    if (tid < kCoarse) { t_cnt[tid] = 0; t_cur[tid] = 0; }
    __syncthreads();
    for (size_t t0 = 0; t0 < len; t0 += kPartTile) {
        const unsigned nt = (unsigned)(len - t0 < (size_t)kPartTile ? len - t0 : kPartTile);
        uint64_t a[U], b[U], m[U];
        unsigned bin[U], fine[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned q = tid + u * 1024;
            bin[u] = kCoarse;
            fine[u] = 0;
            if (q < nt) {
                const size_t i = s0 + t0 + q;
                a[u] = slo[i]; b[u] = shi[i]; m[u] = sme[i];
                const uint64_t h = rec_hash(a[u], b[u], m[u]);
                bin[u] = (unsigned)(h >> shift) & (kCoarse - 1);
                fine[u] = (unsigned)(h >> (shift - kCoarseBits)) & (kCoarse - 1);
                atomicAdd(&t_cnt[bin[u]], 1u);
            }
        }
        __syncthreads();
        if (tid < 64) {   // one wave: the tile's bin offsets
            const unsigned v = t_cnt[tid];
            unsigned x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned y = __shfl_up(x, o);
                if (tid >= o) x += y;
            }
            t_off[tid] = x - v;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (bin[u] == kCoarse) continue;
            const unsigned q = t_off[bin[u]] + atomicAdd(&t_cur[bin[u]], 1u);
            st_lo[q] = a[u]; st_hi[q] = b[u]; st_me[q] = m[u]; st_bin[q] = (uint8_t)bin[u];
            st_fine[q] = (uint8_t)fine[u];
        }
        __syncthreads();
        for (unsigned q = tid; q < nt; q += 1024) {   // consecutive q of one bin: one run
            const unsigned bb = st_bin[q];
            const size_t g = paged(cur[bb] + (q - t_off[bb]), dpage);
            dlo[g] = st_lo[q]; dhi[g] = st_hi[q]; dme[g] = st_me[q];
            if (dfine) dfine[g] = st_fine[q];
        }
        __syncthreads();
        if (tid < kCoarse) { cur[tid] += t_cnt[tid]; t_cnt[tid] = 0; t_cur[tid] = 0; }
        __syncthreads();
    }
}

// level 1: one workgroup per listed pool page
__global__ void __launch_bounds__(1024) k_rec_part1(RecPool R, const unsigned* __restrict__ list,
                                                    const unsigned* __restrict__ list_n,
                                                    const unsigned* __restrict__ coff,
                                                    const unsigned long long* __restrict__ cbase,
                                                    uint64_t* __restrict__ dlo, uint64_t* __restrict__ dhi,
                                                    uint64_t* __restrict__ dme, uint8_t* __restrict__ dfine) {
    __shared__ unsigned long long cur[kCoarse];
    if (blockIdx.x >= *list_n) return;   // (the grid is sized for every page)
    const unsigned pg = list[blockIdx.x];
    if (threadIdx.x < kCoarse) cur[threadIdx.x] = cbase[threadIdx.x] + coff[(size_t)blockIdx.x * kCoarse + threadIdx.x];
    part_tiles(R.lo, R.hi, R.meta, (size_t)pg * kPageRecs, R.page_used[pg], 64 - kCoarseBits, cur, dlo, dhi, dme,
               nullptr, dfine);
}

// level 2, histogram: per tile of a coarse bin's run, records per fine bin
__global__ void __launch_bounds__(1024) k_rec_fhist(const uint8_t* __restrict__ rfine, const L2Tile* __restrict__ tiles,
                                                    const unsigned* __restrict__ n_tiles, unsigned* __restrict__ fhist) {
    __shared__ unsigned h[kCoarse];
    if (blockIdx.x >= *n_tiles) return;   // (the grid is sized for the largest batch)
    const L2Tile T = tiles[blockIdx.x];
    if (threadIdx.x < kCoarse) h[threadIdx.x] = 0;
    __syncthreads();
    constexpr int U = 4;
    for (unsigned q0 = threadIdx.x; q0 < T.len; q0 += U * 1024) {
        unsigned f[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned q = q0 + u * 1024;
            f[u] = q < T.len ? (unsigned)rfine[T.start + q] : kCoarse;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (f[u] != kCoarse) atomicAdd(&h[f[u]], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kCoarse) fhist[(size_t)blockIdx.x * kCoarse + threadIdx.x] = h[threadIdx.x];
}

// level 2, offsets: per (coarse c, fine f) an exclusive scan over c's tiles; totals per final bin
__global__ void __launch_bounds__(256) k_rec_fscan(unsigned* __restrict__ fhist, const unsigned* __restrict__ tile0,
                                                   unsigned long long* __restrict__ ftot) {
    typedef rocprim::block_scan<unsigned, 256> Scan;
    __shared__ typename Scan::storage_type tmp;
    __shared__ unsigned carry;
    const unsigned c = blockIdx.x / kCoarse, f = blockIdx.x % kCoarse;
    const unsigned a = tile0[c], e = tile0[c + 1];
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (unsigned b0 = a; b0 < e; b0 += 256) {
        const unsigned i = b0 + threadIdx.x;
        const unsigned v = i < e ? fhist[(size_t)i * kCoarse + f] : 0u;
        unsigned ex, agg;
        Scan().exclusive_scan(v, ex, 0u, agg, tmp);
        const unsigned cb = carry;
        if (i < e) fhist[(size_t)i * kCoarse + f] = cb + ex;
        __syncthreads();
        if (threadIdx.x == 0) carry = cb + agg;
        __syncthreads();
    }
    if (threadIdx.x == 0) ftot[blockIdx.x] = carry;
}

// level 2, move: one workgroup per tile, into the final bins
__global__ void __launch_bounds__(1024) k_rec_part2(const uint64_t* __restrict__ rlo, const uint64_t* __restrict__ rhi,
                                                    const uint64_t* __restrict__ rme, const L2Tile* __restrict__ tiles,
                                                    const unsigned* __restrict__ n_tiles,
                                                    const unsigned* __restrict__ foff,
                                                    const unsigned long long* __restrict__ base,
                                                    uint64_t* __restrict__ dlo, uint64_t* __restrict__ dhi,
                                                    uint64_t* __restrict__ dme, const unsigned* __restrict__ dpage) {
    __shared__ unsigned long long cur[kCoarse];
    if (blockIdx.x >= *n_tiles) return;
    const L2Tile T = tiles[blockIdx.x];
    if (threadIdx.x < kCoarse)
        cur[threadIdx.x] = base[T.coarse * kCoarse + threadIdx.x] + foff[(size_t)blockIdx.x * kCoarse + threadIdx.x];
    part_tiles(rlo, rhi, rme, T.start, T.len, 64 - 2 * kCoarseBits, cur, dlo, dhi, dme, dpage);
}

constexpr int kRedSlots = 4096;   // LDS table of k_rec_reduce (a bin holds ~1/4096 of the words)
constexpr int kRedProbe = 64;

// per bin: sum the records in LDS, then one global table_add per distinct word
__global__ void __launch_bounds__(1024) k_rec_reduce(const uint64_t* __restrict__ rlo, const uint64_t* __restrict__ rhi,
                                                     const uint64_t* __restrict__ rmeta,
                                                     const unsigned long long* __restrict__ base,
                                                     const unsigned* __restrict__ dpage,
                                                     const uint8_t* __restrict__ s, unsigned long long* __restrict__ kv,
                                                     unsigned long long* __restrict__ pos, size_t mask,
                                                     unsigned long long* __restrict__ fill, unsigned* __restrict__ status) {
    __shared__ unsigned long long t_key[kRedSlots];   // len << 40 | offset + 1 (kBusy while claimed)
    __shared__ uint64_t t_lo[kRedSlots], t_hi[kRedSlots];
    __shared__ unsigned long long t_cnt[kRedSlots];
    for (int i = threadIdx.x; i < kRedSlots; i += blockDim.x) { t_key[i] = 0; t_cnt[i] = 0; }
    __syncthreads();
    const unsigned long long b0 = base[blockIdx.x], b1 = base[blockIdx.x + 1];
    unsigned long long inserted = 0;
    constexpr int U = 4;
    for (unsigned long long i0 = b0 + threadIdx.x; i0 < b1; i0 += U * blockDim.x) {
      uint64_t ul[U], uh[U], um[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
          const unsigned long long i = i0 + (unsigned long long)u * blockDim.x;
          if (i < b1) {
              const size_t g = paged(i, dpage);
              ul[u] = rlo[g]; uh[u] = rhi[g]; um[u] = rmeta[g];
          }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i0 + (unsigned long long)u * blockDim.x >= b1) break;
        const uint64_t wl = ul[u], wh = uh[u], m = um[u];
        const size_t len = (size_t)(m & 31u);
        const size_t off = (size_t)((m >> 5) & kOffMask);
        const unsigned long long c = m >> 45;
        const uint64_t h = short_hash(wl, wh, len);
        const unsigned long long mine = ((unsigned long long)len << 40) | (off + 1);
        unsigned sl = (unsigned)(h >> 20) & (kRedSlots - 1);
        bool done = false;
        for (int probe = 0; probe < kRedProbe && !done; ++probe, sl = (sl + 1) & (kRedSlots - 1)) {
            unsigned long long k = t_key[sl];
            if (k == 0) {
                k = atomicCAS(&t_key[sl], 0ULL, kBusy);
                if (k == 0) {
                    t_lo[sl] = wl;
                    t_hi[sl] = wh;
                    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    atomicExch(&t_key[sl], mine);
                    atomicAdd(&t_cnt[sl], c);
                    done = true;
                    break;
                }
            }
            if (k != kBusy && (k >> 40) == len) {   // (a slot being claimed is passed over: the
                __asm__ volatile("" ::: "memory");  // word may then sit twice; the table merges)
                if (t_lo[sl] == wl && t_hi[sl] == wh) {
                    atomicAdd(&t_cnt[sl], c);
                    done = true;
                }
            }
        }
        if (!done) {   // the LDS table is full here: straight to the global table
            bool ins;
            table_add(s, s, off, len, wl, wh, h, c, kv, pos, mask, status, &ins);
            inserted += ins;
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kRedSlots; i += blockDim.x) {
        const unsigned long long k = t_key[i];
        if (k == 0) continue;
        const size_t len = (size_t)(k >> 40), off = (size_t)(k & kOffMask) - 1;
        const uint64_t wl = t_lo[i], wh = t_hi[i];
        bool ins;
        table_add(s, s, off, len, wl, wh, short_hash(wl, wh, len), t_cnt[i], kv, pos, mask, status, &ins);
        inserted += ins;
    }
    inserted = wave_sum(inserted);
    if ((threadIdx.x & 63) == 0 && inserted) atomicAdd(fill, inserted);
}

int count2_per_cu() {
    static int per_cu = 0;
    if (!per_cu)
        BPE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_count2<true>, 256, kStage));
    return std::max(per_cu, 1);
}

}  // namespace

unsigned count2_grid(size_t n_chunks) {
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        BPE_HIP(hipGetDevice(&dev));
        BPE_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    (void)n_chunks;
    unsigned grid = (unsigned)count2_per_cu() * (unsigned)std::max(1, n_cu);
    if (const char* e = std::getenv("BPE355_STREAM_WG"))   // test knob: fewer workgroups, each
        grid = std::max(1u, std::min(grid, (unsigned)std::atoi(e)));   // streaming many chunks
    return grid;
}

void count2_launch(const uint8_t* text, size_t lo, size_t hi, size_t c0, size_t nc, unsigned grid,
                   const WordCounts& wc, unsigned long long* fill, unsigned* status, unsigned long long* ntok,
                   const RecPool& R, const unsigned long long* gate, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    static const int mode = std::getenv("BPE355_COUNT_MODE") ? std::atoi(std::getenv("BPE355_COUNT_MODE")) : 0;
    const bool aligned = (reinterpret_cast<uintptr_t>(text) & 15u) == 0;
    auto kern = aligned ? k_count2<true> : k_count2<false>;
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(256), kStage, s, e0, e1, 0, text, lo, hi, c0, nc, wc.kv.p, wc.pos.p,
                          wc.cap - 1, (unsigned long long)(wc.cap / 2), fill, status, ntok, R, gate, mode);
    BPE_HIP(hipGetLastError());
}

void count_long_launch(const uint8_t* text, const WordCounts& wc, unsigned long long* fill, unsigned* status,
                       const RecPool& R, unsigned grid, hipStream_t s) {
    if (!R.lw) return;
    hipLaunchKernelGGL(k_count_long, dim3(grid), dim3(256), 0, s, text, R, wc.kv.p, wc.pos.p, wc.cap - 1, fill, status);
    BPE_HIP(hipGetLastError());
}

namespace {
struct ScratchArrays {
    std::mutex m;
    std::vector<std::unique_ptr<Arrays3>> free_;
};
ScratchArrays& scratch() {
    static ScratchArrays* p = new ScratchArrays;   // lives as long as the process
    return *p;
}
}  // namespace

std::unique_ptr<Arrays3> scratch_take(size_t cap) {
    int dev = 0;
    BPE_HIP(hipGetDevice(&dev));
    std::unique_ptr<Arrays3> x;
    {
        std::lock_guard<std::mutex> g(scratch().m);
        auto& f = scratch().free_;
        size_t best = f.size();
        for (size_t i = 0; i < f.size(); ++i)   // the smallest free set of this device that fits
            if (f[i]->dev == dev && f[i]->cap >= cap && (best == f.size() || f[i]->cap < f[best]->cap)) best = i;
        if (best == f.size())                   // none fits: replace this device's largest
            for (size_t i = 0; i < f.size(); ++i)
                if (f[i]->dev == dev && (best == f.size() || f[i]->cap > f[best]->cap)) best = i;
        if (best < f.size()) {
            x = std::move(f[best]);
            f.erase(f.begin() + best);
        }
    }
    if (x && x->cap >= cap) return x;
    x.reset();
    x = std::make_unique<Arrays3>();
    x->dev = dev;
    x->cap = cap;
    try {
        x->a.alloc(cap);
        x->b.alloc(cap);
        x->c.alloc(cap);
    } catch (const Error& e) {
        if (e.code != BPE_E_NOMEM) throw;
        // the cache holds this device's other free sets: give them back and try once more
        x->a.release(); x->b.release(); x->c.release(); x->d.release();
        scratch_release(dev);
        x->a.alloc(cap);
        x->b.alloc(cap);
        x->c.alloc(cap);
    }
    return x;
}

size_t scratch_cached_bytes(int dev) {
    std::lock_guard<std::mutex> g(scratch().m);
    size_t b = 0;
    for (auto& f : scratch().free_)
        if (f->dev == dev) b += f->bytes();
    return b;
}

size_t scratch_release(int dev) {
    std::vector<std::unique_ptr<Arrays3>> drop;
    size_t bytes = 0;
    {
        std::lock_guard<std::mutex> g(scratch().m);
        auto& f = scratch().free_;
        for (size_t i = 0; i < f.size();)
            if (dev < 0 || f[i]->dev == dev) {
                bytes += f[i]->bytes();
                drop.push_back(std::move(f[i]));
                f.erase(f.begin() + i);
            } else {
                ++i;
            }
    }
    if (drop.empty()) return bytes;
    int cur = 0;
    BPE_HIP(hipGetDevice(&cur));
    for (auto& x : drop) {   // hipFree outside the lock, on the arrays' own device
        (void)hipSetDevice(x->dev);
        x.reset();
    }
    BPE_HIP(hipSetDevice(cur));
    return bytes;
}

void scratch_give(std::unique_ptr<Arrays3> x) {
    if (!x) return;
    std::lock_guard<std::mutex> g(scratch().m);
    scratch().free_.push_back(std::move(x));
}

RecPoolOwner::~RecPoolOwner() {
    scratch_give(std::move(rec));
    scratch_give(std::move(B));
}

void RecPoolOwner::init(size_t n_bytes, unsigned grid, hipStream_t s) {
    // pool: ~1 record per 10 corpus bytes (the bench corpus spills one per 15); when it runs out,
    // the remaining misses go to the global table (correct, slower)
    size_t want = std::max<size_t>(n_bytes / 10, (size_t)grid * kPageRecs);
    if (const char* e = std::getenv("BPE355_REC_POOL")) want = (size_t)std::atof(e);   // test knob: records
    // The pool and the aggregation's level-1 copy take 48 B per record (two sets of three u64
    // arrays).  Cap them by the device memory that is free (plus the cache's free sets, which
    // scratch_take reuses or hands back), keeping a reserve for the word table and the merge
    // loop; a pool that cannot hold one page per counting workgroup is not worth having: the
    // counter then sends its misses to the global table (R.on = 0: correct, slower).
    int dev = 0;
    BPE_HIP(hipGetDevice(&dev));
    size_t free_b = 0, total_b = 0;
    BPE_HIP(hipMemGetInfo(&free_b, &total_b));
    const size_t avail = free_b + scratch_cached_bytes(dev);
    const size_t reserve = std::max<size_t>(total_b / 16, n_bytes / 2);
    size_t fit = avail > reserve ? (avail - reserve) / (6 * sizeof(uint64_t) + 1) : 0;
    if (const char* e = std::getenv("BPE355_REC_POOL_FIT")) fit = (size_t)std::atof(e);   // test knob
    if (fit < want) {
        if (fit < (size_t)grid * kPageRecs / 4)
            throw Error{BPE_E_NOMEM, "record pool: " + std::to_string(avail) + " bytes of device memory free"};
        want = fit;
    }
    max_pages = (unsigned)std::max<size_t>(1, std::min<size_t>((want + kPageRecs - 1) / kPageRecs, 1u << 30));
    const size_t cap = (size_t)max_pages * kPageRecs;
    if (std::getenv("BPE355_REC_POOL_FAIL"))   // test knob: the pool's allocation fails
        throw Error{BPE_E_NOMEM, "record pool allocation failed (BPE355_REC_POOL_FAIL)"};
    rec = scratch_take(cap);
    page_used.alloc(max_pages);
    page_ch.alloc((size_t)max_pages * kCoarse);
    n_pages.alloc(1);
    wg_page.alloc(grid);
    wg_used.alloc(grid);
    wg_ch.alloc((size_t)grid * kCoarse);
    BPE_HIP(hipMemsetAsync(wg_ch.p, 0, 4ull * grid * kCoarse, s));
    held.alloc(max_pages);
    done.alloc(max_pages);
    // long-word segments: ~1 entry per KiB of text (the bench corpus has one per 2.3 KiB); a
    // full segment sends the rest of its workgroup's long words to the table directly
    lw_per_wg = (unsigned)std::min<size_t>(1u << 24, std::max<size_t>(1024, n_bytes / 1024 / grid + 1));
    if (const char* e = std::getenv("BPE355_LONG_SEG")) lw_per_wg = (unsigned)std::max(1, std::atoi(e));   // test knob
    lw.alloc((size_t)lw_per_wg * grid);
    lw_n.alloc(grid);
    BPE_HIP(hipMemsetAsync(lw_n.p, 0, 4ull * grid, s));
    // the aggregation's buffers, sized for one batch of every page (no allocation while the
    // file path aggregates between segment copies): level 1 lands in B, level 2 back in the pages
    B = scratch_take(cap);
    if (B->d.n < cap) B->d.alloc(cap);   // (kept with the set across calls)
    max_tiles = max_pages + kCoarse;
    coff.alloc((size_t)kCoarse * max_pages);
    ctot.alloc(kCoarse);
    cbase.alloc(kCoarse + 1);
    d_tl.alloc(max_tiles);
    d_t0.alloc(kCoarse + 1);
    fhist.alloc((size_t)kCoarse * max_tiles);
    ftot.alloc(kBins);
    fbase.alloc(kBins + 1);
    n_tiles.alloc(1);
    d_records.alloc(1);
    BPE_HIP(hipMemsetAsync(d_records.p, 0, 8, s));
    list.alloc(max_pages);
    list_n.alloc(1);
    BPE_HIP(hipMemsetAsync(held.p, 0, 4ull * max_pages, s));
    BPE_HIP(hipMemsetAsync(done.p, 0, 4ull * max_pages, s));
    n_wg = grid;
    BPE_HIP(hipMemsetAsync(n_pages.p, 0, 4, s));
    BPE_HIP(hipMemsetAsync(wg_used.p, 0, 4ull * grid, s));
    std::vector<int> none(grid, -2);   // -2: no page yet
    BPE_HIP(hipMemcpyAsync(wg_page.p, none.data(), 4ull * grid, hipMemcpyHostToDevice, s));
    BPE_HIP(hipStreamSynchronize(s));
}

RecPool RecPoolOwner::dev() const {
    RecPool R{};
    R.lo = rec ? rec->a.p : nullptr;
    R.hi = rec ? rec->b.p : nullptr;
    R.meta = rec ? rec->c.p : nullptr;
    R.page_used = page_used.p;
    R.n_pages = n_pages.p;
    R.max_pages = max_pages;
    R.wg_page = wg_page.p;
    R.wg_used = wg_used.p;
    R.page_ch = page_ch.p;
    R.wg_ch = wg_ch.p;
    R.lw = lw.p;
    R.lw_n = lw_n.p;
    R.lw_per_wg = lw_per_wg;
    R.on = rec != nullptr;
    return R;
}

void RecPoolOwner::aggregate(bool final, const uint8_t* text, const WordCounts& wc, unsigned long long* fill,
                             unsigned* status, hipStream_t s) {
    const RecPool R = dev();
    if (final) {   // the pages the workgroups hold are complete now
        hipLaunchKernelGGL(k_rec_retire, dim3(ceil_div(n_wg, 256)), dim3(256), 0, s, R, n_wg);
    } else {
        hipLaunchKernelGGL(k_rec_hold, dim3(ceil_div(n_wg, 256)), dim3(256), 0, s, R, n_wg, held.p);
    }
    BPE_HIP(hipMemsetAsync(list_n.p, 0, 4, s));
    hipLaunchKernelGGL(k_rec_pick, dim3(ceil_div(max_pages, 256)), dim3(256), 0, s, R, held.p, done.p, list.p,
                       list_n.p);
    // Every size below stays on the device (the grids are sized for a batch of every page and the
    // surplus workgroups leave at once): the file path enqueues a batch between segment launches
    // without waiting for it, its host-to-device copies continuing underneath.
    ++batches;
    // level 1: the listed pages -> coarse bins (B)
    hipLaunchKernelGGL(k_rec_cscan, dim3(kCoarse), dim3(1024), 0, s, page_ch.p, list.p, list_n.p, coff.p, ctot.p);
    hipLaunchKernelGGL(k_rec_tiles, dim3(1), dim3(64), 0, s, ctot.p, cbase.p, d_tl.p, d_t0.p, n_tiles.p,
                       d_records.p);
    hipLaunchKernelGGL(k_rec_part1, dim3(max_pages), dim3(1024), 0, s, R, list.p, list_n.p, coff.p, cbase.p, B->a.p,
                       B->b.p, B->c.p, B->d.p);
    // level 2: each coarse bin's run, in tiles -> the final bins, laid over the listed pages
    // (their records are all in B now)
    hipLaunchKernelGGL(k_rec_fhist, dim3(max_tiles), dim3(1024), 0, s, B->d.p, d_tl.p, n_tiles.p, fhist.p);
    hipLaunchKernelGGL(k_rec_fscan, dim3(kBins), dim3(256), 0, s, fhist.p, d_t0.p, ftot.p);
    hipLaunchKernelGGL(k_rec_base, dim3(1), dim3(1024), 0, s, ftot.p, kBins, fbase.p);
    hipLaunchKernelGGL(k_rec_part2, dim3(max_tiles), dim3(1024), 0, s, B->a.p, B->b.p, B->c.p, d_tl.p, n_tiles.p,
                       fhist.p, fbase.p, R.lo, R.hi, R.meta, list.p);
    hipLaunchKernelGGL(k_rec_reduce, dim3(kBins), dim3(1024), 0, s, R.lo, R.hi, R.meta, fbase.p, list.p, text,
                       wc.kv.p, wc.pos.p, wc.cap - 1, fill, status);
    BPE_HIP(hipGetLastError());
    if (final) {
        unsigned long long tot = 0;
        unsigned allocated = 0;
        BPE_HIP(hipMemcpyAsync(&tot, d_records.p, 8, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipMemcpyAsync(&allocated, n_pages.p, 4, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipStreamSynchronize(s));
        records = tot;
        pages_used = std::min(allocated, max_pages);
    }
}

}  // namespace bpe
