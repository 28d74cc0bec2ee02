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
#include <hipcub/hipcub.hpp>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "count.h"
#include "pretok.h"
#include "stage.h"
#include "stage2.h"
#include "tokstart.h"

namespace bpe {

namespace {

constexpr int kCache2 = 1024;                     // LDS word-cache entries (2-way sets)
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
__global__ void __launch_bounds__(256) k_count2(const uint8_t* __restrict__ s, size_t lo, size_t n, size_t chunk0,
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
    __shared__ int s_stop, s_page;
    __shared__ unsigned s_used;
    const int tid = threadIdx.x;
    for (int i = tid; i < kCache2; i += blockDim.x) { c_key[i] = 0; c_cnt[i] = 0; c_mark[i] = 0; }
    load_cls2(tid, blockDim.x);
    if (tid == 0) {
        s_page = R.on ? R.wg_page[blockIdx.x] : -1;
        s_used = R.on ? R.wg_used[blockIdx.x] : 0u;
    }
    unsigned long long ntok = 0, inserted = 0, n_miss = 0, n_long = 0;

    // a miss (or an evicted / flushed cache entry): a record in this workgroup's page, else the
    // global table
    auto spill = [&](uint64_t wl, uint64_t wh, size_t len, size_t gpos, unsigned long long c) {
        const int pg = s_page;
        if (pg >= 0 && c < (1ULL << kCntBits)) {
            const unsigned idx = atomicAdd(&s_used, 1u);
            const size_t gi = (size_t)pg * kPageRecs + idx;
            R.lo[gi] = wl;
            R.hi[gi] = wh;
            R.meta[gi] = (unsigned long long)len | ((unsigned long long)gpos << 5) | (c << 45);
            return;
        }
        bool ins;
        table_add(s, s, gpos, len, wl, wh, short_hash(wl, wh, len), c, kv, pos, mask, status, &ins);
        inserted += ins;
    };

    uint4 pre[kSVec];
    if (blockIdx.x < n_chunks) fetch2<kAligned>(pre, s, n, (chunk0 + blockIdx.x) * kChunk, tid);
    for (size_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        __syncthreads();   // the previous chunk is done with the stage, the masks and the page
        store2(pre, tid);
        if (tid == 0) {
            s_stop = *(volatile unsigned long long*)fill > max_fill;
            if (R.on && s_page != -1 && (s_page == -2 || s_used + kRecReserve > (unsigned)kPageRecs)) {
                if (s_page >= 0) R.page_used[s_page] = s_used;
                const unsigned pg = atomicAdd(R.n_pages, 1u);
                s_page = pg < R.max_pages ? (int)pg : -1;   // -1: the pool is spent
                s_used = 0;
            }
        }
        __syncthreads();
        if (s_stop) {
            if (tid == 0) atomicOr(status, 1u);
            break;
        }
        const size_t base = (chunk0 + c) * kChunk;

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
        // the next chunk's loads fly during the token phase (not the register-heavy mask phase)
        if (c + gridDim.x < n_chunks) fetch2<kAligned>(pre, s, n, (chunk0 + c + gridDim.x) * kChunk, tid);
        __syncthreads();

        // ---- the pre-tokens that start in this thread's 64 bytes
        // (analysis knob BPE355_COUNT_MODE, timing only -- counts are then incomplete: 1 masks
        // only, 2 + token bounds, 3 + packing and hashing, 4 + the LDS cache, misses dropped)
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
                if (mode != 4) spill(wl, wh, len, gpos, 1);
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
                spill(c_lo[i], c_hi[i], (size_t)(k >> 40), (size_t)(k & kOffMask) - 1, cc);
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
        spill(c_lo[i], c_hi[i], (size_t)(k >> 40), (size_t)(k & kOffMask) - 1, c_cnt[i]);
    }
    __syncthreads();
    if (tid == 0 && R.on) {   // the next launch's workgroup continues this page
        R.wg_page[blockIdx.x] = s_page;
        R.wg_used[blockIdx.x] = s_used;
    }
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

// ------------------------------------------------------------------ record aggregation
__device__ __forceinline__ uint64_t rec_hash(uint64_t lo, uint64_t hi, uint64_t meta) {
    return short_hash(lo, hi, (size_t)(meta & 31u));
}

// the pages' last fill levels (each workgroup's current page)
__global__ void k_rec_retire(RecPool R, unsigned n_wg) {
    const unsigned b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_wg) return;
    const int pg = R.wg_page[b];
    if (pg >= 0) R.page_used[pg] = R.wg_used[b];
}

// per page: bin histogram, stored bin-major (hist[bin * n_pages + page])
__global__ void __launch_bounds__(1024) k_rec_hist(RecPool R, unsigned n_pages, unsigned* __restrict__ hist) {
    __shared__ unsigned h[kBins];
    const unsigned pg = blockIdx.x;
    for (int i = threadIdx.x; i < kBins; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const unsigned used = R.page_used[pg];
    const size_t g0 = (size_t)pg * kPageRecs;
    constexpr int U = 4;
    for (unsigned i0 = threadIdx.x; i0 < used; i0 += U * blockDim.x) {
        unsigned bin[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned i = i0 + u * blockDim.x;
            bin[u] = i < used ? rec_bin(rec_hash(R.lo[g0 + i], R.hi[g0 + i], R.meta[g0 + i])) : ~0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (bin[u] != ~0u) atomicAdd(&h[bin[u]], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kBins; i += blockDim.x) hist[(size_t)i * n_pages + pg] = h[i];
}

// per bin: exclusive scan over the pages (in place), the bin's total
__global__ void __launch_bounds__(1024) k_rec_binscan(unsigned* __restrict__ hist, unsigned n_pages,
                                                      unsigned long long* __restrict__ tot) {
    typedef hipcub::BlockScan<unsigned, 1024> Scan;
    __shared__ typename Scan::TempStorage tmp;
    __shared__ unsigned carry;
    unsigned* row = hist + (size_t)blockIdx.x * n_pages;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (unsigned b0 = 0; b0 < n_pages; b0 += 1024) {
        const unsigned i = b0 + threadIdx.x;
        const unsigned v = i < n_pages ? row[i] : 0u;
        unsigned ex, agg;
        Scan(tmp).ExclusiveSum(v, ex, agg);
        const unsigned cb = carry;
        if (i < n_pages) row[i] = cb + ex;
        __syncthreads();
        if (threadIdx.x == 0) carry = cb + agg;
        __syncthreads();
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

// bin bases (exclusive scan of the totals; base[kBins] = all records)
__global__ void __launch_bounds__(1024) k_rec_binbase(const unsigned long long* __restrict__ tot,
                                                      unsigned long long* __restrict__ base) {
    typedef hipcub::BlockScan<unsigned long long, 1024> Scan;
    __shared__ typename Scan::TempStorage tmp;
    constexpr int per = kBins / 1024;
    unsigned long long v[per], ex[per], agg;
#pragma unroll
    for (int k = 0; k < per; ++k) v[k] = tot[threadIdx.x * per + k];
    Scan(tmp).ExclusiveSum(v, ex, agg);
#pragma unroll
    for (int k = 0; k < per; ++k) base[threadIdx.x * per + k] = ex[k];
    if (threadIdx.x == 0) base[kBins] = agg;
}

// per page: every record to its bin's run
__global__ void __launch_bounds__(1024) k_rec_scatter(RecPool R, unsigned n_pages, const unsigned* __restrict__ hist,
                                                      const unsigned long long* __restrict__ base,
                                                      uint64_t* __restrict__ olo, uint64_t* __restrict__ ohi,
                                                      uint64_t* __restrict__ ometa) {
    __shared__ unsigned long long cur[kBins];
    const unsigned pg = blockIdx.x;
    for (int i = threadIdx.x; i < kBins; i += blockDim.x) cur[i] = base[i] + hist[(size_t)i * n_pages + pg];
    __syncthreads();
    const unsigned used = R.page_used[pg];
    const size_t g0 = (size_t)pg * kPageRecs;
    constexpr int U = 4;   // records per thread per step: their loads are all in flight together
    for (unsigned i0 = threadIdx.x; i0 < used; i0 += U * blockDim.x) {
        uint64_t a[U], b[U], m[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned i = i0 + u * blockDim.x;
            if (i < used) { a[u] = R.lo[g0 + i]; b[u] = R.hi[g0 + i]; m[u] = R.meta[g0 + i]; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i0 + u * blockDim.x >= used) break;
            const unsigned long long p = atomicAdd(&cur[rec_bin(rec_hash(a[u], b[u], m[u]))], 1ULL);
            olo[p] = a[u];
            ohi[p] = b[u];
            ometa[p] = m[u];
        }
    }
}

constexpr int kRedSlots = 4096;   // LDS table of k_rec_reduce (a bin holds ~1/4096 of the words)
constexpr int kRedProbe = 64;

// per bin: sum the records in LDS, then one global table_add per distinct word
__global__ void __launch_bounds__(1024) k_rec_reduce(const uint64_t* __restrict__ rlo, const uint64_t* __restrict__ rhi,
                                                     const uint64_t* __restrict__ rmeta,
                                                     const unsigned long long* __restrict__ base,
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
          if (i < b1) { ul[u] = rlo[i]; uh[u] = rhi[i]; um[u] = rmeta[i]; }
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
    x->a.alloc(cap);
    x->b.alloc(cap);
    x->c.alloc(cap);
    return x;
}

void scratch_give(std::unique_ptr<Arrays3> x) {
    if (!x) return;
    std::lock_guard<std::mutex> g(scratch().m);
    scratch().free_.push_back(std::move(x));
}

RecPoolOwner::~RecPoolOwner() { scratch_give(std::move(rec)); }

void RecPoolOwner::init(size_t n_bytes, unsigned grid, hipStream_t s) {
    // pool: ~1 record per 10 corpus bytes (the bench corpus spills one per 15); when it runs out,
    // the remaining misses go to the global table (correct, slower)
    size_t want = std::max<size_t>(n_bytes / 10, (size_t)grid * kPageRecs);
    if (const char* e = std::getenv("BPE355_REC_POOL")) want = (size_t)std::atof(e);   // test knob: records
    max_pages = (unsigned)std::max<size_t>(1, std::min<size_t>((want + kPageRecs - 1) / kPageRecs, 1u << 30));
    const size_t cap = (size_t)max_pages * kPageRecs;
    rec = scratch_take(cap);
    page_used.alloc(max_pages);
    n_pages.alloc(1);
    wg_page.alloc(grid);
    wg_used.alloc(grid);
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
    R.on = rec != nullptr;
    return R;
}

void RecPoolOwner::reduce(const uint8_t* text, const WordCounts& wc, unsigned long long* fill, unsigned* status,
                          hipStream_t s) {
    const RecPool R = dev();
    hipLaunchKernelGGL(k_rec_retire, dim3(ceil_div(n_wg, 256)), dim3(256), 0, s, R, n_wg);
    unsigned np = 0;
    BPE_HIP(hipMemcpyAsync(&np, n_pages.p, 4, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipStreamSynchronize(s));
    np = std::min(np, max_pages);
    pages_used = np;
    if (np == 0) return;
    DevBuf<unsigned> hist((size_t)kBins * np);
    DevBuf<unsigned long long> tot(kBins), base(kBins + 1);
    hipLaunchKernelGGL(k_rec_hist, dim3(np), dim3(1024), 0, s, R, np, hist.p);
    hipLaunchKernelGGL(k_rec_binscan, dim3(kBins), dim3(1024), 0, s, hist.p, np, tot.p);
    hipLaunchKernelGGL(k_rec_binbase, dim3(1), dim3(1024), 0, s, tot.p, base.p);
    unsigned long long total = 0;
    BPE_HIP(hipMemcpyAsync(&total, base.p + kBins, 8, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipStreamSynchronize(s));
    records = total;
    if (total == 0) return;
    std::unique_ptr<Arrays3> out = scratch_take(total);
    hipLaunchKernelGGL(k_rec_scatter, dim3(np), dim3(1024), 0, s, R, np, hist.p, base.p, out->a.p, out->b.p,
                       out->c.p);
    hipLaunchKernelGGL(k_rec_reduce, dim3(kBins), dim3(1024), 0, s, out->a.p, out->b.p, out->c.p, base.p, text,
                       wc.kv.p, wc.pos.p, wc.cap - 1, fill, status);
    BPE_HIP(hipGetLastError());
    BPE_HIP(hipStreamSynchronize(s));
    scratch_give(std::move(out));
}

}  // namespace bpe
