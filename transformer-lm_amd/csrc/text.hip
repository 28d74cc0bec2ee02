// Text preparation and unique-word counting on the device.
//
//   prepare_text : reference models/tokenizer/train.py:22, open(path, "r", encoding="utf-8")
//                  .read() -- strict UTF-8 (UnicodeDecodeError) + universal newlines.
//   count_words  : reference models/tokenizer/train.py:16-28 extract_subword_frequencies,
//                  GPT-2 pattern of train.py:143-146 (pretok.h).
//
// HBM layout: the corpus is read once, coalesced; the word-count table is two flat u64
// arrays (key, count) of power-of-two capacity.  A key packs (length << 40 | offset + 1):
// the offset of the first occurrence that claimed the slot IS the word's identity, so a
// single 64-bit CAS publishes a slot completely and a later thread verifies a match by
// comparing bytes against the corpus itself -- exact counting with no spin-waits.

#include <cstdio>
#include <cstdlib>

#include <hip/hip_ext.h>

#include "count.h"
#include "internal.h"
#include "prims.h"
#include "pretok.h"
#include "stage.h"

namespace bpe {

// ------------------------------------------------------------------ UTF-8 validation
__device__ __forceinline__ int utf8_len_valid(const uint8_t* __restrict__ s, size_t n, size_t i) {
    const uint32_t b0 = s[i];
    uint32_t need, lo = 0x80, hi = 0xBF;
    if (b0 < 0x80u) return 1;
    if (b0 >= 0xC2u && b0 <= 0xDFu) need = 2;
    else if (b0 == 0xE0u) { need = 3; lo = 0xA0; }
    else if (b0 >= 0xE1u && b0 <= 0xECu) need = 3;
    else if (b0 == 0xEDu) { need = 3; hi = 0x9F; }
    else if (b0 >= 0xEEu && b0 <= 0xEFu) need = 3;
    else if (b0 == 0xF0u) { need = 4; lo = 0x90; }
    else if (b0 >= 0xF1u && b0 <= 0xF3u) need = 4;
    else if (b0 == 0xF4u) { need = 4; hi = 0x8F; }
    else return 0;
    if (i + need > n) return 0;
    const uint32_t b1 = s[i + 1];
    if (b1 < lo || b1 > hi) return 0;
    for (uint32_t k = 2; k < need; ++k)
        if ((s[i + k] & 0xC0u) != 0x80u) return 0;
    return (int)need;
}

// byte i is well-formed iff it is ASCII, a lead byte of a valid sequence, or a continuation
// byte covered by the nearest lead byte within 3 positions before it.
__device__ __forceinline__ bool byte_ok(const uint8_t* __restrict__ s, size_t n, size_t i) {
    const uint32_t b = s[i];
    if (b < 0x80u) return true;
    if ((b & 0xC0u) != 0x80u) return utf8_len_valid(s, n, i) > 0;
    size_t q = i;
    for (int k = 0; k < 3 && q > 0; ++k) {
        --q;
        if ((s[q] & 0xC0u) != 0x80u) {
            const int l = utf8_len_valid(s, n, q);
            return l > 0 && i < q + (size_t)l;
        }
    }
    return false;
}

constexpr int kValidateBytes = 16;

// Units [u0, u1) of kValidateBytes (global positions: unit u is s[16u, 16u + 16)), with the
// text taken to end at n.  A segment of a corpus that is still arriving validates its units
// with n = the segment's end, a safe split point: its last byte is ASCII, so no well-formed
// sequence crosses it and an ill-formed one is ill-formed whatever follows.
__device__ __forceinline__ void validate_unit(const uint8_t* __restrict__ s, size_t n, size_t t, size_t u1,
                                              unsigned long long* __restrict__ err_pos, unsigned* __restrict__ has_cr) {
    const size_t lo = t * kValidateBytes;
    if (t >= u1 || lo >= n) return;
    bool cr = false;
    if (lo + kValidateBytes <= n && (((uintptr_t)(s + lo)) & 15) == 0) {
        const uint4 v = *reinterpret_cast<const uint4*>(s + lo);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t hi_bits = 0, cr_bits = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            hi_bits |= w[k] & 0x80808080u;
            const uint32_t x = w[k] ^ 0x0D0D0D0Du;                 // zero byte <=> '\r'
            cr_bits |= (x - 0x01010101u) & ~x & 0x80808080u;
        }
        if (cr_bits) atomicOr(has_cr, 1u);
        // neighbours for the sequences that cross the unit: the adjacent lanes hold the adjacent
        // units (a unit at a wave's edge reads its neighbour from memory)
        const int lane = threadIdx.x & 63;
        uint32_t prev = __shfl_up(w[3], 1), next = __shfl_down(w[0], 1);
        if (!hi_bits) return;                                       // all ASCII: done
        if (lane == 0) prev = lo >= 4 ? *reinterpret_cast<const uint32_t*>(s + lo - 4) : 0u;
        // the next unit is not a full one in a lane (past the text, the wave or the launch's range)
        if (lane == 63 || t + 1 >= u1 || lo + 2 * kValidateBytes > n) {
            next = 0;
            for (int k = 0; k < 4 && lo + kValidateBytes + k < n; ++k) next |= (uint32_t)s[lo + kValidateBytes + k] << (8 * k);
        }
        // window b[0..24): 4 bytes before the unit, its 16, 4 after
        uint8_t b[24];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            b[k] = (uint8_t)(prev >> (8 * k));
            b[20 + k] = (uint8_t)(next >> (8 * k));
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) b[4 + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
        // bytes of the text left from window index x (the window may run past the end)
        auto avail = [&](int x) -> size_t { const size_t i = lo + (size_t)x - 4; return i < n ? n - i : 0; };
        auto len_valid = [&](int x) -> int {   // utf8_len_valid on the window (x: a constant)
            const uint32_t b0 = b[x];
            uint32_t need, lo8 = 0x80, hi8 = 0xBF;
            if (b0 < 0x80u) return 1;
            if (b0 >= 0xC2u && b0 <= 0xDFu) need = 2;
            else if (b0 == 0xE0u) { need = 3; lo8 = 0xA0; }
            else if (b0 >= 0xE1u && b0 <= 0xECu) need = 3;
            else if (b0 == 0xEDu) { need = 3; hi8 = 0x9F; }
            else if (b0 >= 0xEEu && b0 <= 0xEFu) need = 3;
            else if (b0 == 0xF0u) { need = 4; lo8 = 0x90; }
            else if (b0 >= 0xF1u && b0 <= 0xF3u) need = 4;
            else if (b0 == 0xF4u) { need = 4; hi8 = 0x8F; }
            else return 0;
            if (avail(x) < need) return 0;
            const uint32_t b1 = b[x + 1];
            if (b1 < lo8 || b1 > hi8) return 0;
            if (need >= 3 && (b[x + 2] & 0xC0u) != 0x80u) return 0;
            if (need == 4 && (b[x + 3] & 0xC0u) != 0x80u) return 0;
            return (int)need;
        };
        int bad_k = -1;
#pragma unroll
        for (int k = 0; k < kValidateBytes; ++k) {   // byte_ok for the high-bit bytes
            const int x = 4 + k;
            if (bad_k >= 0 || b[x] < 0x80u) continue;
            bool ok;
            if ((b[x] & 0xC0u) != 0x80u) {
                ok = len_valid(x) > 0;
            } else {   // a continuation byte: covered by the nearest lead byte within 3 before it
                ok = false;
                bool found = false;
#pragma unroll
                for (int d = 1; d <= 3; ++d) {
                    if (found || lo + (size_t)k < (size_t)d) continue;   // no byte before the text
                    if ((b[x - d] & 0xC0u) != 0x80u) {
                        found = true;
                        const int l = len_valid(x - d);
                        ok = l > 0 && d < l;
                    }
                }
            }
            if (!ok) bad_k = k;
        }
        if (bad_k >= 0) atomicMin(err_pos, (unsigned long long)(lo + (size_t)bad_k));
        return;
    }
    const size_t hi = lo + kValidateBytes < n ? lo + kValidateBytes : n;
    for (size_t i = lo; i < hi; ++i) {
        if (s[i] == 0x0D) cr = true;
        if (!byte_ok(s, n, i)) {
            atomicMin(err_pos, (unsigned long long)i);
            break;
        }
    }
    if (cr) atomicOr(has_cr, 1u);
}

// grid-stride over the units, whole workgroups per step (the unit body exchanges neighbours
// between lanes)
__global__ void k_validate(const uint8_t* __restrict__ s, size_t n, size_t u0, size_t u1,
                           unsigned long long* __restrict__ err_pos, unsigned* __restrict__ has_cr) {
    for (size_t b0 = u0 + (size_t)blockIdx.x * blockDim.x; b0 < u1; b0 += (size_t)gridDim.x * blockDim.x)
        validate_unit(s, n, b0 + threadIdx.x, u1, err_pos, has_cr);
}

// universal newlines: "\r\n" -> "\n", lone "\r" -> "\n"
__global__ void k_newline_map(const uint8_t* __restrict__ s, size_t n, uint8_t* __restrict__ out,
                              uint8_t* __restrict__ keep) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint8_t b = s[i];
        out[i] = (b == 0x0D) ? 0x0A : b;
        keep[i] = !(b == 0x0D && i + 1 < n && s[i + 1] == 0x0A);
    }
}

const uint8_t* prepare_text(const uint8_t* d_in, size_t n, DevBuf<uint8_t>& scratch,
                            size_t* n_out, hipStream_t stream) {
    *n_out = n;
    if (n == 0) return d_in;
    DevBuf<unsigned long long> flags(2);
    const unsigned long long h_init[2] = {~0ULL, 0ULL};
    to_device(flags.p, h_init, sizeof(h_init), stream);
    const size_t threads = (n + kValidateBytes - 1) / kValidateBytes;
    hipLaunchKernelGGL(k_validate, dim3(grid_for(threads, 256)), dim3(256), 0, stream, d_in, n,
                       (size_t)0, threads, flags.p, reinterpret_cast<unsigned*>(flags.p + 1));
    BPE_HIP(hipGetLastError());
    unsigned long long h[2];
    to_host(h, flags.p, sizeof(h), stream);
    if (h[0] != ~0ULL)
        throw Error{BPE_E_UTF8, "'utf-8' codec can't decode byte at position " + std::to_string(h[0])};
    if ((unsigned)h[1] == 0) return d_in;

    DevBuf<uint8_t> mapped(n), keep(n);
    scratch.alloc(n);
    hipLaunchKernelGGL(k_newline_map, dim3(grid_for(n, 256)), dim3(256), 0, stream, d_in, n,
                       mapped.p, keep.p);
    DevBuf<unsigned long long> d_nsel(1);
    select_flagged(mapped.p, keep.p, scratch.p, d_nsel.p, n, stream);
    unsigned long long nsel = 0;
    to_host(&nsel, d_nsel.p, 8, stream);
    *n_out = (size_t)nsel;
    return scratch.p;
}

// ------------------------------------------------------------------ word counting
template <class Src>
__device__ __forceinline__ bool global_add(const uint8_t* __restrict__ s, const Src& t, size_t p, size_t len,
                                           uint64_t wl, uint64_t wh, uint64_t h, unsigned long long c,
                                           unsigned long long* __restrict__ kv,
                                           unsigned long long* __restrict__ pos, size_t mask,
                                           unsigned* __restrict__ status) {
    bool ins;
    table_add(s, t, p, len, wl, wh, h, c, kv, pos, mask, status, &ins);
    return ins;
}

constexpr int kCache = 1024;         // LDS word-cache entries
constexpr int kWays = 2;             // associativity (a set is kWays adjacent entries)
constexpr int kEpoch = 4;            // chunks between cache evictions
constexpr unsigned kKeep = 2;        // an entry stays if it was hit this often in the epoch

// Persistent workgroups stream the corpus in kChunk pieces: coalesced 16-B loads of the next
// chunk (+halo) go to registers while the current one is scanned out of LDS.  Each of the 256
// threads owns a 64-byte nominal span that starts at the first safe point at or after its
// start and stops at the first safe point at or after its end, so the spans tile the corpus
// exactly along token boundaries (tokens that run past the staged window read global memory).
// Words <= 16 bytes are counted in an LDS cache holding their packed bytes (2-way; a slot is
// published only after its bytes are written); the rest, and cache conflicts, go to the global
// table.  The cache is flushed once at the end.  If the table passes max_fill keys, every
// workgroup stops early and the host recounts with a larger table.
//
// A launch counts the text [lo, n) (lo = 0, or a safe split point: a token start) over the
// kChunk-aligned chunks chunk0 .. chunk0 + n_chunks - 1, so a corpus arriving in segments is
// counted segment by segment into one table, with the same tokens as one pass over it.
template <bool kAligned>
__global__ void __launch_bounds__(256, 3) k_count_words(const uint8_t* __restrict__ s, size_t lo, size_t n,
                                                     size_t chunk0, size_t n_chunks, unsigned long long* __restrict__ kv,
                                                     unsigned long long* __restrict__ pos, size_t mask, unsigned long long max_fill,
                                                     unsigned long long* __restrict__ fill,
                                                     unsigned* __restrict__ status,
                                                     unsigned long long* __restrict__ n_tok, int mode,
                                                     const unsigned long long* __restrict__ gate) {
    // a segment is counted only behind a clean validation of everything before it (gate: the
    // first bad byte, ~0 = none): ill-formed UTF-8 is never scanned
    if (gate && *gate != ~0ULL) return;
    __shared__ unsigned long long c_key[kCache];
    __shared__ uint64_t c_lo[kCache], c_hi[kCache];
    __shared__ unsigned c_cnt[kCache];
    __shared__ uint16_t c_mark[kCache];   // low 16 bits of c_cnt at the last epoch end
    __shared__ unsigned long long s_red[4];
    __shared__ uint32_t s_start[257];
    __shared__ int s_stop;
    const int tid = threadIdx.x;
    for (int i = tid; i < kCache; i += blockDim.x) { c_key[i] = 0; c_cnt[i] = 0; c_mark[i] = 0; }
    unsigned long long ntok = 0, inserted = 0, n_miss = 0, n_long = 0;

    uint4 pre[kVec];
    // one pre-token of length len at position r of src (global offset gpos)
    auto count_token = [&](const auto& src, auto r, size_t len, size_t gpos) {
        if (len < 2) return;
        ++ntok;
        if (mode == 1) return;   // analysis knob (BPE355_COUNT_MODE=1): the scan alone
        if (len >= kMaxPretok) {
            atomicOr(status, 2u);
        } else if (len <= kInline) {
            uint64_t wl = 0, wh = 0;
            for (uint32_t i = 0; i < (uint32_t)len; ++i) {
                const uint64_t b = src[r + i];
                if (i < 8) wl |= b << (8 * i);
                else wh |= b << (8 * (i - 8));
            }
            const uint64_t h = short_hash(wl, wh, len);
            const unsigned ls = (unsigned)(h >> 40) & (kCache - kWays);
            const unsigned long long mine = ((unsigned long long)len << 40) | (gpos + 1);
            for (int way = 0; way < kWays; ++way) {
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
                        return;
                    }
                }
                if (k != kBusy && (k >> 40) == len) {
                    __asm__ volatile("" ::: "memory");
                    if (c_lo[sl] == wl && c_hi[sl] == wh) {
                        atomicAdd(&c_cnt[sl], 1u);
                        return;
                    }
                }
            }
            ++n_miss;
            if (mode == 2) return;   // analysis knob: LDS cache only, misses dropped
            inserted += global_add(s, s, gpos, len, wl, wh, h, 1, kv, pos, mask, status);
        } else {
            ++n_long;
            if (mode == 2) return;
            inserted += global_add(s, s, gpos, len, 0, 0, hash_word(s, gpos, len), 1, kv, pos, mask, status);
        }
    };
    if (blockIdx.x < n_chunks) stage_fetch<kAligned>(pre, s, n, (chunk0 + blockIdx.x) * kChunk, tid);
    for (size_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
        __syncthreads();   // the previous chunk's scan is done with buf
        stage_store(pre, tid);
        if (tid == 0) s_stop = *(volatile unsigned long long*)fill > max_fill;
        __syncthreads();
        if (s_stop) {
            if (tid == 0) atomicOr(status, 1u);
            break;
        }
        if (c + gridDim.x < n_chunks)   // in flight during the scan
            stage_fetch<kAligned>(pre, s, n, (chunk0 + c + gridDim.x) * kChunk, tid);

        const size_t base = (chunk0 + c) * kChunk;
        const uint32_t rlo = lo > base ? (uint32_t)(lo - base) : 0u;   // the text starts here
        const size_t rem = n - base;
        const bool text_ends = rem <= (size_t)kWin;          // the window reaches the end of text
        const uint32_t nloc = text_ends ? (uint32_t)rem : (uint32_t)kWin;
        const uint32_t search_end = text_ends ? nloc : nloc - 2;   // safe points need p+1 staged
        // span starts: the first safe point at or after each nominal start, searched inside the
        // window only (kNotFound: it lies past the window)
        const LdsText L{};
        auto find_start = [&](uint32_t r) -> uint32_t {
            if (base <= lo && r <= rlo) return rlo;   // the text (or segment) start
            if (r >= nloc) return text_ends ? nloc : kNotFound;
            if (r == 0) {   // position 0's left neighbour is the previous chunk's last byte
                if (nloc > 1 && L[0] == 0x20 && ascii_nonspace(s[base - 1]) && ascii_nonspace(L[1]))
                    return 0;
                r = 1;
            }
            for (; r < search_end; ++r)
                if (is_safe_point(L, nloc, r)) return r;
            return text_ends ? nloc : kNotFound;
        };
        s_start[tid] = find_start((uint32_t)tid * 64);
        if (tid == 0) s_start[256] = find_start((uint32_t)kChunk);
        __syncthreads();
        const uint32_t r0 = s_start[tid], r1 = s_start[tid + 1];
        if (r0 != kNotFound && r1 != kNotFound) {
            // fast path: [r0, r1) and its one-byte lookahead are staged
            for (uint32_t r = r0; r < r1;) {
                const uint32_t e = token_end(L, nloc, r);
                count_token(L, r, e - r, base + r);
                r = e;
            }
        } else if (r0 != kNotFound) {
            // slow path (rare): no safe point in the rest of the window -- scan global memory
            // from r0 to the first safe point past this thread's nominal end
            const size_t hi = base + (size_t)tid * 64 + 64;
            for (size_t p = base + r0; p < n;) {   // (tokens end at n: a safe point or the end)
                if (p >= hi && is_safe_point(s, n, p)) break;
                const size_t e = token_end(s, n, p);
                count_token(s, p, e - p, p);
                p = e;
            }
        }
        // epoch end: entries hit fewer than kKeep times since the last epoch go to the global
        // table and free their slot (the cache fills first-come; without eviction a frequent
        // word whose two ways were taken early would miss for the whole stream)
        if ((c - blockIdx.x) / gridDim.x % kEpoch == kEpoch - 1) {
            __syncthreads();
            for (int i = tid; i < kCache; i += blockDim.x) {
                const unsigned long long k = c_key[i];
                if (k == 0 || k == kBusy) continue;
                const unsigned cc = c_cnt[i];
                if ((uint16_t)(cc - c_mark[i]) >= kKeep) {   // < 65536 hits per 64 KB epoch
                    c_mark[i] = (uint16_t)cc;
                    continue;
                }
                const size_t len = (size_t)(k >> 40), p0 = (size_t)(k & kOffMask) - 1;
                const uint64_t wl = c_lo[i], wh = c_hi[i];
                inserted += global_add(s, s, p0, len, wl, wh, short_hash(wl, wh, len), cc, kv, pos, mask, status);
                c_key[i] = 0;
                c_cnt[i] = 0;
                c_mark[i] = 0;
            }
        }
        // publish this chunk's new keys (one atomic per workgroup per chunk)
        const unsigned long long ins = wave_sum(inserted);
        inserted = 0;
        if ((tid & 63) == 0) s_red[tid >> 6] = ins;
        __syncthreads();
        if (tid == 0) {
            const unsigned long long b = s_red[0] + s_red[1] + s_red[2] + s_red[3];
            if (b) atomicAdd(fill, b);
        }
    }
    __syncthreads();
    // flush the cache: one global add per distinct cached word
    for (int i = tid; i < kCache; i += blockDim.x) {
        const unsigned long long k = c_key[i];
        if (k == 0 || k == kBusy) continue;
        const size_t len = (size_t)(k >> 40), p0 = (size_t)(k & kOffMask) - 1;
        const uint64_t wl = c_lo[i], wh = c_hi[i];
        inserted += global_add(s, s, p0, len, wl, wh, short_hash(wl, wh, len), c_cnt[i], kv, pos, mask, status);
    }
    ntok = wave_sum(ntok);
    inserted = wave_sum(inserted);
    n_miss = wave_sum(n_miss);
    n_long = wave_sum(n_long);
    if ((tid & 63) == 0 && (n_miss | n_long)) {   // diagnostics (BPE355_TRACE)
        atomicAdd(n_tok + 1, n_miss);
        atomicAdd(n_tok + 2, n_long);
    }
    __syncthreads();
    if ((tid & 63) == 0) s_red[tid >> 6] = ntok;
    __syncthreads();
    if (tid == 0) {
        const unsigned long long b = s_red[0] + s_red[1] + s_red[2] + s_red[3];
        if (b) atomicAdd(n_tok, b);
    }
    __syncthreads();
    if ((tid & 63) == 0) s_red[tid >> 6] = inserted;
    __syncthreads();
    if (tid == 0) {
        const unsigned long long b = s_red[0] + s_red[1] + s_red[2] + s_red[3];
        if (b) atomicAdd(fill, b);
    }
}

namespace {

// per-launch grid of the persistent counter: one resident wave of workgroups (every workgroup
// takes the same number of chunks, so a second, queued wave would nearly double the time)
unsigned count_grid(size_t n_chunks, bool aligned) {
    auto kern = aligned ? k_count_words<true> : k_count_words<false>;
    static int per_cu = 0, n_cu = 0;
    if (!per_cu) {
        int dev = 0;
        BPE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, kPadded));
        BPE_HIP(hipGetDevice(&dev));
        BPE_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    unsigned grid = (unsigned)std::min<size_t>(std::max<size_t>(n_chunks, 1),
                                               (size_t)std::max(1, per_cu) * std::max(1, n_cu));
    if (const char* e = std::getenv("BPE355_STREAM_WG"))   // test knob: fewer workgroups, each
        grid = std::max(1u, std::min(grid, (unsigned)std::atoi(e)));   // streaming many chunks
    return grid;
}

// first guess ~1 slot per KiB of a large corpus (7.4 M words in 11.9 GB of OWT-like text:
// load 0.46), 1 per 16 bytes below 64 MiB (small texts have many more unique words per byte);
// the kernel stops early past load 1/2 and the count reruns with 4x the slots
size_t first_cap(size_t n) {
    size_t cap = next_pow2(std::max<size_t>(1 << 16, n < (1u << 26) ? n / 16 : n / 1024));
    if (const char* e = std::getenv("BPE355_WORD_CAP_LOG2"))   // test knob: force the regrow path
        cap = size_t(1) << std::max(8, std::min(34, std::atoi(e)));
    return cap;
}

}  // namespace

void CountPass::begin(const uint8_t* d_text, size_t n, size_t cap, hipStream_t stream, bool timing) {
    BPE_REQUIRE(n < (1ULL << 40) - 1, BPE_E_LIMIT, "corpus slab larger than 1 TiB");
    text = d_text;
    total = n;
    s = stream;
    timed = timing;
    kernel_ms = 0;
    for (auto& e : ev) (void)hipEventDestroy(e);
    ev.clear();
    if (!status.p) {
        status.alloc(1);
        ntok.alloc(3);
        fill.alloc(1);
    }
    wc.kv.alloc(2 * cap);
    wc.pos.alloc(cap);
    wc.cap = cap;
    BPE_HIP(hipMemsetAsync(wc.kv.p, 0, wc.kv.bytes(), s));
    BPE_HIP(hipMemsetAsync(status.p, 0, 4, s));
    BPE_HIP(hipMemsetAsync(ntok.p, 0, 24, s));
    BPE_HIP(hipMemsetAsync(fill.p, 0, 8, s));
    static const bool v1 = std::getenv("BPE355_COUNT_V1") != nullptr;   // A/B knob: the serial counter
    v2 = !v1;
    rec.reset();
    pool_fallback = false;
    if (v2) {
        grid2 = count2_grid((n + kChunk - 1) / kChunk);
        // misses spill as records (aggregated in LDS by bin afterwards) when the text is large
        // enough for the per-workgroup pages to pay off; BPE355_REC_POOL forces it (tests)
        if (n >= (size_t(256) << 20) || std::getenv("BPE355_REC_POOL")) {
            rec = std::make_unique<RecPoolOwner>();
            try {
                rec->init(n, grid2, s);
            } catch (const Error& e) {
                if (e.code != BPE_E_NOMEM) throw;
                // no room for the pool: every miss goes to the global table instead (same counts)
                BPE_HIP(hipStreamSynchronize(s));
                rec.reset();
                pool_fallback = true;
            }
        }
    }
}

void CountPass::range(size_t lo, size_t hi) {
    if (hi <= lo) return;
    const size_t c0 = lo / kChunk, c1 = (hi + kChunk - 1) / kChunk;
    const bool aligned = (reinterpret_cast<uintptr_t>(text) & 15u) == 0;
    auto kern = aligned ? k_count_words<true> : k_count_words<false>;
    const unsigned grid = count_grid(c1 - c0, aligned);
    // analysis knob: 1 = scan only, 2 = LDS word cache only (counts incomplete: timing only)
    static const int count_mode = std::getenv("BPE355_COUNT_MODE") ? std::atoi(std::getenv("BPE355_COUNT_MODE")) : 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timed) {
        BPE_HIP(hipEventCreate(&e0));
        BPE_HIP(hipEventCreate(&e1));
        ev.push_back(e0);
        ev.push_back(e1);
    }
    if (v2) {
        RecPool R{};
        if (rec) R = rec->dev();
        count2_launch(text, lo, hi, c0, c1 - c0, grid2, wc, fill.p, status.p, ntok.p, R, gate, s, e0, e1);
        count_long_launch(text, wc, fill.p, status.p, R, grid2, s);
        return;
    }
    // timed launch: the events are stamped by the kernel's own dispatch packet (the interval
    // rocprofv3 reports), not by marker packets around it
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(256), kPadded, s, e0, e1, 0, text, lo, hi, c0, c1 - c0,
                          wc.kv.p, wc.pos.p, wc.cap - 1, (unsigned long long)(wc.cap / 2), fill.p, status.p,
                          ntok.p, count_mode, gate);
    BPE_HIP(hipGetLastError());
}

void CountPass::partial() {
    if (!rec) return;
    hipEvent_t r0 = nullptr, r1 = nullptr;
    if (timed) {
        BPE_HIP(hipEventCreate(&r0));
        BPE_HIP(hipEventCreate(&r1));
        BPE_HIP(hipEventRecord(r0, s));
    }
    rec->aggregate(false, text, wc, fill.p, status.p, s);   // enqueued only: the host goes on
    if (timed) {
        BPE_HIP(hipEventRecord(r1, s));
        pev.push_back(r0);
        pev.push_back(r1);
    }
}

bool CountPass::finish() {
    if (rec) {   // aggregate the spilled records into the table
        hipEvent_t r0 = nullptr, r1 = nullptr;
        if (timed) {
            BPE_HIP(hipEventCreate(&r0));
            BPE_HIP(hipEventCreate(&r1));
            BPE_HIP(hipEventRecord(r0, s));
        }
        rec->aggregate(true, text, wc, fill.p, status.p, s);
        wc.n_records = rec->records;
        wc.batches = rec->batches;
        if (timed) {
            BPE_HIP(hipEventRecord(r1, s));
            BPE_HIP(hipEventSynchronize(r1));
            float ms = 0;
            BPE_HIP(hipEventElapsedTime(&ms, r0, r1));
            wc.reduce_ms = ms;
            (void)hipEventDestroy(r0);
            (void)hipEventDestroy(r1);
        }
        rec.reset();   // the pool's memory goes back before the merge loop
    }
    unsigned st = 0;
    BPE_HIP(hipMemcpyAsync(&st, status.p, 4, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipMemcpyAsync(&wc.n_pretokens, ntok.p, 8, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipStreamSynchronize(s));
    if (st & 2u) throw Error{BPE_E_LIMIT, "a pre-token is 8 MiB or longer"};
    for (size_t i = 0; i + 1 < ev.size(); i += 2) {
        float ms = 0;
        BPE_HIP(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
        kernel_ms += ms;
    }
    for (size_t i = 0; i + 1 < pev.size(); i += 2) {
        float ms = 0;
        BPE_HIP(hipEventElapsedTime(&ms, pev[i], pev[i + 1]));
        wc.partial_ms += ms;
    }
    if (std::getenv("BPE355_TRACE")) {
        unsigned long long d[3];
        BPE_HIP(hipMemcpy(d, ntok.p, 24, hipMemcpyDeviceToHost));
        std::fprintf(stderr,
                     "[bpe355] count: cap %zu pretokens %llu cache-miss %llu long %llu launches %zu records %llu"
                     " (batches %u, partial %.1f ms, tail %.1f ms)\n",
                     wc.cap, d[0], d[1], d[2], ev.size() / 2, (unsigned long long)wc.n_records, wc.batches, wc.partial_ms,
                     wc.reduce_ms);
    }
    return !(st & 1u);
}

CountPass::CountPass() = default;

CountPass::~CountPass() {
    for (auto& e : ev) (void)hipEventDestroy(e);
    for (auto& e : pev) (void)hipEventDestroy(e);
}

size_t CountPass::initial_cap(size_t n) { return first_cap(n); }

void count_words(const uint8_t* d_text, size_t n, WordCounts& wc, hipStream_t stream,
                 float* kernel_ms) {
    CountPass cp;
    size_t cap = first_cap(n);
    for (int attempt = 0;; ++attempt) {
        cp.begin(d_text, n, cap, stream, kernel_ms != nullptr);
        cp.range(0, n);
        if (cp.finish()) break;
        BPE_REQUIRE(attempt < 8, BPE_E_NOMEM, "word table overflow");
        cap *= 4;  // the table filled up: grow and recount
    }
    if (kernel_ms) *kernel_ms = (float)cp.kernel_ms;
    wc = std::move(cp.wc);
}

// ------------------------------------------------------------------ validation by segment
void ValidatePass::begin(const uint8_t* d_text, size_t n, hipStream_t stream) {
    text = d_text;
    total = n;
    s = stream;
    if (!flags.p) flags.alloc(2);
    const unsigned long long h_init[2] = {~0ULL, 0ULL};
    to_device(flags.p, h_init, sizeof(h_init), s);
    done_units = 0;
}

size_t ValidatePass::prefix(size_t loaded) {
    // a unit's window is [16u - 4, 16u + 20) (k_validate): units with 16u + 20 <= loaded see
    // loaded bytes only, and they are checked against the whole text (end `total`) exactly as
    // one pass over it would
    const size_t u1 = loaded >= total ? (total + kValidateBytes - 1) / kValidateBytes
                                      : (loaded >= 20 ? (loaded - 20) / kValidateBytes + 1 : 0);
    if (u1 > done_units) {
        hipLaunchKernelGGL(k_validate, dim3(grid_for(u1 - done_units, 256)), dim3(256), 0, s, text, total,
                           done_units, u1, flags.p, reinterpret_cast<unsigned*>(flags.p + 1));
        BPE_HIP(hipGetLastError());
        done_units = u1;
    }
    return std::min(total, done_units * kValidateBytes);
}

void ValidatePass::range(size_t lo, size_t hi) {
    // units [lo / 16, hi / 16) against a text that ends at hi; the last segment (hi = total)
    // takes the partial unit too
    const size_t u0 = lo / kValidateBytes;
    const size_t u1 = hi == total ? (hi + kValidateBytes - 1) / kValidateBytes : hi / kValidateBytes;
    if (u1 <= u0) return;
    hipLaunchKernelGGL(k_validate, dim3(grid_for(u1 - u0, 256)), dim3(256), 0, s, text, hi, u0, u1, flags.p,
                       reinterpret_cast<unsigned*>(flags.p + 1));
    BPE_HIP(hipGetLastError());
}

void ValidatePass::finish(unsigned long long* err_pos, bool* has_cr) {
    unsigned long long h[2];
    to_host(h, flags.p, sizeof(h), s);
    *err_pos = h[0];
    *has_cr = (unsigned)h[1] != 0;
}

}  // namespace bpe
