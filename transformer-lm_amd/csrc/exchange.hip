// Multi-GPU word exchange: one all-to-all of the ranks' unique words by owner (the rank the word's
// hash names sums its counts), then one all-gather of the owners' tables, then every rank trains
// on the union with no per-round collective.
//
// Why this is exact: the reference's trainer (models/tokenizer/train.py:16-49) sees the corpus
// only through the multiset of pre-tokens, {word -> count}.  Slabs cut at safe points keep that
// multiset (pretok.h), so summing the ranks' local tables word by word gives the global table,
// and the merge loop on the global table is the single-GPU merge loop.  Every rank runs it on
// identical input and takes identical decisions (ties broken by bytes), so every rank ends with
// the same merges and vocab.
//
// Cost at the bench config: ~7.4 M local words per rank, ~150 MB per rank to gather over xGMI
// (once per training), against the per-round alternative: 31,743 small
// all-reduces in the merge loop's critical path.
//
// Segment a rank contributes to the all-gather (all ranks pad to the largest):
//   u64 cnt[maxw] | u64 len_off[maxw] (len << 32 | byte offset in this segment's byte area) |
//   bytes[maxb]

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <chrono>

#include "internal.h"
#include "prims.h"
#include "stage.h"

namespace bpe {

namespace {

// occupied local-table slots -> (offset in text, length, count) records
__global__ void k_local_words(const unsigned long long* __restrict__ kv, const unsigned long long* __restrict__ pos,
                              size_t cap, unsigned long long* __restrict__ w_off, uint32_t* __restrict__ w_len,
                              unsigned long long* __restrict__ w_cnt, unsigned* __restrict__ n_words) {
    const size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long k = s < cap ? kv[2 * s] : 0ULL;
    const bool keep = k != 0;
    const bool inl = (k >> 63) != 0;
    const unsigned idx = wave_append(keep, n_words);
    if (!keep) return;
    w_len[idx] = inl ? (unsigned)((k >> 56) & 0x7f) : (unsigned)(k >> 40);
    w_off[idx] = inl ? pos[s] : (k & kOffMask) - 1;
    w_cnt[idx] = kv[2 * s + 1];
}

__global__ void k_len_to_u64(const uint32_t* __restrict__ w_len, unsigned n, unsigned long long* __restrict__ o) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = w_len[i];
}

// one word per thread: its record and its bytes into this rank's segment
__global__ void k_pack_words(const uint8_t* __restrict__ text, const unsigned long long* __restrict__ w_off,
                             const uint32_t* __restrict__ w_len, const unsigned long long* __restrict__ w_cnt,
                             const unsigned long long* __restrict__ b_off, unsigned n, size_t maxw,
                             uint8_t* __restrict__ seg) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long* cnt = reinterpret_cast<unsigned long long*>(seg);
    unsigned long long* lo = cnt + maxw;
    uint8_t* bytes = reinterpret_cast<uint8_t*>(lo + maxw);
    const uint32_t len = w_len[i];
    const unsigned long long o = b_off[i];
    cnt[i] = w_cnt[i];
    lo[i] = ((unsigned long long)len << 32) | o;
    const uint8_t* src = text + w_off[i];
    for (uint32_t k = 0; k < len; ++k) bytes[o + k] = src[k];
}

// every gathered record into the union table (counts summed); a word's bytes are addressed in
// the gathered buffer, which becomes the merge loop's "text"
__global__ void k_union_insert(const uint8_t* __restrict__ all, size_t seg_bytes, size_t maxw,
                               const unsigned long long* __restrict__ nw_per_rank, int nranks,
                               unsigned long long* __restrict__ kv, unsigned long long* __restrict__ pos,
                               size_t mask, unsigned* __restrict__ status) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t r = g / maxw, i = g % maxw;
    if ((int)r >= nranks || i >= nw_per_rank[r]) return;
    const uint8_t* seg = all + r * seg_bytes;
    const unsigned long long* cnt = reinterpret_cast<const unsigned long long*>(seg);
    const unsigned long long* lo = cnt + maxw;
    const size_t byte_base = r * seg_bytes + 16 * maxw;
    const unsigned long long c = cnt[i], x = lo[i];
    const size_t len = (size_t)(x >> 32), p = byte_base + (x & 0xffffffffULL);
    uint64_t wl = 0, wh = 0, h;
    if (len <= (size_t)kInline) {
        pack_word(all, p, len, wl, wh);
        h = short_hash(wl, wh, len);
    } else {
        h = hash_word(all, p, len);
    }
    bool ins;
    (void)table_add(all, all, p, len, wl, wh, h, c, kv, pos, mask, status, &ins);
}

// ---- the all-to-all by owner (SURVEY 8e's optional step): every word goes to the rank that owns
// its hash, which sums its counts over all ranks; the all-gather then ships each word once
constexpr unsigned kMaxOwners = 256;

// a word's hash as the tables take it (packed bytes up to kInline, else FNV-1a) and its owner
// (the hash's top bits: the owner's own table slots use the low ones)
__device__ __forceinline__ uint64_t word_hash_at(const uint8_t* __restrict__ t, size_t p, size_t len, uint64_t& wl,
                                                 uint64_t& wh) {
    wl = 0;
    wh = 0;
    if (len <= (size_t)kInline) {
        pack_word(t, p, len, wl, wh);
        return short_hash(wl, wh, len);
    }
    return hash_word(t, p, len);
}
__device__ __forceinline__ unsigned owner_of(uint64_t h, unsigned R) { return (unsigned)(((h >> 40) * R) >> 24); }

// per local word: its owner; per owner the records and bytes it will receive from this rank
__global__ void __launch_bounds__(256) k_own_count(const uint8_t* __restrict__ text,
                                                   const unsigned long long* __restrict__ w_off,
                                                   const uint32_t* __restrict__ w_len, unsigned n, unsigned R,
                                                   unsigned* __restrict__ owner, unsigned long long* __restrict__ tot) {
    __shared__ unsigned h_rec[kMaxOwners], h_b[kMaxOwners];
    for (unsigned q = threadIdx.x; q < R; q += blockDim.x) { h_rec[q] = 0; h_b[q] = 0; }
    __syncthreads();
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint64_t wl, wh;
        const uint32_t len = w_len[i];
        const unsigned o = owner_of(word_hash_at(text, w_off[i], len, wl, wh), R);
        owner[i] = o;
        atomicAdd(&h_rec[o], 1u);
        atomicAdd(&h_b[o], len);
    }
    __syncthreads();
    for (unsigned q = threadIdx.x; q < R; q += blockDim.x)
        if (h_rec[q]) {
            atomicAdd(&tot[q], (unsigned long long)h_rec[q]);
            atomicAdd(&tot[R + q], (unsigned long long)h_b[q]);
        }
}

// each local word's record {count, len << 32 | byte offset} and bytes into its owner's segment
// of the send buffer (segment: u64 cnt[nrec] | u64 lo[nrec] | bytes); one reservation per
// workgroup and owner
__global__ void __launch_bounds__(256) k_own_place(const uint8_t* __restrict__ text,
                                                   const unsigned long long* __restrict__ w_off,
                                                   const uint32_t* __restrict__ w_len,
                                                   const unsigned long long* __restrict__ w_cnt,
                                                   const unsigned* __restrict__ owner, unsigned n, unsigned R,
                                                   const unsigned long long* __restrict__ seg_off,
                                                   const unsigned long long* __restrict__ seg_nrec,
                                                   unsigned long long* __restrict__ cur, uint8_t* __restrict__ send) {
    __shared__ unsigned l_rec[kMaxOwners], l_b[kMaxOwners];
    __shared__ unsigned long long b_rec[kMaxOwners], b_b[kMaxOwners];
    for (unsigned q = threadIdx.x; q < R; q += blockDim.x) { l_rec[q] = 0; l_b[q] = 0; }
    __syncthreads();
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned o = 0, r_loc = 0, b_loc = 0, len = 0;
    if (i < n) {
        o = owner[i];
        len = w_len[i];
        r_loc = atomicAdd(&l_rec[o], 1u);
        b_loc = atomicAdd(&l_b[o], len);
    }
    __syncthreads();
    for (unsigned q = threadIdx.x; q < R; q += blockDim.x)
        if (l_rec[q]) {
            b_rec[q] = atomicAdd(&cur[q], (unsigned long long)l_rec[q]);
            b_b[q] = atomicAdd(&cur[R + q], (unsigned long long)l_b[q]);
        }
    __syncthreads();
    if (i >= n) return;
    const unsigned long long nrec = seg_nrec[o];
    uint8_t* seg = send + seg_off[o];
    unsigned long long* cnt = reinterpret_cast<unsigned long long*>(seg);
    unsigned long long* lo = cnt + nrec;
    uint8_t* bytes = reinterpret_cast<uint8_t*>(lo + nrec);
    const unsigned long long ri = b_rec[o] + r_loc, bo = b_b[o] + b_loc;
    cnt[ri] = w_cnt[i];
    lo[ri] = ((unsigned long long)len << 32) | bo;
    const uint8_t* src = text + w_off[i];
    for (uint32_t k = 0; k < len; ++k) bytes[bo + k] = src[k];
}

// every record of nseg segments of `buf` into a table over `buf` (counts summed); segment r at
// seg_off[r] holds seg_nrec[r] records, its lo[] at cnt + seg_stride[r] and its bytes after lo[]
__global__ void k_seg_insert(const uint8_t* __restrict__ buf, const unsigned long long* __restrict__ seg_off,
                             const unsigned long long* __restrict__ seg_nrec,
                             const unsigned long long* __restrict__ seg_stride, int nseg, size_t maxw,
                             unsigned long long* __restrict__ kv, unsigned long long* __restrict__ pos, size_t mask,
                             unsigned* __restrict__ status) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t r = g / maxw, i = g % maxw;
    if ((int)r >= nseg || i >= seg_nrec[r]) return;
    const unsigned long long* cnt = reinterpret_cast<const unsigned long long*>(buf + seg_off[r]);
    const unsigned long long* lo = cnt + seg_stride[r];
    const size_t byte_base = seg_off[r] + 16 * seg_stride[r];
    const unsigned long long c = cnt[i], x = lo[i];
    const size_t len = (size_t)(x >> 32), p = byte_base + (x & 0xffffffffULL);
    uint64_t wl, wh;
    const uint64_t h = word_hash_at(buf, p, len, wl, wh);
    bool ins;
    (void)table_add(buf, buf, p, len, wl, wh, h, c, kv, pos, mask, status, &ins);
}

}  // namespace

// Default all-to-all through allgather_bytes: every rank's whole send buffer (padded to the
// largest), of which each rank keeps its shares (the host-staged test communicator)
void Comm::alltoallv_bytes(const void* d_send, const size_t* soff, const size_t* scnt, void* d_recv,
                           const size_t* roff, const size_t* rcnt, hipStream_t stream) {
    const int R = nranks;
    // every rank's offsets and sizes, and the largest send buffer
    std::vector<int64_t> meta(2 * (size_t)R * R, 0);
    size_t mine = 0;
    for (int p = 0; p < R; ++p) {
        meta[2 * ((size_t)rank * R + p)] = (int64_t)soff[p];
        meta[2 * ((size_t)rank * R + p) + 1] = (int64_t)scnt[p];
        mine = std::max(mine, soff[p] + scnt[p]);
    }
    std::vector<int64_t> mx(R, 0);
    mx[rank] = (int64_t)mine;
    {
        DevBuf<int64_t> d(meta.size() + R);
        BPE_HIP(hipMemcpyAsync(d.p, meta.data(), meta.size() * 8, hipMemcpyHostToDevice, stream));
        BPE_HIP(hipMemcpyAsync(d.p + meta.size(), mx.data(), R * 8, hipMemcpyHostToDevice, stream));
        allreduce_i64(d.p, d.n, stream);
        BPE_HIP(hipMemcpyAsync(meta.data(), d.p, meta.size() * 8, hipMemcpyDeviceToHost, stream));
        BPE_HIP(hipMemcpyAsync(mx.data(), d.p + meta.size(), R * 8, hipMemcpyDeviceToHost, stream));
        BPE_HIP(hipStreamSynchronize(stream));
    }
    size_t width = 16;
    for (int p = 0; p < R; ++p) width = std::max(width, (size_t)mx[p]);
    DevBuf<uint8_t> pad(width), all((size_t)R * width);
    BPE_HIP(hipMemsetAsync(pad.p, 0, width, stream));
    if (mine) BPE_HIP(hipMemcpyAsync(pad.p, d_send, mine, hipMemcpyDeviceToDevice, stream));
    allgather_bytes(pad.p, width, all.p, stream);
    for (int q = 0; q < R; ++q) {
        const size_t o = (size_t)meta[2 * ((size_t)q * R + rank)], c = (size_t)meta[2 * ((size_t)q * R + rank) + 1];
        BPE_REQUIRE(c == rcnt[q], BPE_E_RCCL, "all-to-all: ranks disagree on a size");
        if (c)
            BPE_HIP(hipMemcpyAsync(static_cast<uint8_t*>(d_recv) + roff[q], all.p + (size_t)q * width + o, c,
                                   hipMemcpyDeviceToDevice, stream));
    }
    BPE_HIP(hipStreamSynchronize(stream));
}

// Every local word to its owner rank (one all-to-all), where the ranks' counts of it are summed:
// `wc` becomes this rank's owner table, keyed over `owned` (the received segments).  Each word
// of the corpus then lives in exactly one owner table, so the all-gather that follows ships
// every unique word once instead of once per rank that saw it.
static void owner_exchange(const uint8_t* text, WordCounts& wc, Comm* comm, hipStream_t stream,
                           DevBuf<uint8_t>& owned, bpe_train_stats* stats) {
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    const int R = comm->nranks;
    BPE_REQUIRE(R <= (int)kMaxOwners, BPE_E_LIMIT, "more ranks than the word exchange's owner bins");
    // ---- local records and their owners
    DevBuf<unsigned> nwd(1);
    BPE_HIP(hipMemsetAsync(nwd.p, 0, 4, stream));
    DevBuf<unsigned long long> w_off(std::max<size_t>(wc.cap, 1)), w_cnt(std::max<size_t>(wc.cap, 1));
    DevBuf<uint32_t> w_len(std::max<size_t>(wc.cap, 1));
    if (wc.cap)
        hipLaunchKernelGGL(k_local_words, dim3(ceil_div(wc.cap, 256)), dim3(256), 0, stream, wc.kv.p, wc.pos.p,
                           wc.cap, w_off.p, w_len.p, w_cnt.p, nwd.p);
    unsigned n = 0;
    BPE_HIP(hipMemcpyAsync(&n, nwd.p, 4, hipMemcpyDeviceToHost, stream));
    BPE_HIP(hipStreamSynchronize(stream));
    { WordCounts drop = std::move(wc); }
    DevBuf<unsigned> owner(std::max(n, 1u));
    DevBuf<unsigned long long> tot(2 * (size_t)R);
    BPE_HIP(hipMemsetAsync(tot.p, 0, tot.bytes(), stream));
    if (n)
        hipLaunchKernelGGL(k_own_count, dim3(ceil_div(n, 256)), dim3(256), 0, stream, text, w_off.p, w_len.p, n,
                           (unsigned)R, owner.p, tot.p);
    std::vector<unsigned long long> ht(2 * (size_t)R);
    BPE_HIP(hipMemcpyAsync(ht.data(), tot.p, 16 * (size_t)R, hipMemcpyDeviceToHost, stream));
    BPE_HIP(hipStreamSynchronize(stream));
    // ---- segment layout (one segment per owner) and everyone's sizes: the R x R matrix of
    // (records, bytes) each rank sends each owner, one small all-reduce
    auto seg_size = [](unsigned long long nrec, unsigned long long nb) { return 16 * nrec + (nb + 15) / 16 * 16; };
    std::vector<int64_t> mat(2 * (size_t)R * R, 0);
    for (int o = 0; o < R; ++o) {
        BPE_REQUIRE(ht[R + o] < (1ULL << 32), BPE_E_LIMIT, "a rank's words for one owner exceed 4 GiB");
        mat[2 * ((size_t)comm->rank * R + o)] = (int64_t)ht[o];
        mat[2 * ((size_t)comm->rank * R + o) + 1] = (int64_t)ht[R + o];
    }
    {
        DevBuf<int64_t> d(mat.size());
        BPE_HIP(hipMemcpyAsync(d.p, mat.data(), mat.size() * 8, hipMemcpyHostToDevice, stream));
        comm->allreduce_i64(d.p, mat.size(), stream);
        BPE_HIP(hipMemcpyAsync(mat.data(), d.p, mat.size() * 8, hipMemcpyDeviceToHost, stream));
        BPE_HIP(hipStreamSynchronize(stream));
    }
    std::vector<size_t> soff(R), scnt(R), roff(R), rcnt(R);
    std::vector<unsigned long long> h_soff(R), h_snrec(R), r_off(R), r_nrec(R);
    size_t stot = 0, rtot = 0;
    unsigned long long rrec = 0;
    for (int o = 0; o < R; ++o) {
        soff[o] = stot;
        scnt[o] = seg_size(ht[o], ht[R + o]);
        h_soff[o] = stot;
        h_snrec[o] = ht[o];
        stot += scnt[o];
        const size_t q = (size_t)o * R + comm->rank;   // rank o's segment for this rank
        roff[o] = rtot;
        rcnt[o] = seg_size((unsigned long long)mat[2 * q], (unsigned long long)mat[2 * q + 1]);
        r_off[o] = rtot;
        r_nrec[o] = (unsigned long long)mat[2 * q];
        rrec += r_nrec[o];
        rtot += rcnt[o];
    }
    // ---- pack by owner, exchange
    DevBuf<uint8_t> send(std::max<size_t>(stot, 16));
    {
        DevBuf<unsigned long long> d_soff(R), d_snrec(R), cur(2 * (size_t)R);
        BPE_HIP(hipMemcpyAsync(d_soff.p, h_soff.data(), 8 * (size_t)R, hipMemcpyHostToDevice, stream));
        BPE_HIP(hipMemcpyAsync(d_snrec.p, h_snrec.data(), 8 * (size_t)R, hipMemcpyHostToDevice, stream));
        BPE_HIP(hipMemsetAsync(cur.p, 0, cur.bytes(), stream));
        if (n)
            hipLaunchKernelGGL(k_own_place, dim3(ceil_div(n, 256)), dim3(256), 0, stream, text, w_off.p, w_len.p,
                               w_cnt.p, owner.p, n, (unsigned)R, d_soff.p, d_snrec.p, cur.p, send.p);
        BPE_HIP(hipGetLastError());
        BPE_HIP(hipStreamSynchronize(stream));
    }
    w_off.release(); w_cnt.release(); w_len.release(); owner.release();
    owned.alloc(std::max<size_t>(rtot, 16));
    const auto ta = clk::now();
    comm->alltoallv_bytes(send.p, soff.data(), scnt.data(), owned.p, roff.data(), rcnt.data(), stream);
    BPE_HIP(hipStreamSynchronize(stream));
    if (stats) {
        stats->t_alltoall_ms = ms(ta);
        stats->exchange_a2a_bytes = (int64_t)stot;
        stats->n_exchanged_words = 0;
    }
    send.release();
    // ---- this rank's owner table over the received segments (counts summed over the ranks)
    const auto tu = clk::now();
    size_t maxw = 1;
    for (int o = 0; o < R; ++o) maxw = std::max<size_t>(maxw, (size_t)r_nrec[o]);
    DevBuf<unsigned long long> d_off(R), d_nrec(R);
    BPE_HIP(hipMemcpyAsync(d_off.p, r_off.data(), 8 * (size_t)R, hipMemcpyHostToDevice, stream));
    BPE_HIP(hipMemcpyAsync(d_nrec.p, r_nrec.data(), 8 * (size_t)R, hipMemcpyHostToDevice, stream));
    DevBuf<unsigned> status(1);
    const size_t cap = next_pow2(std::max<unsigned long long>(2 * rrec, 1 << 16));
    wc.kv.alloc(2 * cap);
    wc.pos.alloc(cap);
    wc.cap = cap;
    BPE_HIP(hipMemsetAsync(wc.kv.p, 0, wc.kv.bytes(), stream));
    BPE_HIP(hipMemsetAsync(status.p, 0, 4, stream));
    const size_t items = (size_t)R * maxw;
    hipLaunchKernelGGL(k_seg_insert, dim3(ceil_div(items, 256)), dim3(256), 0, stream, owned.p, d_off.p, d_nrec.p,
                       d_nrec.p, R, maxw, wc.kv.p, wc.pos.p, cap - 1, status.p);
    BPE_HIP(hipGetLastError());
    unsigned st = 0;
    BPE_HIP(hipMemcpyAsync(&st, status.p, 4, hipMemcpyDeviceToHost, stream));
    BPE_HIP(hipStreamSynchronize(stream));
    BPE_REQUIRE(!(st & 1u), BPE_E_NOMEM, "owner word table overflow");
    if (stats) {
        stats->t_owner_ms = ms(tu);
        stats->n_exchanged_words = (int64_t)rrec;   // this rank's share; summed below
    }
}

// Default all-gather through the sum all-reduce: zero buffer, own segment, sum (exact on int64).
void Comm::allgather_bytes(const void* d_send, size_t bytes, void* d_recv, hipStream_t stream) {
    const size_t words = (bytes + 7) / 8;
    DevBuf<int64_t> tmp((size_t)nranks * words);
    BPE_HIP(hipMemsetAsync(tmp.p, 0, tmp.bytes(), stream));
    BPE_HIP(hipMemcpyAsync(tmp.p + (size_t)rank * words, d_send, bytes, hipMemcpyDeviceToDevice, stream));
    allreduce_i64(tmp.p, tmp.n, stream);
    for (int r = 0; r < nranks; ++r)
        BPE_HIP(hipMemcpyAsync(static_cast<uint8_t*>(d_recv) + (size_t)r * bytes, tmp.p + (size_t)r * words, bytes,
                               hipMemcpyDeviceToDevice, stream));
}

void union_word_tables(const uint8_t* text, WordCounts& wc, Comm* comm, hipStream_t stream,
                       DevBuf<uint8_t>& all, uint64_t* union_words, bpe_train_stats* stats) {
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    const int R = comm->nranks;
    // the all-to-all by owner first (default with several ranks; BPE355_EXCHANGE_OWNER=0: the
    // ranks' local tables are gathered as they are and deduplicated by every rank)
    DevBuf<uint8_t> owned;
    const char* eo = std::getenv("BPE355_EXCHANGE_OWNER");
    const bool by_owner = eo ? eo[0] != '0' : R > 1;
    int64_t a2a_records = 0;
    if (by_owner) {
        owner_exchange(text, wc, comm, stream, owned, stats);
        text = owned.p;
        if (stats) a2a_records = stats->n_exchanged_words;
    }
    // ---- local records (the owner table's: every word of the corpus in exactly one of them)
    DevBuf<unsigned> nwd(1);
    BPE_HIP(hipMemsetAsync(nwd.p, 0, 4, stream));
    DevBuf<unsigned long long> w_off(std::max<size_t>(wc.cap, 1)), w_cnt(std::max<size_t>(wc.cap, 1));
    DevBuf<uint32_t> w_len(std::max<size_t>(wc.cap, 1));
    if (wc.cap)
        hipLaunchKernelGGL(k_local_words, dim3(ceil_div(wc.cap, 256)), dim3(256), 0, stream, wc.kv.p, wc.pos.p,
                           wc.cap, w_off.p, w_len.p, w_cnt.p, nwd.p);
    unsigned n = 0;
    BPE_HIP(hipMemcpyAsync(&n, nwd.p, 4, hipMemcpyDeviceToHost, stream));
    BPE_HIP(hipStreamSynchronize(stream));
    DevBuf<unsigned long long> b_off(std::max(n, 1u)), len64(std::max(n, 1u));
    unsigned long long nbytes = 0;
    if (n) {
        hipLaunchKernelGGL(k_len_to_u64, dim3(ceil_div(n, 256)), dim3(256), 0, stream, w_len.p, n, len64.p);
        exclusive_sum(len64.p, b_off.p, n, stream);
        unsigned long long last[2];
        BPE_HIP(hipMemcpyAsync(&last[0], b_off.p + n - 1, 8, hipMemcpyDeviceToHost, stream));
        BPE_HIP(hipMemcpyAsync(&last[1], len64.p + n - 1, 8, hipMemcpyDeviceToHost, stream));
        BPE_HIP(hipStreamSynchronize(stream));
        nbytes = last[0] + last[1];
    }
    // ---- sizes of every rank's segment (one small all-reduce)
    std::vector<int64_t> sz(2 * (size_t)R, 0);
    sz[2 * comm->rank] = n;
    sz[2 * comm->rank + 1] = (int64_t)nbytes;
    {
        DevBuf<int64_t> d_sz(sz.size());
        BPE_HIP(hipMemcpyAsync(d_sz.p, sz.data(), sz.size() * 8, hipMemcpyHostToDevice, stream));
        comm->allreduce_i64(d_sz.p, sz.size(), stream);
        BPE_HIP(hipMemcpyAsync(sz.data(), d_sz.p, sz.size() * 8, hipMemcpyDeviceToHost, stream));
        BPE_HIP(hipStreamSynchronize(stream));
    }
    size_t maxw = 1, maxb = 16;
    std::vector<unsigned long long> nw_r(R);
    unsigned long long total_w = 0;
    for (int r = 0; r < R; ++r) {
        nw_r[r] = (unsigned long long)sz[2 * r];
        total_w += nw_r[r];
        maxw = std::max<size_t>(maxw, (size_t)sz[2 * r]);
        maxb = std::max<size_t>(maxb, (size_t)sz[2 * r + 1]);
    }
    BPE_REQUIRE(maxb < (1ULL << 32), BPE_E_LIMIT, "a rank's unique words exceed 4 GiB");
    maxb = (maxb + 15) / 16 * 16;
    const size_t seg_bytes = 16 * maxw + maxb;
    // ---- pack, gather
    DevBuf<uint8_t> seg(seg_bytes);
    BPE_HIP(hipMemsetAsync(seg.p, 0, seg_bytes, stream));
    if (n)
        hipLaunchKernelGGL(k_pack_words, dim3(ceil_div(n, 256)), dim3(256), 0, stream, text, w_off.p, w_len.p,
                           w_cnt.p, b_off.p, n, maxw, seg.p);
    BPE_HIP(hipGetLastError());
    { WordCounts drop = std::move(wc); }
    w_off.release(); w_cnt.release(); w_len.release(); b_off.release(); len64.release();
    all.alloc((size_t)R * seg_bytes);
    BPE_HIP(hipStreamSynchronize(stream));
    const auto tg = clk::now();
    comm->allgather_bytes(seg.p, seg_bytes, all.p, stream);
    BPE_HIP(hipStreamSynchronize(stream));
    if (stats) {
        stats->t_gather_ms = ms(tg);
        stats->exchange_seg_bytes = (int64_t)seg_bytes;
    }
    seg.release();
    owned.release();   // (the gathered segments hold copies of the owners' words)
    const auto tu = clk::now();
    // ---- union table (load <= 1/2 even if no word repeats across ranks)
    DevBuf<unsigned long long> d_nw(R);
    BPE_HIP(hipMemcpyAsync(d_nw.p, nw_r.data(), R * 8, hipMemcpyHostToDevice, stream));
    DevBuf<unsigned> status(1);
    const size_t cap = next_pow2(std::max<unsigned long long>(2 * total_w, 1 << 16));
    wc.kv.alloc(2 * cap);
    wc.pos.alloc(cap);
    wc.cap = cap;
    BPE_HIP(hipMemsetAsync(wc.kv.p, 0, wc.kv.bytes(), stream));
    BPE_HIP(hipMemsetAsync(status.p, 0, 4, stream));
    const size_t items = (size_t)R * maxw;
    hipLaunchKernelGGL(k_union_insert, dim3(ceil_div(items, 256)), dim3(256), 0, stream, all.p, seg_bytes, maxw,
                       d_nw.p, R, wc.kv.p, wc.pos.p, cap - 1, status.p);
    BPE_HIP(hipGetLastError());
    unsigned st = 0;
    BPE_HIP(hipMemcpyAsync(&st, status.p, 4, hipMemcpyDeviceToHost, stream));
    BPE_HIP(hipStreamSynchronize(stream));
    BPE_REQUIRE(!(st & 1u), BPE_E_NOMEM, "union word table overflow");
    if (stats) stats->t_union_ms = ms(tu);
    if (union_words) *union_words = total_w;
    if (by_owner) {   // the records every rank sent (before the owners' dedupe), summed over the ranks
        std::vector<int64_t> v(1, a2a_records);
        DevBuf<int64_t> d(1);
        BPE_HIP(hipMemcpyAsync(d.p, v.data(), 8, hipMemcpyHostToDevice, stream));
        comm->allreduce_i64(d.p, 1, stream);
        BPE_HIP(hipMemcpyAsync(v.data(), d.p, 8, hipMemcpyDeviceToHost, stream));
        BPE_HIP(hipStreamSynchronize(stream));
        if (union_words) *union_words = (uint64_t)v[0];
    }
    if (std::getenv("BPE355_TRACE"))
        std::fprintf(stderr, "[bpe355 r%d] word exchange: %u local words, %llu bytes; segment %zu B x %d ranks\n",
                     comm->rank, n, nbytes, seg_bytes, R);
}

}  // namespace bpe
