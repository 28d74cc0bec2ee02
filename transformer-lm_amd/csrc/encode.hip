// Tokenizer.encode on the device -- reference models/tokenizer/tokenizer.py:
//   12-38   construction: vocab_inv (last id wins), specials deduped + longest first,
//           missing specials appended with ids len(vocab), len(vocab)+1, ...
//   63-66   segment: re.split on the specials alternation (leftmost match, longest first)
//   68-90   pretokenize each non-special segment on its own with the GPT-2 pattern; drop
//           matches equal to a special; special segments stay whole
//   92-138  per pretoken: repeatedly merge ALL occurrences of the adjacent pair with the lowest
//           merge rank (ties: leftmost) until no pair is ranked; ids via vocab_inv (KeyError)
//
// Device pipeline (one stream):
//   1. k_find_specials marks where a special starts (first-byte bitmap, then compare);
//      the sparse candidate list is resolved left-to-right on the host into segments.
//   2. k_scan<INSERT>: threads own byte spans that start/stop at boundary points (segment
//      starts, or safe points inside normal segments) and insert every pre-token into a
//      unique-word table keyed by (length, first offset), exactly like training's count.
//   3. k_encode_words: one thread per unique word runs the rank-ordered merge loop against a
//      device hash map (pair -> rank, product) and writes its vocab ids once (word cache).
//   4. k_scan<COUNT> + exclusive scan + k_scan<WRITE>: re-walk the pre-tokens and emit each
//      occurrence's cached ids at its output offset, specials as their ids.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "internal.h"
#include "pretok.h"

namespace bpe {
namespace {

constexpr unsigned long long kOff40 = (1ULL << 40) - 1;
constexpr size_t kSpan = 256;

struct Seg {                 // a piece of the text: normal (special = -1) or one special token
    unsigned long long start, end;
    int special;
    int pad;
};

struct EncTables {
    const unsigned long long* pm_key;  // ((a << 32) | b) + 1
    const uint2* pm_val;               // (rank, product)
    unsigned long long pm_mask;
    const int64_t* tok2vid;            // internal token -> vocab id, -1 if absent
    const uint32_t* byte2tok;          // 256 entries
    const uint8_t* sp_bytes;
    const uint32_t* sp_off;
    const uint32_t* sp_len;
    const int64_t* sp_vid;
    int n_sp;
};

__device__ __forceinline__ bool bytes_eq(const uint8_t* x, const uint8_t* y, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (x[i] != y[i]) return false;
    return true;
}

// ------------------------------------------------------------------ 1. special candidates
__global__ void k_find_specials(const uint8_t* __restrict__ s, size_t n, EncTables E,
                                const unsigned* __restrict__ first_mask,
                                unsigned long long* __restrict__ pos_out, int* __restrict__ sp_out,
                                unsigned* __restrict__ n_out, unsigned long long cap) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    int hit = -1;
    if (i < n) {
        const unsigned b = s[i];
        if ((first_mask[b >> 5] >> (b & 31)) & 1u) {
            for (int k = 0; k < E.n_sp; ++k) {  // specials are sorted longest first: first hit wins
                const unsigned l = E.sp_len[k];
                if (i + l <= n && bytes_eq(s + i, E.sp_bytes + E.sp_off[k], l)) { hit = k; break; }
            }
        }
    }
    const unsigned idx = wave_append(hit >= 0, n_out);
    if (hit >= 0) {
        if (idx < cap) { pos_out[idx] = i; sp_out[idx] = hit; }
    }
}

// ------------------------------------------------------------------ 2/4. segment-aware scan
enum { SCAN_INSERT = 0, SCAN_COUNT = 1, SCAN_WRITE = 2 };

__device__ __forceinline__ int seg_of(const Seg* __restrict__ segs, int nseg, size_t p) {
    int lo = 0, hi = nseg - 1;  // last segment with start <= p
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].start <= p) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// a position where an independent scan may start: a segment start, or a safe point inside
// a normal segment
__device__ __forceinline__ bool is_boundary(const uint8_t* __restrict__ s, const Seg& sg, size_t p) {
    if (p == sg.start) return true;
    return sg.special < 0 && p + 1 < sg.end && is_safe_point(s, (size_t)sg.end, p);
}

__device__ __forceinline__ size_t word_lookup(const uint8_t* __restrict__ s, size_t p, size_t len,
                                              const unsigned long long* __restrict__ key, size_t mask) {
    size_t slot = hash_word(s + p, len) & mask;
    for (;;) {
        const unsigned long long k = key[slot];
        if (k == 0) return ~(size_t)0;
        if ((k >> 40) == len && bytes_eq(s + ((k & kOff40) - 1), s + p, len)) return slot;
        slot = (slot + 1) & mask;
    }
}

template <int MODE>
__global__ void __launch_bounds__(256)
k_scan(const uint8_t* __restrict__ s, size_t n, const Seg* __restrict__ segs, int nseg, EncTables E,
       unsigned long long* __restrict__ key, size_t mask, const uint32_t* __restrict__ slot_word,
       const uint32_t* __restrict__ w_nids, const unsigned long long* __restrict__ w_idoff,
       const uint32_t* __restrict__ ids_pool, unsigned long long* __restrict__ per_thread,
       uint32_t* __restrict__ out, unsigned* __restrict__ status) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t lo = t * kSpan;
    if (lo >= n) return;
    const size_t hi = lo + kSpan;
    int k = seg_of(segs, nseg, lo);
    size_t p;
    {
        const Seg sg = segs[k];
        if (lo == sg.start) p = lo;
        else if (sg.special >= 0) p = sg.end;
        else {
            p = lo;
            while (p < sg.end && !is_safe_point(s, (size_t)sg.end, p)) ++p;
        }
    }
    unsigned long long emitted = 0, woff = (MODE == SCAN_WRITE) ? per_thread[t] : 0;
    while (p < n) {
        while (k < nseg && p >= segs[k].end) ++k;
        if (k >= nseg) break;
        const Seg sg = segs[k];
        if (p >= hi && is_boundary(s, sg, p)) break;
        if (sg.special >= 0) {  // a special segment (p == sg.start here)
            if (MODE == SCAN_WRITE) out[woff++] = (uint32_t)E.sp_vid[sg.special];
            ++emitted;
            p = sg.end;
            continue;
        }
        const size_t e = token_end(s, (size_t)sg.end, p);
        const size_t len = e - p;
        if (MODE == SCAN_INSERT) {
            if (len >= (1ULL << 24)) { atomicOr(status, 2u); p = e; continue; }
            const unsigned long long mine = ((unsigned long long)len << 40) | (p + 1);
            size_t slot = hash_word(s + p, len) & mask;
            int probe = 0;
            for (; probe < (1 << 16); ++probe) {
                unsigned long long kk = key[slot];
                if (kk == 0) {
                    kk = atomicCAS(&key[slot], 0ULL, mine);
                    if (kk == 0) break;
                }
                if ((kk >> 40) == len && bytes_eq(s + ((kk & kOff40) - 1), s + p, len)) break;
                slot = (slot + 1) & mask;
            }
            if (probe == (1 << 16)) atomicOr(status, 1u);
        } else {
            const size_t slot = word_lookup(s, p, len, key, mask);
            if (slot == ~(size_t)0) { atomicOr(status, 8u); p = e; continue; }
            const uint32_t w = slot_word[slot];
            const uint32_t m = w_nids[w];
            if (MODE == SCAN_WRITE) {
                const uint32_t* src = ids_pool + w_idoff[w];
                for (uint32_t j = 0; j < m; ++j) out[woff + j] = src[j];
                woff += m;
            }
            emitted += m;
        }
        p = e;
    }
    if (MODE == SCAN_COUNT) per_thread[t] = emitted;
}

// ------------------------------------------------------------------ 3. unique words
__global__ void k_collect(const unsigned long long* __restrict__ key, size_t cap,
                          uint32_t* __restrict__ slot_word, unsigned long long* __restrict__ w_off,
                          uint32_t* __restrict__ w_len, unsigned* __restrict__ n_words) {
    const size_t sidx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long k = sidx < cap ? key[sidx] : 0ULL;
    const unsigned w = wave_append(k != 0, n_words);
    if (!k) return;
    slot_word[sidx] = w;
    w_off[w] = (k & kOff40) - 1;
    w_len[w] = (uint32_t)(k >> 40);
}

__device__ __forceinline__ uint2 rank_of(const EncTables& E, uint32_t a, uint32_t b) {
    const unsigned long long key = ((((unsigned long long)a) << 32) | b) + 1ULL;
    size_t s = mix64(key) & E.pm_mask;
    for (;;) {
        const unsigned long long k = E.pm_key[s];
        if (k == key) return E.pm_val[s];
        if (k == 0) return make_uint2(0xffffffffu, 0);
        s = (s + 1) & E.pm_mask;
    }
}

// tokenizer.py:124-136 for one unique word; the ids are written once into the word's slot
__global__ void __launch_bounds__(256)
k_encode_words(const uint8_t* __restrict__ s, EncTables E, const unsigned long long* __restrict__ w_off,
               const uint32_t* __restrict__ w_len, const unsigned long long* __restrict__ w_idoff,
               unsigned n_words, uint32_t* __restrict__ pool, uint32_t* __restrict__ w_nids,
               unsigned* __restrict__ status) {
    const unsigned w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n_words) return;
    const uint8_t* src = s + w_off[w];
    const uint32_t len = w_len[w];
    for (int k = 0; k < E.n_sp; ++k)  // match() drops pre-tokens equal to a special (73)
        if (E.sp_len[k] == len && bytes_eq(src, E.sp_bytes + E.sp_off[k], len)) { w_nids[w] = 0; return; }
    uint32_t* t = pool + w_idoff[w];
    for (uint32_t i = 0; i < len; ++i) t[i] = E.byte2tok[src[i]];
    uint32_t m = len;
    while (m > 1) {
        uint32_t best = 0xffffffffu, prod = 0, ba = 0, bb = 0;
        for (uint32_t i = 0; i + 1 < m; ++i) {
            const uint2 r = rank_of(E, t[i], t[i + 1]);
            if (r.x < best) { best = r.x; prod = r.y; ba = t[i]; bb = t[i + 1]; }
        }
        if (best == 0xffffffffu) break;
        uint32_t j = 0;  // merge() (92-109): every occurrence, left to right
        for (uint32_t i = 0; i < m;) {
            if (t[i] == ba && i + 1 < m && t[i + 1] == bb) { t[j++] = prod; i += 2; }
            else t[j++] = t[i++];
        }
        m = j;
    }
    for (uint32_t i = 0; i < m; ++i) {
        const int64_t v = E.tok2vid[t[i]];
        if (v < 0) atomicOr(status, 4u);
        t[i] = (uint32_t)v;
    }
    w_nids[w] = m;
}

__global__ void k_word_len64(const uint32_t* __restrict__ w_len, unsigned n, unsigned long long* __restrict__ o) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = w_len[i];
}

}  // namespace
}  // namespace bpe

// =================================================================== the tokenizer object
struct bpe_tokenizer {
    std::vector<std::string> specials;     // deduped, longest first
    std::vector<int64_t> special_vid;
    hipStream_t stream = nullptr;
    bpe::DevBuf<unsigned long long> pm_key;
    bpe::DevBuf<uint2> pm_val;
    size_t pm_cap = 0;
    bpe::DevBuf<int64_t> tok2vid;
    bpe::DevBuf<uint32_t> byte2tok;
    bpe::DevBuf<uint8_t> sp_bytes;
    bpe::DevBuf<uint32_t> sp_off, sp_len;
    bpe::DevBuf<int64_t> sp_vid;
    bpe::DevBuf<unsigned> first_mask;
    ~bpe_tokenizer() {
        if (stream) (void)hipStreamDestroy(stream);
    }
    bpe::EncTables tables() const {
        return bpe::EncTables{pm_key.p, pm_val.p, (unsigned long long)(pm_cap - 1), tok2vid.p,
                              byte2tok.p, sp_bytes.p, sp_off.p, sp_len.p, sp_vid.p,
                              (int)specials.size()};
    }
};

namespace bpe {
namespace {

uint32_t rd_u32(const uint8_t*& p, const uint8_t* end) {
    BPE_REQUIRE(p + 4 <= end, BPE_E_ARG, "truncated blob");
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
}

void build_tokenizer(bpe_tokenizer& T, const uint8_t* vb, size_t vn, const uint8_t* mb, size_t mn,
                     const std::vector<std::string>& sp_in) {
    std::unordered_map<std::string, uint32_t> intern;
    std::vector<int64_t> vid;
    auto tok = [&](const std::string& s) {
        auto it = intern.find(s);
        if (it != intern.end()) return it->second;
        const uint32_t id = (uint32_t)intern.size();
        intern.emplace(s, id);
        vid.push_back(-1);
        return id;
    };
    // vocab_inv = {bytes: id}: last id wins (tokenizer.py:19)
    const uint8_t* p = vb;
    const uint8_t* end = vb + vn;
    const uint32_t nv = rd_u32(p, end);
    for (uint32_t i = 0; i < nv; ++i) {
        BPE_REQUIRE(p + 12 <= end, BPE_E_ARG, "truncated vocab blob");
        int64_t id;
        std::memcpy(&id, p, 8);
        p += 8;
        const uint32_t l = rd_u32(p, end);
        BPE_REQUIRE(p + l <= end, BPE_E_ARG, "truncated vocab blob");
        BPE_REQUIRE(id >= 0 && id < (1LL << 32), BPE_E_ARG, "vocab id outside [0, 2^32)");
        vid[tok(std::string((const char*)p, l))] = id;
        p += l;
    }
    // specials: dedupe (first occurrence), longest first; missing ones get ids len(vocab), ...
    for (const auto& s : sp_in) {
        BPE_REQUIRE(!s.empty(), BPE_E_ARG, "empty special token is not supported");
        if (std::find(T.specials.begin(), T.specials.end(), s) == T.specials.end()) T.specials.push_back(s);
    }
    std::stable_sort(T.specials.begin(), T.specials.end(),
                     [](const std::string& x, const std::string& y) { return x.size() > y.size(); });
    int64_t next_id = (int64_t)nv;
    for (const auto& s : T.specials) {
        const uint32_t t = tok(s);
        if (vid[t] < 0) vid[t] = next_id++;
        T.special_vid.push_back(vid[t]);
    }
    // merges: rank = index, later duplicates overwrite (tokenizer.py:115)
    std::unordered_map<unsigned long long, std::pair<uint32_t, uint32_t>> rank;
    p = mb;
    end = mb + mn;
    const uint32_t nm = rd_u32(p, end);
    for (uint32_t i = 0; i < nm; ++i) {
        const uint32_t la = rd_u32(p, end);
        BPE_REQUIRE(p + la <= end, BPE_E_ARG, "truncated merges blob");
        std::string a((const char*)p, la);
        p += la;
        const uint32_t lb = rd_u32(p, end);
        BPE_REQUIRE(p + lb <= end, BPE_E_ARG, "truncated merges blob");
        std::string b((const char*)p, lb);
        p += lb;
        const uint32_t ta = tok(a), tb = tok(b), tp = tok(a + b);
        rank[((unsigned long long)ta << 32) | tb] = {i, tp};
    }
    std::vector<uint32_t> b2t(256);
    for (int b = 0; b < 256; ++b) b2t[b] = tok(std::string(1, (char)b));

    // device tables
    T.pm_cap = next_pow2(std::max<size_t>(64, rank.size() * 2 + 1));
    std::vector<unsigned long long> hk(T.pm_cap, 0);
    std::vector<uint2> hv(T.pm_cap);
    for (const auto& kv : rank) {
        const unsigned long long key = kv.first + 1ULL;
        size_t s = mix64(key) & (T.pm_cap - 1);
        while (hk[s]) s = (s + 1) & (T.pm_cap - 1);
        hk[s] = key;
        hv[s] = make_uint2(kv.second.first, kv.second.second);
    }
    BPE_HIP(hipStreamCreateWithFlags(&T.stream, hipStreamNonBlocking));
    auto up = [&](auto& buf, const auto& vec) {
        buf.alloc(std::max<size_t>(vec.size(), 1));
        if (!vec.empty())
            BPE_HIP(hipMemcpyAsync(buf.p, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice, T.stream));
    };
    up(T.pm_key, hk);
    up(T.pm_val, hv);
    up(T.tok2vid, vid);
    up(T.byte2tok, b2t);
    std::string spb;
    std::vector<uint32_t> spo, spl;
    std::vector<unsigned> fm(8, 0);
    for (const auto& s : T.specials) {
        spo.push_back((uint32_t)spb.size());
        spl.push_back((uint32_t)s.size());
        spb += s;
        const unsigned char c = (unsigned char)s[0];
        fm[c >> 5] |= 1u << (c & 31);
    }
    std::vector<uint8_t> spbv(spb.begin(), spb.end());
    up(T.sp_bytes, spbv);
    up(T.sp_off, spo);
    up(T.sp_len, spl);
    up(T.sp_vid, T.special_vid);
    up(T.first_mask, fm);
    BPE_HIP(hipStreamSynchronize(T.stream));
}

// encode d_text[0..n) into d_out; returns the id count
size_t encode_device(bpe_tokenizer& T, const uint8_t* d_text, size_t n, uint32_t* d_out,
                     hipStream_t s) {
    if (n == 0) return 0;
    EncTables E = T.tables();
    // 1. segments
    std::vector<Seg> segs;
    {
        unsigned long long cnt = 0;
        std::vector<unsigned long long> pos;
        std::vector<int> spk;
        if (!T.specials.empty()) {
            unsigned long long cap = std::max<unsigned long long>(1024, n / 64);
            for (;;) {
                DevBuf<unsigned long long> d_pos(cap);
                DevBuf<unsigned> d_n(1);
                DevBuf<int> d_sp(cap);
                BPE_HIP(hipMemsetAsync(d_n.p, 0, 4, s));
                hipLaunchKernelGGL(k_find_specials, dim3(ceil_div(n, 256)), dim3(256), 0, s, d_text, n, E,
                                   T.first_mask.p, d_pos.p, d_sp.p, d_n.p, cap);
                BPE_HIP(hipGetLastError());
                unsigned cnt32 = 0;
                BPE_HIP(hipMemcpyAsync(&cnt32, d_n.p, 4, hipMemcpyDeviceToHost, s));
                BPE_HIP(hipStreamSynchronize(s));
                cnt = cnt32;
                BPE_HIP(hipStreamSynchronize(s));
                if (cnt > cap) { cap = cnt; continue; }
                pos.resize(cnt);
                spk.resize(cnt);
                if (cnt) {
                    BPE_HIP(hipMemcpyAsync(pos.data(), d_pos.p, cnt * 8, hipMemcpyDeviceToHost, s));
                    BPE_HIP(hipMemcpyAsync(spk.data(), d_sp.p, cnt * 4, hipMemcpyDeviceToHost, s));
                    BPE_HIP(hipStreamSynchronize(s));
                }
                break;
            }
        }
        std::vector<size_t> order(cnt);
        for (size_t i = 0; i < cnt; ++i) order[i] = i;
        std::sort(order.begin(), order.end(), [&](size_t x, size_t y) { return pos[x] < pos[y]; });
        unsigned long long cur = 0;
        for (size_t oi : order) {  // leftmost, non-overlapping (re.split)
            const unsigned long long p0 = pos[oi];
            if (p0 < cur) continue;
            if (p0 > cur) segs.push_back(Seg{cur, p0, -1, 0});
            const unsigned long long e = p0 + T.specials[spk[oi]].size();
            segs.push_back(Seg{p0, e, spk[oi], 0});
            cur = e;
        }
        if (cur < n) segs.push_back(Seg{cur, n, -1, 0});
    }
    const int nseg = (int)segs.size();
    DevBuf<Seg> d_segs(nseg);
    BPE_HIP(hipMemcpyAsync(d_segs.p, segs.data(), nseg * sizeof(Seg), hipMemcpyHostToDevice, s));

    // 2. unique pre-tokens
    const size_t threads = (n + kSpan - 1) / kSpan;
    const unsigned grid = ceil_div(threads, 256);
    size_t cap = next_pow2(std::max<size_t>(1 << 12, n / 48));
    DevBuf<unsigned long long> key;
    DevBuf<unsigned> status(1);
    for (int attempt = 0;; ++attempt) {
        key.alloc(cap);
        BPE_HIP(hipMemsetAsync(key.p, 0, key.bytes(), s));
        BPE_HIP(hipMemsetAsync(status.p, 0, 4, s));
        hipLaunchKernelGGL(k_scan<SCAN_INSERT>, dim3(grid), dim3(256), 0, s, d_text, n, d_segs.p, nseg, E,
                           key.p, cap - 1, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, status.p);
        BPE_HIP(hipGetLastError());
        unsigned st = 0;
        BPE_HIP(hipMemcpyAsync(&st, status.p, 4, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipStreamSynchronize(s));
        if (st & 2u) throw Error{BPE_E_LIMIT, "a pre-token is longer than 16 MiB"};
        if (!(st & 1u)) break;
        BPE_REQUIRE(attempt < 4, BPE_E_NOMEM, "word table overflow");
        cap *= 4;
    }
    DevBuf<uint32_t> slot_word(cap);
    DevBuf<unsigned long long> w_off(cap);
    DevBuf<uint32_t> w_len(cap);
    DevBuf<unsigned> d_nw(1);
    BPE_HIP(hipMemsetAsync(d_nw.p, 0, 4, s));
    hipLaunchKernelGGL(k_collect, dim3(ceil_div(cap, 256)), dim3(256), 0, s, key.p, cap, slot_word.p,
                       w_off.p, w_len.p, d_nw.p);
    unsigned nw = 0;
    BPE_HIP(hipMemcpyAsync(&nw, d_nw.p, 4, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipStreamSynchronize(s));

    // 3. encode each unique word once
    DevBuf<unsigned long long> len64(std::max(nw, 1u)), idoff(std::max(nw, 1u) + 1);
    DevBuf<uint32_t> nids(std::max(nw, 1u));
    unsigned long long pool_n = 0;
    if (nw) {
        hipLaunchKernelGGL(k_word_len64, dim3(ceil_div(nw, 256)), dim3(256), 0, s, w_len.p, nw, len64.p);
        size_t tb = 0;
        BPE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, len64.p, idoff.p, (int)nw + 0, s));
        DevBuf<uint8_t> tmp(tb);
        BPE_HIP(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, len64.p, idoff.p, (int)nw, s));
        unsigned long long last[2];
        BPE_HIP(hipMemcpyAsync(&last[0], idoff.p + nw - 1, 8, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipMemcpyAsync(&last[1], len64.p + nw - 1, 8, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipStreamSynchronize(s));
        pool_n = last[0] + last[1];
    }
    DevBuf<uint32_t> pool(std::max<unsigned long long>(pool_n, 1));
    BPE_HIP(hipMemsetAsync(status.p, 0, 4, s));
    if (nw) {
        hipLaunchKernelGGL(k_encode_words, dim3(ceil_div(nw, 256)), dim3(256), 0, s, d_text, E, w_off.p,
                           w_len.p, idoff.p, nw, pool.p, nids.p, status.p);
        BPE_HIP(hipGetLastError());
    }
    // 4. output offsets per thread, then write
    DevBuf<unsigned long long> per(threads), per_off(threads);
    hipLaunchKernelGGL(k_scan<SCAN_COUNT>, dim3(grid), dim3(256), 0, s, d_text, n, d_segs.p, nseg, E,
                       key.p, cap - 1, slot_word.p, nids.p, idoff.p, pool.p, per.p, nullptr, status.p);
    size_t tb = 0;
    BPE_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, per.p, per_off.p, (int64_t)threads, s));
    DevBuf<uint8_t> tmp(tb);
    BPE_HIP(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, per.p, per_off.p, (int64_t)threads, s));
    unsigned long long last[2];
    unsigned st = 0;
    BPE_HIP(hipMemcpyAsync(&last[0], per_off.p + threads - 1, 8, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipMemcpyAsync(&last[1], per.p + threads - 1, 8, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipMemcpyAsync(&st, status.p, 4, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipStreamSynchronize(s));
    if (st & 4u) throw Error{BPE_E_KEY, "a merged token is not in the vocab"};
    BPE_REQUIRE(!(st & 8u), BPE_E_HIP, "encode lost a pre-token between passes");
    const size_t total = last[0] + last[1];
    BPE_REQUIRE(total <= n, BPE_E_HIP, "encode produced more ids than input bytes");
    hipLaunchKernelGGL(k_scan<SCAN_WRITE>, dim3(grid), dim3(256), 0, s, d_text, n, d_segs.p, nseg, E,
                       key.p, cap - 1, slot_word.p, nids.p, idoff.p, pool.p, per_off.p, d_out, status.p);
    BPE_HIP(hipGetLastError());
    BPE_HIP(hipStreamSynchronize(s));
    return total;
}

template <class F>
int guarded_enc(F&& f) {
    try {
        f();
        set_error(0, "");
        return BPE_OK;
    } catch (const Error& e) {
        set_error(e.code, e.msg);
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error(BPE_E_NOMEM, "host allocation failed");
        return BPE_E_NOMEM;
    }
}

}  // namespace
}  // namespace bpe

extern "C" {

int bpe_tok_create(const uint8_t* vocab_blob, size_t vocab_n, const uint8_t* merges_blob, size_t merges_n,
                   const char* const* specials, int n_specials, bpe_tokenizer** out) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(out && vocab_blob && merges_blob, BPE_E_ARG, "NULL argument");
        BPE_REQUIRE(n_specials >= 0 && (n_specials == 0 || specials), BPE_E_ARG, "bad specials");
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            throw bpe::Error{BPE_E_HIP, "no HIP device visible (libbpe355 needs an MI355X / gfx950 GPU)"};
        std::vector<std::string> sp;
        for (int i = 0; i < n_specials; ++i) {
            BPE_REQUIRE(specials[i], BPE_E_ARG, "null special");
            sp.emplace_back(specials[i]);
        }
        auto T = std::make_unique<bpe_tokenizer>();
        bpe::build_tokenizer(*T, vocab_blob, vocab_n, merges_blob, merges_n, sp);
        *out = T.release();
    });
}

int64_t bpe_tok_special_id(const bpe_tokenizer* tok, int i) {
    if (!tok || i < 0 || i >= (int)tok->special_vid.size()) return -1;
    return tok->special_vid[i];
}

int bpe_tok_encode(bpe_tokenizer* tok, const uint8_t* utf8, size_t n, uint32_t* ids_out, size_t cap,
                   size_t* n_out) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(tok && n_out && (n == 0 || (utf8 && ids_out)), BPE_E_ARG, "NULL argument");
        BPE_REQUIRE(cap >= n, BPE_E_ARG, "ids_out capacity must be >= input bytes");
        *n_out = 0;
        if (n == 0) return;
        bpe::DevBuf<uint8_t> d_text(n);
        bpe::DevBuf<uint32_t> d_out(n);
        BPE_HIP(hipMemcpyAsync(d_text.p, utf8, n, hipMemcpyHostToDevice, tok->stream));
        const size_t m = bpe::encode_device(*tok, d_text.p, n, d_out.p, tok->stream);
        if (m) BPE_HIP(hipMemcpyAsync(ids_out, d_out.p, m * 4, hipMemcpyDeviceToHost, tok->stream));
        BPE_HIP(hipStreamSynchronize(tok->stream));
        *n_out = m;
    });
}

int bpe_tok_encode_device(bpe_tokenizer* tok, const uint8_t* d_utf8, size_t n, uint32_t* d_out,
                          size_t* n_out, void* hip_stream) {
    return bpe::guarded_enc([&] {
        BPE_REQUIRE(tok && n_out && (n == 0 || (d_utf8 && d_out)), BPE_E_ARG, "NULL argument");
        hipStream_t s = hip_stream ? (hipStream_t)hip_stream : tok->stream;
        *n_out = bpe::encode_device(*tok, d_utf8, n, d_out, s);
    });
}

void bpe_tok_free(bpe_tokenizer* tok) { delete tok; }

}  // extern "C"
