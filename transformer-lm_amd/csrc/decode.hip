// Tokenizer.decode on the device -- reference
// models/tokenizer/tokenizer.py:155-157:
//     raw_bytes = b"".join([self.vocab[i] for i in ids])      <- here: a gather on the GPU
//     return raw_bytes.decode("utf-8", errors="replace")     <- the caller (CPython's decoder,
//                                                               so the replacement rule is exact)
// self.vocab[i] raises KeyError for an id it lacks: BPE_E_KEY here.
//
// Layout: a dense (offset, length) table over ids 0..max_id (length ~0 = no such id) and one
// byte pool.  Decoding: length lookup -> exclusive scan -> one thread per id copies its bytes.

#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "internal.h"
#include "prims.h"

struct bpe_decoder {
    bpe::DevBuf<unsigned long long> off;
    bpe::DevBuf<uint32_t> len;
    bpe::DevBuf<uint8_t> pool;
    uint64_t n_ids = 0;   // table size (max id + 1)
    hipStream_t stream = nullptr;
    ~bpe_decoder() {
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace bpe {
namespace {

constexpr uint32_t kNoId = 0xffffffffu;
constexpr uint64_t kMaxDecodeIds = 1ull << 28;   // dense table bound (vocab ids are dense in practice)

__global__ void k_dec_len(const uint32_t* __restrict__ ids, size_t n, const uint32_t* __restrict__ len,
                          uint64_t n_tab, unsigned long long* __restrict__ out_len,
                          unsigned long long* __restrict__ first_bad) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t id = ids[i];
        const uint32_t l = id < n_tab ? len[id] : kNoId;
        if (l == kNoId) {
            atomicMin(first_bad, (unsigned long long)i);
            out_len[i] = 0;
            continue;
        }
        out_len[i] = l;
    }
}

__global__ void k_dec_gather(const uint32_t* __restrict__ ids, size_t n, const unsigned long long* __restrict__ off,
                             const uint32_t* __restrict__ len, const uint8_t* __restrict__ pool,
                             const unsigned long long* __restrict__ out_off, uint8_t* __restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t id = ids[i];
        const uint32_t l = len[id];
        const uint8_t* src = pool + off[id];
        uint8_t* dst = out + out_off[i];
        for (uint32_t k = 0; k < l; ++k) dst[k] = src[k];
    }
}

template <class F>
int guarded_dec(F&& f) {
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

// d_ids -> bytes at d_out (capacity cap); returns the byte count (or throws)
size_t decode_device(bpe_decoder& D, const uint32_t* d_ids, size_t n, uint8_t* d_out, size_t cap,
                     size_t* needed, hipStream_t s) {
    *needed = 0;
    if (n == 0) return 0;
    DevBuf<unsigned long long> lens(n), offs(n), bad(1);
    const unsigned long long none = ~0ULL;
    BPE_HIP(hipMemcpyAsync(bad.p, &none, 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_dec_len, dim3(grid_for(n, 256)), dim3(256), 0, s, d_ids, n, D.len.p, D.n_ids, lens.p,
                       bad.p);
    exclusive_sum(lens.p, offs.p, n, s);
    unsigned long long h[3];
    BPE_HIP(hipMemcpyAsync(&h[0], offs.p + n - 1, 8, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipMemcpyAsync(&h[1], lens.p + n - 1, 8, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipMemcpyAsync(&h[2], bad.p, 8, hipMemcpyDeviceToHost, s));
    BPE_HIP(hipStreamSynchronize(s));
    if (h[2] != none) {
        uint32_t id = 0;
        BPE_HIP(hipMemcpy(&id, d_ids + h[2], 4, hipMemcpyDeviceToHost));
        throw Error{BPE_E_KEY, std::to_string(id)};
    }
    const size_t total = (size_t)(h[0] + h[1]);
    *needed = total;
    BPE_REQUIRE(cap >= total, BPE_E_ARG, "decode output capacity too small");
    hipLaunchKernelGGL(k_dec_gather, dim3(grid_for(n, 256)), dim3(256), 0, s, d_ids, n, D.off.p, D.len.p,
                       D.pool.p, offs.p, d_out);
    BPE_HIP(hipGetLastError());
    BPE_HIP(hipStreamSynchronize(s));
    return total;
}

}  // namespace
}  // namespace bpe

extern "C" {

int bpe_dec_create(const uint8_t* vocab_blob, size_t vocab_n, bpe_decoder** out) {
    return bpe::guarded_dec([&] {
        BPE_REQUIRE(out && (vocab_n == 0 || vocab_blob), BPE_E_ARG, "NULL argument");
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
            throw bpe::Error{BPE_E_HIP, "no HIP device visible (libbpe355 needs an MI355X / gfx950 GPU)"};
        // blob: u32 count, then (i64 id, u32 len, bytes) per entry
        const uint8_t* p = vocab_blob;
        const uint8_t* end = vocab_blob + vocab_n;
        BPE_REQUIRE(vocab_n >= 4, BPE_E_ARG, "truncated vocab blob");
        uint32_t nv;
        std::memcpy(&nv, p, 4);
        p += 4;
        std::vector<std::pair<uint64_t, std::string>> ents;
        uint64_t max_id = 0;
        for (uint32_t i = 0; i < nv; ++i) {
            BPE_REQUIRE(p + 12 <= end, BPE_E_ARG, "truncated vocab blob");
            int64_t id;
            uint32_t l;
            std::memcpy(&id, p, 8);
            std::memcpy(&l, p + 8, 4);
            p += 12;
            BPE_REQUIRE(p + l <= end, BPE_E_ARG, "truncated vocab blob");
            BPE_REQUIRE(id >= 0 && (uint64_t)id < bpe::kMaxDecodeIds, BPE_E_LIMIT, "vocab id outside [0, 2^28)");
            ents.emplace_back((uint64_t)id, std::string((const char*)p, l));
            max_id = std::max<uint64_t>(max_id, (uint64_t)id);
            p += l;
        }
        auto D = std::make_unique<bpe_decoder>();
        D->n_ids = ents.empty() ? 0 : max_id + 1;
        std::vector<unsigned long long> off(std::max<uint64_t>(D->n_ids, 1), 0);
        std::vector<uint32_t> len(std::max<uint64_t>(D->n_ids, 1), bpe::kNoId);
        std::string pool;
        for (const auto& e : ents) {   // a repeated id: the later entry wins, as in a dict literal
            off[e.first] = pool.size();
            len[e.first] = (uint32_t)e.second.size();
            pool += e.second;
        }
        BPE_HIP(hipStreamCreateWithFlags(&D->stream, hipStreamNonBlocking));
        D->off.alloc(off.size());
        D->len.alloc(len.size());
        D->pool.alloc(std::max<size_t>(pool.size(), 1));
        BPE_HIP(hipMemcpyAsync(D->off.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, D->stream));
        BPE_HIP(hipMemcpyAsync(D->len.p, len.data(), len.size() * 4, hipMemcpyHostToDevice, D->stream));
        if (!pool.empty())
            BPE_HIP(hipMemcpyAsync(D->pool.p, pool.data(), pool.size(), hipMemcpyHostToDevice, D->stream));
        BPE_HIP(hipStreamSynchronize(D->stream));
        *out = D.release();
    });
}

int bpe_dec_decode(bpe_decoder* dec, const uint32_t* ids, size_t n, uint8_t* out, size_t cap, size_t* n_out) {
    return bpe::guarded_dec([&] {
        BPE_REQUIRE(dec && n_out && (n == 0 || ids), BPE_E_ARG, "NULL argument");
        *n_out = 0;
        if (n == 0) return;
        bpe::DevBuf<uint32_t> d_ids(n);
        BPE_HIP(hipMemcpyAsync(d_ids.p, ids, n * 4, hipMemcpyHostToDevice, dec->stream));
        // size first, then gather into a device buffer of exactly that size
        size_t needed = 0;
        try {
            bpe::decode_device(*dec, d_ids.p, n, nullptr, 0, &needed, dec->stream);
        } catch (const bpe::Error& e) {
            if (e.code != BPE_E_ARG) throw;
        }
        *n_out = needed;
        BPE_REQUIRE(out || needed == 0, BPE_E_ARG, "NULL output");
        BPE_REQUIRE(cap >= needed, BPE_E_ARG, "decode output capacity too small");
        bpe::DevBuf<uint8_t> d_out(std::max<size_t>(needed, 1));
        const size_t m = bpe::decode_device(*dec, d_ids.p, n, d_out.p, needed, &needed, dec->stream);
        if (m) BPE_HIP(hipMemcpyAsync(out, d_out.p, m, hipMemcpyDeviceToHost, dec->stream));
        BPE_HIP(hipStreamSynchronize(dec->stream));
    });
}

int bpe_dec_decode_device(bpe_decoder* dec, const uint32_t* d_ids, size_t n, uint8_t* d_out, size_t cap,
                          size_t* n_out, void* hip_stream) {
    return bpe::guarded_dec([&] {
        BPE_REQUIRE(dec && n_out && (n == 0 || d_ids), BPE_E_ARG, "NULL argument");
        hipStream_t s = hip_stream ? (hipStream_t)hip_stream : dec->stream;
        size_t needed = 0;
        *n_out = 0;
        try {
            *n_out = bpe::decode_device(*dec, d_ids, n, d_out, cap, &needed, s);
        } catch (const bpe::Error& e) {
            if (e.code == BPE_E_ARG) *n_out = needed;   // capacity too small: report the size
            throw;
        }
    });
}

void bpe_dec_free(bpe_decoder* dec) { delete dec; }

}  // extern "C"
