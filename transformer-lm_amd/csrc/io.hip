// Bulk-encode plumbing on the device, for the reference's dataset encoder
// (models/tokenizer/encode.py:31-38) and its consumer (train.py:230-232):
//   bpe_text_prepare_device      open(path, "r", encoding="utf-8").read(): strict UTF-8 and
//                                universal newlines (text.hip prepare_text)
//   bpe_utf8_chunk_starts_device byte offsets of characters 0, K, 2K, ... -- the pieces
//                                f.read(K) returns one after another
//   bpe_ids_to_u16_device        np.array(token_ids, dtype=np.uint16), refusing ids > 65535
//                                instead of wrapping them

#include <algorithm>
#include <vector>

#include <sys/stat.h>

#include "drive.h"
#include "internal.h"
#include "prims.h"

namespace bpe {
namespace {

// Character counting for the pieces: a workgroup owns kCharBlock bytes and reads them as
// coalesced 16-byte units (thread t takes unit i * 256 + t in round i); a byte starts a character
// unless it is a continuation byte 10xxxxxx, counted four at a time with one AND-NOT and a popcount.
constexpr int kCharThreads = 256;
constexpr int kCharRounds = 16;
constexpr size_t kCharBlock = (size_t)kCharThreads * 16 * kCharRounds;   // 64 KiB

// bit 7 of each byte of x set iff that byte is a continuation byte
__device__ __forceinline__ uint32_t cont_bits(uint32_t x) { return x & ~(x << 1) & 0x80808080u; }

// the 16 bytes of unit u as four words (bytes past n read 0x80, a continuation: never counted)
__device__ __forceinline__ uint4 load_unit(const uint8_t* __restrict__ s, size_t n, size_t u) {
    const size_t lo = u * 16;
    if (lo + 16 <= n && ((uintptr_t)(s + lo) & 15u) == 0) return *reinterpret_cast<const uint4*>(s + lo);
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const size_t i = lo + 4 * k + j;
            x |= (uint32_t)(i < n ? s[i] : 0x80u) << (8 * j);
        }
        w[k] = x;
    }
    return uint4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ unsigned unit_chars(const uint4 v) {
    return 16u - (unsigned)(__popc(cont_bits(v.x)) + __popc(cont_bits(v.y)) + __popc(cont_bits(v.z)) +
                            __popc(cont_bits(v.w)));
}

__global__ void __launch_bounds__(kCharThreads) k_char_count(const uint8_t* __restrict__ s, size_t n,
                                                             unsigned long long* __restrict__ cnt) {
    __shared__ unsigned s_part[kCharThreads / 64];
    const size_t b = blockIdx.x, u0 = b * (kCharBlock / 16);
    unsigned c = 0;
#pragma unroll 4
    for (int i = 0; i < kCharRounds; ++i) {
        const size_t u = u0 + (size_t)i * kCharThreads + threadIdx.x;
        if (u * 16 < n) c += unit_chars(load_unit(s, n, u));
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[b] = (unsigned long long)s_part[0] + s_part[1] + s_part[2] + s_part[3];
}

// marks[c / k - mark0] = byte offset of character c for every c % k == 0 (c counted from c_base
// at the start of the text given); a block none of whose
// characters [first, first + cnt) is a multiple of k returns at once (all but ~1 in 16 at
// 1 M-character pieces)
__global__ void __launch_bounds__(kCharThreads) k_char_marks(const uint8_t* __restrict__ s, size_t n,
                                                             const unsigned long long* __restrict__ first,
                                                             const unsigned long long* __restrict__ cnt,
                                                             unsigned long long k, unsigned long long c_base,
                                                             unsigned long long mark0,
                                                             unsigned long long* __restrict__ marks) {
    typedef rocprim::block_scan<unsigned, kCharThreads> Scan;
    __shared__ typename Scan::storage_type tmp;
    const size_t b = blockIdx.x, u0 = b * (kCharBlock / 16);
    unsigned long long c0 = c_base + first[b];
    const unsigned long long cb = cnt[b];
    if (cb == 0 || (c0 + k - 1) / k * k >= c0 + cb) return;   // uniform over the block
    for (int i = 0; i < kCharRounds; ++i) {
        const size_t u = u0 + (size_t)i * kCharThreads + threadIdx.x;
        const bool in = u * 16 < n;
        const uint4 v = in ? load_unit(s, n, u) : uint4{0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u};
        const unsigned m = in ? unit_chars(v) : 0u;
        unsigned before = 0, total = 0;
        Scan().exclusive_scan(m, before, 0u, total, tmp);
        unsigned long long c = c0 + before;
        if (m && (c + k - 1) / k * k < c + m) {   // a multiple of k among this unit's characters
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            for (int j = 0; j < 16; ++j) {
                const uint32_t byte = (w[j >> 2] >> (8 * (j & 3))) & 0xffu;
                if ((byte & 0xC0u) == 0x80u) continue;
                if (c % k == 0) marks[c / k - mark0] = u * 16 + (size_t)j;
                ++c;
            }
        }
        c0 += total;
        __syncthreads();   // the scan's storage is reused next round
    }
}

__global__ void k_narrow_u16(const uint32_t* __restrict__ ids, size_t n, uint16_t* __restrict__ out,
                             unsigned* __restrict__ over) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t v = ids[i];
        if (v > 0xFFFFu) atomicOr(over, 1u);
        out[i] = (uint16_t)v;
    }
}

template <class F>
int guarded_io(F&& f) {
    try {
        f();
        set_error(0, "");
        return BPE_OK;
    } catch (const Error& e) {
        set_error(e.code, e.msg, e.sys_errno);
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error(BPE_E_NOMEM, "host allocation failed");
        return BPE_E_NOMEM;
    }
}

}  // namespace

uint64_t piece_starts_range(const uint8_t* d_text, size_t n, size_t k, uint64_t c_base, uint64_t offset,
                            hipStream_t s, std::vector<uint64_t>& out, PieceScratch* scratch) {
    if (n == 0) return 0;
    const size_t blocks = (n + kCharBlock - 1) / kCharBlock;
    PieceScratch local;
    PieceScratch& S = scratch ? *scratch : local;
    S.cnt.reserve(blocks);
    S.first.reserve(blocks);
    DevBuf<unsigned long long>&cnt = S.cnt, &first = S.first;
    hipLaunchKernelGGL(k_char_count, dim3(blocks), dim3(kCharThreads), 0, s, d_text, n, cnt.p);
    BPE_HIP(hipGetLastError());
    exclusive_sum(cnt.p, first.p, blocks, s, &S.tmp);
    unsigned long long last[2];
    to_host(&last[0], first.p + blocks - 1, 8, s);
    to_host(&last[1], cnt.p + blocks - 1, 8, s);
    const unsigned long long chars = last[0] + last[1];
    // the multiples of k in [c_base, c_base + chars)
    const unsigned long long mark0 = (c_base + k - 1) / k, mark1 = (c_base + chars + k - 1) / k;
    if (mark1 > mark0) {
        const size_t m = (size_t)(mark1 - mark0);
        S.marks.reserve(m);
        DevBuf<unsigned long long>& marks = S.marks;
        hipLaunchKernelGGL(k_char_marks, dim3(blocks), dim3(kCharThreads), 0, s, d_text, n, first.p, cnt.p,
                           (unsigned long long)k, (unsigned long long)c_base, mark0, marks.p);
        BPE_HIP(hipGetLastError());
        const size_t at = out.size();
        out.resize(at + m);
        to_host(out.data() + at, marks.p, m * 8, s);
        for (size_t i = at; i < out.size(); ++i) out[i] += offset;
    }
    return chars;
}

std::vector<uint64_t> utf8_piece_starts(const uint8_t* d_text, size_t n, size_t k, hipStream_t s) {
    std::vector<uint64_t> out;
    piece_starts_range(d_text, n, k, 0, 0, s, out);
    return out;
}

}  // namespace bpe

extern "C" {

int bpe_read_file_device(const char* path, uint8_t* d_dst, size_t cap, size_t* n_out) {
    return bpe::guarded_io([&] {
        BPE_REQUIRE(path && n_out, BPE_E_ARG, "NULL argument");
        *n_out = 0;
        struct stat st;
        if (::stat(path, &st) == 0 && !S_ISREG(st.st_mode) && !S_ISDIR(st.st_mode))
            throw bpe::Error{BPE_E_IO, std::string("not a regular file: ") + path, EINVAL};
        const bpe::Source src = bpe::Source::open_path(path);   // missing file / directory: errno
        *n_out = src.size;
        if (!d_dst) return;
        BPE_REQUIRE(cap >= src.size, BPE_E_ARG, "device buffer smaller than the file");
        int dev = 0;
        BPE_HIP(hipGetDevice(&dev));
        bpe::stage_to_device(src, 0, src.size, d_dst, dev, bpe::io_threads());
    });
}

int bpe_copy_to_host(const void* d_src, size_t n, void* h_dst) {
    return bpe::guarded_io([&] {
        BPE_REQUIRE(n == 0 || (d_src && h_dst), BPE_E_ARG, "NULL argument");
        int dev = 0;
        BPE_HIP(hipGetDevice(&dev));
        BPE_HIP(hipDeviceSynchronize());   // the caller's writes (any stream) are done
        bpe::device_to_host(static_cast<const uint8_t*>(d_src), n, static_cast<uint8_t*>(h_dst), dev,
                            bpe::io_threads());
    });
}

int bpe_text_prepare_device(const uint8_t* d_in, size_t n, uint8_t* d_out, size_t* n_out, void* hip_stream) {
    return bpe::guarded_io([&] {
        BPE_REQUIRE(n_out && (n == 0 || (d_in && d_out)), BPE_E_ARG, "NULL argument");
        hipStream_t s = (hipStream_t)hip_stream;
        *n_out = 0;
        if (n == 0) return;
        bpe::DevBuf<uint8_t> scratch;
        size_t m = 0;
        const uint8_t* p = bpe::prepare_text(d_in, n, scratch, &m, s);
        if (p != d_out && m) BPE_HIP(hipMemcpyAsync(d_out, p, m, hipMemcpyDeviceToDevice, s));
        BPE_HIP(hipStreamSynchronize(s));
        *n_out = m;
    });
}

int bpe_utf8_chunk_starts_device(const uint8_t* d_text, size_t n, size_t chars_per_chunk, uint64_t* starts,
                                 size_t cap, size_t* n_starts, void* hip_stream) {
    return bpe::guarded_io([&] {
        BPE_REQUIRE(n_starts && chars_per_chunk > 0 && (n == 0 || d_text), BPE_E_ARG, "bad argument");
        *n_starts = 0;
        if (n == 0) return;
        const std::vector<uint64_t> m = bpe::utf8_piece_starts(d_text, n, chars_per_chunk, (hipStream_t)hip_stream);
        *n_starts = m.size();
        if (!starts) return;   // size query
        BPE_REQUIRE(cap >= m.size(), BPE_E_ARG, "starts capacity too small");
        std::copy(m.begin(), m.end(), starts);
    });
}

int bpe_ids_to_u16_device(const uint32_t* d_ids, size_t n, uint16_t* d_out, void* hip_stream) {
    return bpe::guarded_io([&] {
        BPE_REQUIRE(n == 0 || (d_ids && d_out), BPE_E_ARG, "NULL argument");
        hipStream_t s = (hipStream_t)hip_stream;
        if (n == 0) return;
        bpe::DevBuf<unsigned> over(1);
        BPE_HIP(hipMemsetAsync(over.p, 0, 4, s));
        hipLaunchKernelGGL(bpe::k_narrow_u16, dim3(bpe::grid_for(n, 256)), dim3(256), 0, s, d_ids, n, d_out, over.p);
        BPE_HIP(hipGetLastError());
        unsigned o = 0;
        BPE_HIP(hipMemcpyAsync(&o, over.p, 4, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipStreamSynchronize(s));
        BPE_REQUIRE(!o, BPE_E_LIMIT, "a token id does not fit uint16 (vocab larger than 65536)");
    });
}

}  // extern "C"
