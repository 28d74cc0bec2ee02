// Bulk-encode plumbing on the device, for the reference's dataset encoder
// (models/tokenizer/encode.py:31-38) and its consumer (train.py:230-232):
//   bpe_text_prepare_device      open(path, "r", encoding="utf-8").read(): strict UTF-8 and
//                                universal newlines (text.hip prepare_text)
//   bpe_utf8_chunk_starts_device byte offsets of characters 0, K, 2K, ... -- the pieces
//                                f.read(K) returns one after another
//   bpe_ids_to_u16_device        np.array(token_ids, dtype=np.uint16), refusing ids > 65535
//                                instead of wrapping them

#include <vector>

#include <sys/stat.h>

#include "drive.h"
#include "internal.h"
#include "prims.h"

namespace bpe {
namespace {

constexpr size_t kCharSpan = 4096;   // bytes per thread when counting characters

__device__ __forceinline__ bool is_lead(uint8_t b) { return (b & 0xC0u) != 0x80u; }

__global__ void k_char_count(const uint8_t* __restrict__ s, size_t n, unsigned long long* __restrict__ cnt) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t lo = t * kCharSpan;
    if (lo >= n) return;
    const size_t hi = lo + kCharSpan < n ? lo + kCharSpan : n;
    unsigned long long c = 0;
    for (size_t i = lo; i < hi; ++i) c += is_lead(s[i]);
    cnt[t] = c;
}

__global__ void k_char_marks(const uint8_t* __restrict__ s, size_t n, const unsigned long long* __restrict__ first,
                             unsigned long long k, unsigned long long* __restrict__ marks) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t lo = t * kCharSpan;
    if (lo >= n) return;
    const size_t hi = lo + kCharSpan < n ? lo + kCharSpan : n;
    unsigned long long c = first[t];   // characters before this span
    for (size_t i = lo; i < hi; ++i) {
        if (!is_lead(s[i])) continue;
        if (c % k == 0) marks[c / k] = i;
        ++c;
    }
}

__global__ void k_narrow_u16(const uint32_t* __restrict__ ids, size_t n, uint16_t* __restrict__ out,
                             unsigned* __restrict__ over) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = ids[i];
    if (v > 0xFFFFu) atomicOr(over, 1u);
    out[i] = (uint16_t)v;
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
        hipStream_t s = (hipStream_t)hip_stream;
        *n_starts = 0;
        if (n == 0) return;
        const size_t threads = (n + bpe::kCharSpan - 1) / bpe::kCharSpan;
        bpe::DevBuf<unsigned long long> cnt(threads), first(threads);
        hipLaunchKernelGGL(bpe::k_char_count, dim3(bpe::ceil_div(threads, 256)), dim3(256), 0, s, d_text, n, cnt.p);
        bpe::exclusive_sum(cnt.p, first.p, threads, s);
        unsigned long long last[2];
        BPE_HIP(hipMemcpyAsync(&last[0], first.p + threads - 1, 8, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipMemcpyAsync(&last[1], cnt.p + threads - 1, 8, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipStreamSynchronize(s));
        const unsigned long long chars = last[0] + last[1];
        const size_t m = (size_t)((chars + chars_per_chunk - 1) / chars_per_chunk);
        *n_starts = m;
        if (!starts || cap < m) {   // size query
            BPE_REQUIRE(!starts, BPE_E_ARG, "starts capacity too small");
            return;
        }
        bpe::DevBuf<unsigned long long> marks(std::max<size_t>(m, 1));
        hipLaunchKernelGGL(bpe::k_char_marks, dim3(bpe::ceil_div(threads, 256)), dim3(256), 0, s, d_text, n,
                           first.p, (unsigned long long)chars_per_chunk, marks.p);
        BPE_HIP(hipGetLastError());
        if (m) BPE_HIP(hipMemcpyAsync(starts, marks.p, m * 8, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipStreamSynchronize(s));
    });
}

int bpe_ids_to_u16_device(const uint32_t* d_ids, size_t n, uint16_t* d_out, void* hip_stream) {
    return bpe::guarded_io([&] {
        BPE_REQUIRE(n == 0 || (d_ids && d_out), BPE_E_ARG, "NULL argument");
        hipStream_t s = (hipStream_t)hip_stream;
        if (n == 0) return;
        bpe::DevBuf<unsigned> over(1);
        BPE_HIP(hipMemsetAsync(over.p, 0, 4, s));
        hipLaunchKernelGGL(bpe::k_narrow_u16, dim3(bpe::ceil_div(n, 256)), dim3(256), 0, s, d_ids, n, d_out, over.p);
        BPE_HIP(hipGetLastError());
        unsigned o = 0;
        BPE_HIP(hipMemcpyAsync(&o, over.p, 4, hipMemcpyDeviceToHost, s));
        BPE_HIP(hipStreamSynchronize(s));
        BPE_REQUIRE(!o, BPE_E_LIMIT, "a token id does not fit uint16 (vocab larger than 65536)");
    });
}

}  // extern "C"
