// Small host <-> device transfers that must not queue behind bulk DMA.  The bulk encoder streams
// the file in (stage_to_device) and the ids out (device_to_host) on the copy engines while the
// encode runs; the encode's own scalar read-backs (counts, last offsets, status words) and its
// segment table would wait behind those multi-GB transfers if they were copies too.  Here a
// kernel moves them through a pinned, device-mapped host buffer: stores and loads over the bus,
// no copy-engine queue.  Synchronous with respect to the host, ordered on the caller's stream.
#include <algorithm>
#include <cstring>

#include "internal.h"

namespace bpe {
namespace {

constexpr size_t kMailbox = 8u << 20;   // bytes per thread-local staging buffer

__global__ void k_blit(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15u) == 0) {
        const size_t n16 = n / 16;
        for (size_t i = t; i < n16; i += stride)
            reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
        for (size_t i = n16 * 16 + t; i < n; i += stride) dst[i] = src[i];
    } else {
        for (size_t i = t; i < n; i += stride) dst[i] = src[i];
    }
}

struct Mailbox {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    Mailbox() {
        BPE_HIP(hipHostMalloc(reinterpret_cast<void**>(&host), kMailbox,
                              hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
        BPE_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), host, 0));
    }
    ~Mailbox() {
        if (host) (void)hipHostFree(host);
    }
};
Mailbox& mailbox() {
    thread_local Mailbox m;
    return m;
}

void blit(const uint8_t* src, uint8_t* dst, size_t n, hipStream_t s) {
    const unsigned blocks = (unsigned)std::min<size_t>(1024, std::max<size_t>(1, (n / 16 + 255) / 256));
    hipLaunchKernelGGL(k_blit, dim3(blocks), dim3(256), 0, s, src, dst, n);
    BPE_HIP(hipGetLastError());
}

}  // namespace

void to_host(void* dst, const void* d_src, size_t bytes, hipStream_t s) {
    Mailbox& m = mailbox();
    for (size_t off = 0; off < bytes; off += kMailbox) {
        const size_t k = std::min(kMailbox, bytes - off);
        blit(static_cast<const uint8_t*>(d_src) + off, m.dev, k, s);
        BPE_HIP(hipStreamSynchronize(s));
        std::memcpy(static_cast<uint8_t*>(dst) + off, m.host, k);
    }
}

void to_device(void* d_dst, const void* src, size_t bytes, hipStream_t s) {
    Mailbox& m = mailbox();
    for (size_t off = 0; off < bytes; off += kMailbox) {
        const size_t k = std::min(kMailbox, bytes - off);
        std::memcpy(m.host, static_cast<const uint8_t*>(src) + off, k);
        blit(m.dev, static_cast<uint8_t*>(d_dst) + off, k, s);
        BPE_HIP(hipStreamSynchronize(s));   // the mailbox is refilled next round
    }
}

}  // namespace bpe
