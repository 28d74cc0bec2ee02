// Deterministic synthetic corpora (synth_gen.h): the device writer used by bench.py and the GPU
// parity tests, and its host twin, which writes the identical bytes for the oracle.
#include <algorithm>
#include <thread>
#include <vector>

#include "internal.h"
#include "synth_gen.h"

namespace bpe {
namespace {

__global__ void k_synth(uint8_t* __restrict__ out, size_t n, unsigned long long seed, int flavour,
                        unsigned long long first_block) {
    const size_t lb = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t lo = lb * synth::kBlock;
    if (lo >= n) return;
    const size_t len = (n - lo < synth::kBlock) ? n - lo : synth::kBlock;
    synth::block(out + lo, len, seed, flavour, lb + first_block);
}

}  // namespace
}  // namespace bpe

extern "C" int bpe_synth_corpus_device(uint8_t* d_out, size_t n, uint64_t seed, int flavour,
                                       uint64_t first_block, void* hip_stream) {
    if (!d_out && n) return BPE_E_ARG;
    if (n == 0) return BPE_OK;
    hipStream_t s = (hipStream_t)hip_stream;
    const size_t blocks = (n + bpe::synth::kBlock - 1) / bpe::synth::kBlock;
    hipLaunchKernelGGL(bpe::k_synth, dim3(bpe::ceil_div(blocks, 128)), dim3(128), 0, s, d_out, n,
                       (unsigned long long)seed, flavour, (unsigned long long)first_block);
    if (hipGetLastError() != hipSuccess) return BPE_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return BPE_E_HIP;
    return BPE_OK;
}

extern "C" int bpe_synth_corpus_host(uint8_t* out, size_t n, uint64_t seed, int flavour,
                                     uint64_t first_block, int n_threads) {
    using bpe::synth::kBlock;
    if (!out && n) return BPE_E_ARG;
    const size_t blocks = (n + kBlock - 1) / kBlock;
    auto work = [=](size_t b0, size_t b1) {
        for (size_t b = b0; b < b1; ++b) {
            const size_t lo = b * kBlock, len = std::min(kBlock, n - lo);
            bpe::synth::block(out + lo, len, seed, flavour, b + first_block);
        }
    };
    const size_t t = (size_t)std::max(1, std::min(n_threads, 256));
    if (t == 1 || blocks < 64) {
        work(0, blocks);
        return BPE_OK;
    }
    std::vector<std::thread> th;
    for (size_t i = 0; i < t; ++i) th.emplace_back(work, blocks * i / t, blocks * (i + 1) / t);
    for (auto& x : th) x.join();
    return BPE_OK;
}
