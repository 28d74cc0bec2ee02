// Micro-benchmark: how fast one XCD gathers a merge round's words (a posting list of word
// indices -> 64-byte slots in a 512 MB table), against the whole chip.
//   hipcc -O3 --offload-arch=gfx950 xcd_gather.hip -o xcd_gather && ./xcd_gather
// One-XCD launches keep only the workgroups whose HW_REG_XCC_ID equals that of block 0's XCD
// group (blockIdx % 8 == 0 under round-robin placement; the kernel checks the register itself,
// so a different placement only changes the speed).  Slot loads: plain, or sc1 (8-byte relaxed
// agent-scope atomic loads, L1 bypass).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

template <bool SC1>
__global__ void k_gather(const unsigned* __restrict__ list, unsigned n, const uint4* __restrict__ slots,
                         unsigned* out, int one_xcd, unsigned want_xcc) {
    unsigned team = gridDim.x, rank = blockIdx.x;
    if (one_xcd) {
        if (xcc_id() != want_xcc) return;
        team = gridDim.x / 8;
        rank = blockIdx.x / 8;   // round-robin placement: blocks b, b+8, ... share an XCD
    }
    unsigned acc = 0;
    for (unsigned i = rank * blockDim.x + threadIdx.x; i < n; i += team * blockDim.x) {
        const unsigned w = list[i];
        const uint4* p = slots + (size_t)w * 4;
        if (SC1) {
            const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
            unsigned long long x = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) x ^= __hip_atomic_load(q + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc ^= (unsigned)x ^ (unsigned)(x >> 32);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = p[k];
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_xcc(unsigned* o) {
    if (threadIdx.x == 0) o[blockIdx.x] = xcc_id();
}

int main() {
    const size_t nwords = 8u << 20;   // 8 M words x 64 B = 512 MB
    uint4* slots;
    unsigned *list, *out;
    CK(hipMalloc(&slots, nwords * 64));
    CK(hipMemset(slots, 1, nwords * 64));
    const unsigned maxn = 1u << 20;
    CK(hipMalloc(&list, maxn * 4));
    CK(hipMalloc(&out, 4096));
    std::vector<unsigned> h(maxn);
    unsigned long long z = 88172645463325252ull;
    for (auto& v : h) { z ^= z << 13; z ^= z >> 7; z ^= z << 17; v = (unsigned)(z % nwords); }
    CK(hipMemcpy(list, h.data(), maxn * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_xcc, dim3(8), dim3(64), 0, 0, out);
    unsigned xcc[8];
    CK(hipMemcpy(xcc, out, 32, hipMemcpyDeviceToHost));
    printf("xcc of blocks 0..7:");
    for (unsigned x : xcc) printf(" %u", x);
    printf("\n");
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 200;
    struct Cfg { const char* name; int one; unsigned grid, threads; };
    const Cfg cfgs[] = {
        {"chip 1024x256", 0, 1024, 256},
        {"xcd  32x1024 ", 1, 256, 1024},
        {"xcd  64x512  ", 1, 512, 512},
        {"xcd  128x256 ", 1, 1024, 256},
    };
    for (unsigned n : {1024u, 16384u, 65536u, 262144u, 1048576u}) {
        for (const Cfg& c : cfgs) {
            for (int sc1 = 0; sc1 < 2; ++sc1) {
                float best = 1e9f;
                for (int warm = 0; warm < 2; ++warm) {
                    CK(hipEventRecord(e0, 0));
                    for (int r = 0; r < reps; ++r) {
                        // a different slice of the list each rep (cold lines)
                        const unsigned off = (unsigned)((r * 7919u * 64u) % (maxn - n + 1));
                        if (sc1)
                            hipLaunchKernelGGL(k_gather<true>, dim3(c.grid), dim3(c.threads), 0, 0, list + off, n,
                                               slots, out, c.one, xcc[0]);
                        else
                            hipLaunchKernelGGL(k_gather<false>, dim3(c.grid), dim3(c.threads), 0, 0, list + off, n,
                                               slots, out, c.one, xcc[0]);
                    }
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    best = ms;
                }
                const double us = best * 1e3 / reps;
                printf("n=%8u %s %s %8.2f us/launch  %7.1f GB/s (list + 64 B slots)\n", n, c.name,
                       sc1 ? "sc1  " : "plain", us, n * 68.0 / us / 1e3);
            }
        }
    }
    return 0;
}
