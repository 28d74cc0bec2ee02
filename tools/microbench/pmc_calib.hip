// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the BPE kernels
// use (MI355X_MICROARCH.md, HBM section: only 16-B streaming reads and stores are calibrated there).
// Each kernel touches a known number of bytes / distinct 128-B lines of buffers far larger than the
// 256 MiB Infinity Cache, once; tools/gpu_pmc_calib.sh runs this under two --pmc passes and
// tools/pmc_calib.py divides the counters by the known bytes.
//   hipcc -O3 --offload-arch=gfx950 pmc_calib.hip -o pmc_calib && ./pmc_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr size_t kBig = 4ull << 30;   // 4 GiB buffers: 16x the Infinity Cache

// 16 B per lane, streaming (the guide's calibrated case)
__global__ void c_read16(const uint4* __restrict__ p, size_t n, unsigned* out) {
    uint4 acc{0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = 1;
}
// 4 B per lane, streaming (posting lists, records)
__global__ void c_read4(const unsigned* __restrict__ p, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x9e3779b9u) out[0] = 1;
}
// one W-byte load per lane at a distinct random 128-B line (word tables, hash slots)
template <class T>
__global__ void c_gather(const T* __restrict__ p, size_t lines, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t line = (i * 0x9E3779B1ull) & (lines - 1);   // a bijection of [0, lines): distinct lines
        acc ^= (unsigned)p[line * (128 / sizeof(T))];
    }
    if (acc == 0x9e3779b9u) out[0] = 1;
}
// 16 lanes read one 64-B segment of a random line (a short word's tokens)
__global__ void c_gather64(const unsigned* __restrict__ p, size_t lines, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t g = i >> 4;
        const size_t line = (g * 0x9E3779B1ull) & (lines - 1);
        acc ^= p[line * 32 + (i & 15)];
    }
    if (acc == 0x9e3779b9u) out[0] = 1;
}
__global__ void c_write16(uint4* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = uint4{(unsigned)i, 1, 2, 3};
}
__global__ void c_write4(unsigned* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (unsigned)i;
}
__global__ void c_write2(uint16_t* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint16_t)i;
}
// one 4-B store per lane at a distinct random line
__global__ void c_scatter4(unsigned* __restrict__ p, size_t lines, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t line = (i * 0x9E3779B1ull) & (lines - 1);
        p[line * 32] = (unsigned)i;
    }
}
// one 4-B atomic add per lane at a distinct random line
__global__ void c_atomic4(unsigned* __restrict__ p, size_t lines, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t line = (i * 0x9E3779B1ull) & (lines - 1);
        atomicAdd(&p[line * 32], 1u);
    }
}

int main() {
    uint8_t *a, *b;
    unsigned* out;
    CK(hipMalloc(&a, kBig));
    CK(hipMalloc(&b, kBig));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 1, kBig));
    CK(hipMemset(b, 2, kBig));
    CK(hipDeviceSynchronize());
    const dim3 g(4096), t(256);
    const size_t lines = kBig / 128;
    const size_t ng = 16u << 20;   // 16 M random accesses: 2 GiB of distinct lines at most
    // the known byte counts, for tools/pmc_calib.py
    printf("c_read16 %zu\n", kBig);
    hipLaunchKernelGGL(c_read16, g, t, 0, 0, (const uint4*)a, kBig / 16, out);
    printf("c_read4 %zu\n", kBig);
    hipLaunchKernelGGL(c_read4, g, t, 0, 0, (const unsigned*)a, kBig / 4, out);
    printf("c_gather<unsigned short> lines %zu\n", ng);
    hipLaunchKernelGGL(c_gather<uint16_t>, g, t, 0, 0, (const uint16_t*)b, lines, ng, out);
    printf("c_gather<unsigned int> lines %zu\n", ng);
    hipLaunchKernelGGL(c_gather<unsigned>, g, t, 0, 0, (const unsigned*)a, lines, ng, out);
    printf("c_gather<unsigned long> lines %zu\n", ng);
    hipLaunchKernelGGL(c_gather<unsigned long>, g, t, 0, 0, (const unsigned long*)b, lines, ng, out);
    printf("c_gather64 lines %zu\n", ng / 16);
    hipLaunchKernelGGL(c_gather64, g, t, 0, 0, (const unsigned*)a, lines, ng, out);
    printf("c_write16 %zu\n", kBig);
    hipLaunchKernelGGL(c_write16, g, t, 0, 0, (uint4*)b, kBig / 16);
    printf("c_write4 %zu\n", kBig);
    hipLaunchKernelGGL(c_write4, g, t, 0, 0, (unsigned*)a, kBig / 4);
    printf("c_write2 %zu\n", kBig);
    hipLaunchKernelGGL(c_write2, g, t, 0, 0, (uint16_t*)b, kBig / 2);
    printf("c_scatter4 lines %zu\n", ng);
    hipLaunchKernelGGL(c_scatter4, g, t, 0, 0, (unsigned*)a, lines, ng);
    printf("c_atomic4 lines %zu\n", ng);
    hipLaunchKernelGGL(c_atomic4, g, t, 0, 0, (unsigned*)b, lines, ng);
    CK(hipDeviceSynchronize());
    CK(hipGetLastError());
    printf("done\n");
    return 0;
}
