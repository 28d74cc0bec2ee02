// Micro-benchmark: the fixed cost of the merge loop's launch pattern on MI355X.
// Times N rounds of two dependent launches (grids like k_merge and k_apply_argmax) that do
// (a) nothing, (b) a chain of D dependent global loads in one wave per block.
//   hipcc -O3 --offload-arch=gfx950 launch_floor.hip -o launch_floor && ./launch_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

// a chain of `depth` dependent loads through a permutation table (L2-resident, 1 MB)
__global__ void k_chain(const unsigned* __restrict__ perm, unsigned start, int depth, unsigned* out) {
    if (threadIdx.x >= 64) return;
    unsigned x = start + threadIdx.x + blockIdx.x * 64;
    for (int i = 0; i < depth; ++i) x = perm[x & 0x3ffff];
    if (x == 0xffffffffu) out[0] = x;
}

int main() {
    const int rounds = 5000;
    unsigned* perm;
    unsigned* out;
    CK(hipMalloc(&perm, (1 << 18) * 4));
    CK(hipMalloc(&out, 64));
    std::vector<unsigned> h(1 << 18);
    for (unsigned i = 0; i < h.size(); ++i) h[i] = (i * 2654435761u) & 0x3ffff;
    CK(hipMemcpy(perm, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Cfg { const char* name; int g1, g2, depth; };
    const Cfg cfgs[] = {
        {"empty 1+1 blocks", 1, 1, -1},
        {"empty 1024+600 blocks", 1024, 600, -1},
        {"chain d=1, 1024+600", 1024, 600, 1},
        {"chain d=2, 1024+600", 1024, 600, 2},
        {"chain d=4, 1024+600", 1024, 600, 4},
        {"chain d=8, 1024+600", 1024, 600, 8},
        {"chain d=8, 64+64", 64, 64, 8},
    };
    for (const Cfg& c : cfgs) {
        for (int warm = 0; warm < 2; ++warm) {
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < rounds; ++r) {
                if (c.depth < 0) {
                    hipLaunchKernelGGL(k_empty, dim3(c.g1), dim3(256), 0, s, (int*)out);
                    hipLaunchKernelGGL(k_empty, dim3(c.g2), dim3(256), 0, s, (int*)out);
                } else {
                    hipLaunchKernelGGL(k_chain, dim3(c.g1), dim3(256), 0, s, perm, (unsigned)r, c.depth, out);
                    hipLaunchKernelGGL(k_chain, dim3(c.g2), dim3(256), 0, s, perm, (unsigned)r * 7, c.depth, out);
                }
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (warm) printf("%-28s %8.2f us per round (2 launches)\n", c.name, ms * 1e3 / rounds);
        }
    }
    return 0;
}
