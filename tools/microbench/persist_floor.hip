// Micro-benchmark: what one merge round's synchronisation costs inside ONE persistent launch
// whose workgroups all sit on one XCD (shared L2), against two dependent launches per round.
//   hipcc -O3 --offload-arch=gfx950 persist_floor.hip -o persist_floor && ./persist_floor
// Participants: every workgroup reads HW_REG_XCC_ID; those on the XCD of the first arrival take
// tickets, the first P of them work, everyone else exits.  The participant count is fixed only
// after every workgroup of the grid has checked in, so a placement that puts fewer than P
// workgroups on that XCD shrinks the team instead of hanging it.  Shared data: plain stores
// drained by s_waitcnt vmcnt(0) before the arrival, loads with sc1 (L2, bypassing the CU's L1).
// Every spin is bounded and reports a timeout.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}
__device__ __forceinline__ unsigned ld_sc1(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Team {
    unsigned checkin, xcc, tickets, nteam, bar, timeout, pad[2];
};

constexpr unsigned kSpinLimit = 1u << 22;

// returns the team size once every workgroup has checked in (0 on timeout)
__device__ unsigned team_size(Team* t, unsigned grid, unsigned P) {
    __shared__ unsigned s_n;
    if (threadIdx.x == 0) {
        unsigned spins = 0, n;
        while ((n = ld_sc1(&t->checkin)) < grid) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > kSpinLimit) { atomicOr(&t->timeout, 1u); n = 0; break; }
        }
        s_n = n >= grid ? min(ld_sc1(&t->tickets), P) : 0;
    }
    __syncthreads();
    return s_n;
}

__device__ bool team_barrier(Team* t, unsigned target) {
    __shared__ int s_ok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(&t->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        int ok = 1;
        while (ld_sc1(&t->bar) < target) {
            __builtin_amdgcn_s_sleep(0);
            if (++spins > kSpinLimit) { atomicOr(&t->timeout, 2u); ok = 0; break; }
        }
        s_ok = ok;
    }
    __syncthreads();
    return s_ok;
}

__global__ void k_persist(Team* t, unsigned P, const unsigned* __restrict__ perm, int depth, int rounds,
                          unsigned* out, unsigned* cells) {
    __shared__ unsigned s_role;
    const unsigned grid = gridDim.x;
    if (threadIdx.x == 0) {
        const unsigned x = xcc_id();
        unsigned want = atomicCAS(&t->xcc, 0xffffffffu, x);
        if (want == 0xffffffffu) want = x;
        unsigned role = 0xffffffffu;
        if (x == want) {
            const unsigned k = atomicAdd(&t->tickets, 1u);
            if (k < P) role = k;
        }
        s_role = role;
        __hip_atomic_fetch_add(&t->checkin, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const unsigned role = s_role;
    if (role == 0xffffffffu) return;
    const unsigned n = team_size(t, grid, P);
    if (n == 0) return;
    if (role == 0 && threadIdx.x == 0) out[1] = n;
    unsigned phase = 0;
    for (int r = 0; r < rounds; ++r) {
        // phase A: a dependent chain (the gather), then an atomic delta
        if (threadIdx.x < 64 && depth > 0) {
            unsigned x = r * 131 + threadIdx.x + role * 64;
            for (int i = 0; i < depth; ++i) x = ld_sc1(perm + (x & 0x3ffff));
            atomicAdd(&cells[x & 1023], 1u);
        }
        if (!team_barrier(t, n * ++phase)) return;
        // phase B: read a cell (sc1) then a dependent chain (the probe), then the argmax partial
        if (threadIdx.x < 64 && depth > 0) {
            unsigned x = ld_sc1(cells + ((r + threadIdx.x) & 1023));
            for (int i = 0; i < depth; ++i) x = ld_sc1(perm + (x & 0x3ffff));
            if (x == 0xffffffffu) out[0] = x;
        }
        if (!team_barrier(t, n * ++phase)) return;
    }
}

__global__ void k_chain(const unsigned* __restrict__ perm, unsigned start, int depth, unsigned* out) {
    if (threadIdx.x >= 64) return;
    unsigned x = start + threadIdx.x + blockIdx.x * 64;
    for (int i = 0; i < depth; ++i) x = perm[x & 0x3ffff];
    if (x == 0xffffffffu) out[0] = x;
}

// one wave, dependent sc1 loads: L2-hit latency
__global__ void k_lat(const unsigned* __restrict__ perm, int depth, unsigned* out, long long* cyc) {
    unsigned x = threadIdx.x;
    const long long t0 = clock64();
    for (int i = 0; i < depth; ++i) x = ld_sc1(perm + (x & 0x3ffff));
    const long long t1 = clock64();
    if (x == 0xffffffffu) out[0] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    const int rounds = 4000;
    unsigned *perm, *out, *cells;
    Team* team;
    long long* cyc;
    CK(hipMalloc(&perm, (1 << 18) * 4));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&cells, 4096));
    CK(hipMalloc(&team, sizeof(Team)));
    CK(hipMalloc(&cyc, 8));
    std::vector<unsigned> h(1 << 18);
    for (unsigned i = 0; i < h.size(); ++i) h[i] = (i * 2654435761u) & 0x3ffff;
    CK(hipMemcpy(perm, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(cells, 0, 4096));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    for (int warm = 0; warm < 2; ++warm) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, s, perm, 1000, out, cyc);
        CK(hipStreamSynchronize(s));
        long long c;
        CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
        if (warm) printf("sc1 dependent load (L2-resident 1 MB table): %.0f cycles each\n", c / 1000.0);
    }
    for (int depth : {0, 1, 2, 4}) {
        for (int warm = 0; warm < 2; ++warm) {
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < rounds; ++r) {
                hipLaunchKernelGGL(k_chain, dim3(1024), dim3(256), 0, s, perm, (unsigned)r, depth, out);
                hipLaunchKernelGGL(k_chain, dim3(600), dim3(256), 0, s, perm, (unsigned)r * 7, depth, out);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (warm) printf("2 launches/round, chain d=%d        %8.2f us per round\n", depth, ms * 1e3 / rounds);
        }
    }
    for (unsigned P : {8u, 16u, 32u, 64u}) {
        for (int depth : {0, 1, 2, 4}) {
            for (int warm = 0; warm < 2; ++warm) {
                CK(hipMemsetAsync(team, 0, sizeof(Team), s));
                CK(hipMemsetAsync(&team->xcc, 0xff, 4, s));
                CK(hipMemsetAsync(out, 0, 64, s));
                CK(hipEventRecord(e0, s));
                const unsigned grid = 8 * P;
                hipLaunchKernelGGL(k_persist, dim3(grid), dim3(256), 0, s, team, P, perm, depth, rounds, out, cells);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                Team th;
                unsigned ho[2];
                CK(hipMemcpy(&th, team, sizeof(th), hipMemcpyDeviceToHost));
                CK(hipMemcpy(ho, out, 8, hipMemcpyDeviceToHost));
                if (warm)
                    printf("persistent P=%2u (team %2u, tickets %u) d=%d %8.2f us per round (2 barriers)%s\n", P,
                           ho[1], th.tickets, depth, ms * 1e3 / rounds, th.timeout ? "  TIMEOUT" : "");
            }
        }
    }
    return 0;
}
