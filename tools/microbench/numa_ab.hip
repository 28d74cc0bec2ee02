// Host->HBM DMA rate by the NUMA node of the pinned source buffer and of the copying threads.
//   P(node)   DMA only, T threads x 2 pinned 16 MiB buffers bound to `node` (set_mempolicy +
//             hipHostMallocNumaUser), threads pinned to that node's allowed CPUs
//   A(node)   pread of a page-cache-warm file into those buffers + DMA (drive.hip's pattern)
// usage: numa_ab FILE_TO_WRITE GB
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); std::exit(1); } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
constexpr size_t kChunk = 16u << 20;

static std::string slurp(const std::string& p) { std::ifstream f(p); std::string s; std::getline(f, s); return s; }
static std::vector<int> parse_list(const std::string& s) {   // "0-3,8-11"
    std::vector<int> v; size_t i = 0;
    while (i < s.size()) { size_t j = s.find(',', i); if (j == std::string::npos) j = s.size(); std::string t = s.substr(i, j - i); size_t d = t.find('-');
        if (!t.empty()) { int a = std::atoi(t.c_str()), b = d == std::string::npos ? a : std::atoi(t.c_str() + d + 1); for (int x = a; x <= b; ++x) v.push_back(x); } i = j + 1; }
    return v;
}

static double run(int fd, size_t n, uint8_t* d, int T, int node, const std::vector<int>& cpus, bool rd, int D = 0, size_t kChunk = 16u << 20) {
    std::vector<hipStream_t> shared(D);
    for (auto& s : shared) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::atomic<size_t> next{0};
    const size_t chunks = (n + kChunk - 1) / kChunk;
    std::vector<std::thread> th;
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    double t0 = 0;
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] {
        if (!cpus.empty()) { cpu_set_t cs; CPU_ZERO(&cs); CPU_SET(cpus[t % cpus.size()], &cs); sched_setaffinity(0, sizeof(cs), &cs); }
        unsigned long mask = node >= 0 ? 1ul << node : 0;
        if (node >= 0 && syscall(SYS_set_mempolicy, 2 /*MPOL_BIND*/, &mask, 64) != 0) perror("set_mempolicy");
        hipStream_t s; if (D) s = shared[t % D]; else CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        void* buf[2]; hipEvent_t ev[2]; bool busy[2] = {false, false};
        for (int k = 0; k < 2; ++k) { CK(hipHostMalloc(&buf[k], kChunk, hipHostMallocPortable | (node >= 0 ? hipHostMallocNumaUser : 0))); std::memset(buf[k], 1, kChunk); CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming)); }
        ready.fetch_add(1);
        while (!go.load()) {}
        for (int k = 0;; k ^= 1) {
            const size_t i = next.fetch_add(1);
            if (i >= chunks) break;
            if (busy[k]) CK(hipEventSynchronize(ev[k]));
            const size_t lo = i * kChunk, m = std::min(kChunk, n - lo);
            if (rd) { size_t got = 0; while (got < m) { ssize_t r = pread(fd, (uint8_t*)buf[k] + got, m - got, lo + got); if (r <= 0) { perror("pread"); std::exit(1); } got += r; } }
            CK(hipMemcpyAsync(d + lo, buf[k], m, hipMemcpyHostToDevice, s)); CK(hipEventRecord(ev[k], s)); busy[k] = true;
        }
        for (int k = 0; k < 2; ++k) if (busy[k]) CK(hipEventSynchronize(ev[k]));
        for (int k = 0; k < 2; ++k) { CK(hipHostFree(buf[k])); CK(hipEventDestroy(ev[k])); }
        if (!D) CK(hipStreamDestroy(s));
    });
    while (ready.load() < T) {}
    t0 = now();
    go.store(true);
    for (auto& x : th) x.join();
    const double el = now() - t0;
    for (auto& s : shared) CK(hipStreamDestroy(s));
    return el;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const char* path = argv[1];
    const size_t n = (size_t)(std::atof(argv[2]) * 1e9);
    {   // write the file from this (unpinned) thread set
        int fd = open(path, O_CREAT | O_TRUNC | O_RDWR, 0644);
        if (ftruncate(fd, n) != 0) { perror("ftruncate"); return 1; }
        std::vector<std::thread> th; std::atomic<size_t> next{0}; const size_t chunks = (n + kChunk - 1) / kChunk;
        for (int t = 0; t < 16; ++t) th.emplace_back([&, t] { std::vector<uint8_t> b(kChunk, (uint8_t)('a' + t));
            for (;;) { size_t i = next.fetch_add(1); if (i >= chunks) break; size_t lo = i * kChunk, m = std::min(kChunk, n - lo); if (pwrite(fd, b.data(), m, lo) != (ssize_t)m) { perror("pwrite"); std::exit(1); } } });
        for (auto& x : th) x.join();
        close(fd);
    }
    char bus[64]; CK(hipDeviceGetPCIBusId(bus, sizeof(bus), 0));
    std::string bs(bus); for (auto& c : bs) c = std::tolower(c);
    const int gnode = std::atoi(slurp("/sys/bus/pci/devices/" + bs + "/numa_node").c_str());
    cpu_set_t cs; sched_getaffinity(0, sizeof(cs), &cs);
    std::string allowed; int nall = 0;
    for (int c = 0; c < CPU_SETSIZE; ++c) if (CPU_ISSET(c, &cs)) { ++nall; if (nall <= 64) allowed += std::to_string(c) + " "; }
    std::printf("gpu %s numa_node %d; allowed cpus (%d): %s\n", bus, gnode, nall, allowed.c_str());
    int nodes = 0;
    std::vector<std::vector<int>> node_cpus;
    for (int nd = 0; nd < 8; ++nd) {
        std::string l = slurp("/sys/devices/system/node/node" + std::to_string(nd) + "/cpulist");
        if (l.empty()) break;
        std::vector<int> v; for (int c : parse_list(l)) if (CPU_ISSET(c, &cs)) v.push_back(c);
        node_cpus.push_back(v); ++nodes;
        std::printf("node %d: %zu allowed cpus (list %s)\n", nd, v.size(), l.c_str());
    }
    int fd = open(path, O_RDONLY);
    uint8_t* d; CK(hipMalloc(&d, n)); CK(hipMemset(d, 0, n)); CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 2; ++rep) {
        for (int R : {8, 12, 16, 24, 32})
            for (int D : {2, 4}) {
                double t = run(fd, n, d, R, -1, {}, true, D);
                std::printf("A  %2d readers   D=%2d streams  16M: %.1f ms = %.1f GB/s\n", R, D, t * 1e3, n / t / 1e9);
            }
        for (int R : {16, 24})
            for (size_t C : {(size_t)4 << 20, (size_t)8 << 20}) {
                double t = run(fd, n, d, R, -1, {}, true, 2, C);
                std::printf("A  %2d readers   D= 2 streams %3zuM: %.1f ms = %.1f GB/s\n", R, C >> 20, t * 1e3, n / t / 1e9);
            }
        double t = run(fd, n, d, 16, -1, {}, true);
        std::printf("A  16 readers   own streams   16M: %.1f ms = %.1f GB/s\n", t * 1e3, n / t / 1e9);
        std::fflush(stdout);
    }
    CK(hipFree(d));
    return 0;
}
