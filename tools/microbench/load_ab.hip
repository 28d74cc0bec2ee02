// File -> HBM load strategies, measured on a page-cache-warm file (the bench's load phase).
//   A  pread by T threads into 2 pinned 16 MiB buffers each, DMA per buffer (drive.hip today)
//   R  pread alone into the pinned buffers (no DMA): the host-copy bound
//   P  DMA alone from one pinned buffer reused (no read): the PCIe bound
//   M  mmap the file, hipHostRegister (read-only) slices by T threads, DMA straight from the
//      page cache pages, unregister
// usage: load_ab FILE [GB_TO_WRITE]   (writes FILE first when a size is given)
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <functional>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
constexpr size_t kChunk = 16u << 20;

static void run_threads(int T, const std::function<void(int)>& f) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(f, t);
    for (auto& x : th) x.join();
}

static double mode_A(int fd, size_t n, uint8_t* d, int T, bool dma, bool rd) {
    std::atomic<size_t> next{0};
    const size_t chunks = (n + kChunk - 1) / kChunk;
    const double t0 = now();
    run_threads(T, [&](int) {
        hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        void* buf[2]; hipEvent_t ev[2]; bool busy[2] = {false, false};
        for (int k = 0; k < 2; ++k) { CK(hipHostMalloc(&buf[k], kChunk, hipHostMallocPortable)); CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming)); }
        for (int k = 0;; k ^= 1) {
            const size_t i = next.fetch_add(1);
            if (i >= chunks) break;
            if (busy[k]) CK(hipEventSynchronize(ev[k]));
            const size_t lo = i * kChunk, m = std::min(kChunk, n - lo);
            if (rd) { size_t got = 0; while (got < m) { ssize_t r = pread(fd, (uint8_t*)buf[k] + got, m - got, lo + got); if (r <= 0) { perror("pread"); std::exit(1); } got += r; } }
            if (dma) { CK(hipMemcpyAsync(d + lo, buf[k], m, hipMemcpyHostToDevice, s)); CK(hipEventRecord(ev[k], s)); busy[k] = true; }
        }
        CK(hipStreamSynchronize(s));
        for (int k = 0; k < 2; ++k) { CK(hipHostFree(buf[k])); CK(hipEventDestroy(ev[k])); }
        CK(hipStreamDestroy(s));
    });
    return now() - t0;
}

static void mode_M(int fd, size_t n, uint8_t* d, int T, size_t slice, unsigned flags, bool populate) {
    const double t0 = now();
    void* p = mmap(nullptr, n, PROT_READ, MAP_SHARED | (populate ? MAP_POPULATE : 0), fd, 0);
    if (p == MAP_FAILED) { perror("mmap"); return; }
    const double t1 = now();
    const size_t ns = (n + slice - 1) / slice;
    std::atomic<size_t> next{0};
    std::atomic<int> fail{0};
    std::vector<double> reg_s(T, 0), cp_s(T, 0), unreg_s(T, 0);
    run_threads(T, [&](int t) {
        hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        for (;;) {
            const size_t i = next.fetch_add(1);
            if (i >= ns) break;
            const size_t lo = i * slice, m = std::min(slice, n - lo);
            uint8_t* h = (uint8_t*)p + lo;
            double a = now();
            hipError_t e = hipHostRegister(h, m, flags);
            if (e != hipSuccess) { if (!fail.exchange(1)) std::fprintf(stderr, "hipHostRegister(flags %u): %s\n", flags, hipGetErrorString(e)); continue; }
            double b = now();
            CK(hipMemcpyAsync(d + lo, h, m, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            double c = now();
            CK(hipHostUnregister(h));
            double dd = now();
            reg_s[t] += b - a; cp_s[t] += c - b; unreg_s[t] += dd - c;
        }
        CK(hipStreamDestroy(s));
    });
    const double t2 = now();
    munmap(p, n);
    const double t3 = now();
    double r = 0, c = 0, u = 0;
    for (int t = 0; t < T; ++t) { r += reg_s[t]; c += cp_s[t]; u += unreg_s[t]; }
    std::printf("M  T=%2d slice=%4zu MiB flags=%u populate=%d: %s total %.1f ms = %.1f GB/s (mmap %.1f, work %.1f, munmap %.1f; per-thread sums reg %.0f cp %.0f unreg %.0f ms)\n",
                T, slice >> 20, flags, populate, fail ? "FAILED" : "ok", (t3 - t0) * 1e3, n / (t3 - t0) / 1e9,
                (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, r * 1e3, c * 1e3, u * 1e3);
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: load_ab FILE [GB]\n"); return 2; }
    const char* path = argv[1];
    if (argc > 2) {   // write the file (arbitrary printable bytes), multi-threaded
        const size_t n = (size_t)(std::atof(argv[2]) * 1e9);
        int fd = open(path, O_CREAT | O_TRUNC | O_RDWR, 0644);
        if (fd < 0) { perror("open"); return 1; }
        if (ftruncate(fd, n) != 0) { perror("ftruncate"); return 1; }
        const double t0 = now();
        std::atomic<size_t> next{0};
        const size_t chunks = (n + kChunk - 1) / kChunk;
        run_threads(16, [&](int t) {
            std::vector<uint8_t> b(kChunk);
            for (size_t j = 0; j < kChunk; ++j) b[j] = (uint8_t)('a' + (j * 7 + t) % 26);
            for (;;) { size_t i = next.fetch_add(1); if (i >= chunks) break; size_t lo = i * kChunk, m = std::min(kChunk, n - lo); if (pwrite(fd, b.data(), m, lo) != (ssize_t)m) { perror("pwrite"); std::exit(1); } }
        });
        close(fd);
        std::printf("wrote %.2f GB in %.1f s\n", n / 1e9, now() - t0);
    }
    int fd = open(path, O_RDONLY);
    struct stat st; fstat(fd, &st);
    const size_t n = st.st_size;
    uint8_t* d; CK(hipMalloc(&d, n));
    CK(hipMemset(d, 0, n)); CK(hipDeviceSynchronize());
    std::printf("file %.2f GB\n", n / 1e9);
    for (int rep = 0; rep < 2; ++rep) {
        for (int T : {16, 32}) {
            double t = mode_A(fd, n, d, T, true, true);
            std::printf("A  T=%2d pread+DMA: %.1f ms = %.1f GB/s\n", T, t * 1e3, n / t / 1e9);
        }
        double t = mode_A(fd, n, d, 16, false, true);
        std::printf("R  T=16 pread only: %.1f ms = %.1f GB/s\n", t * 1e3, n / t / 1e9);
        t = mode_A(fd, n, d, 16, true, false);
        std::printf("P  T=16 DMA only (pinned, no read): %.1f ms = %.1f GB/s\n", t * 1e3, n / t / 1e9);
        mode_M(fd, n, d, 16, 256u << 20, hipHostRegisterReadOnly, false);
        mode_M(fd, n, d, 16, 64u << 20, hipHostRegisterReadOnly, false);
        mode_M(fd, n, d, 16, 256u << 20, hipHostRegisterDefault, false);
        mode_M(fd, n, d, 16, 256u << 20, hipHostRegisterReadOnly, true);
        std::fflush(stdout);
    }
    // the M path's bytes must equal the file
    std::vector<uint8_t> a(1 << 20), b(1 << 20);
    for (size_t off : {(size_t)0, n / 3, n - (1u << 20)}) {
        CK(hipMemcpy(a.data(), d + off, 1 << 20, hipMemcpyDeviceToHost));
        if (pread(fd, b.data(), 1 << 20, off) != (1 << 20)) { perror("pread"); return 1; }
        std::printf("check at %zu: %s\n", off, memcmp(a.data(), b.data(), 1 << 20) ? "DIFFER" : "same");
    }
    CK(hipFree(d));
    return 0;
}
