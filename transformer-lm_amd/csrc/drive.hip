// Host driver of train_bpe(input_path, ...): file -> HBM staging and the multi-device trainer.
//
// The reference reads the whole file in text mode and trains in one process
// (models/tokenizer/train.py:16-28, :142-231; its OWT caller perf/bpe/util.py:16 is one process).
// Here the file is read by a pool of host threads with pread into pinned staging buffers, each
// buffer copied to HBM by DMA on the reading thread's own stream while the thread reads the
// next one, so the disk/page-cache read, the copy and (for several GPUs) the slabs all overlap.
//
// Several GPUs in one process (n_gpus > 1): the file is cut into one slab per device at safe
// split points (a U+0020 between two ASCII non-space bytes: the pre-token multiset is unchanged,
// SURVEY.md §8e), each device validates, pre-tokenizes and counts its slab, one RCCL all-gather
// (ncclCommInitRank per device thread, one shared id) exchanges the unique-word tables, and
// device 0 runs the merge loop on their union (exchange.hip).  Errors found while reading or
// validating a slab are agreed on by all ranks before any collective, so no rank waits on a
// collective that another rank never reaches.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "drive.h"

namespace bpe {

namespace {

constexpr size_t kStageChunk = 16u << 20;   // bytes per pread / DMA

// Process-wide pinned staging buffers, allocated on first use and kept: pinning host pages costs
// far more than a read of the same size, so a training call must not pay it again.
struct PinnedPool {
    std::mutex m;
    std::vector<void*> free_;
    void* get() {
        {
            std::lock_guard<std::mutex> g(m);
            if (!free_.empty()) {
                void* p = free_.back();
                free_.pop_back();
                return p;
            }
        }
        void* p = nullptr;
        BPE_HIP(hipHostMalloc(&p, kStageChunk, hipHostMallocPortable));
        return p;
    }
    void put(void* p) {
        std::lock_guard<std::mutex> g(m);
        free_.push_back(p);
    }
};
PinnedPool& pool() {
    static PinnedPool* p = new PinnedPool;   // never freed: lives as long as the process
    return *p;
}

// Device-to-host staging written by a kernel (device_to_host): coherent, device-mapped pinned
// buffers, each with its device address.  HIP serves a device-to-host hipMemcpyAsync with a copy
// KERNEL (__amd_rocclr_copyBuffer, 1399 launches of ~470 us in profiles/r04/n_*), whose
// workgroups take CUs from the encode running beside it in encode_file (1 GiB region encodes went
// from 21.6 to 43 ms while a region's ids were copied out, r04s).  A copy kernel of our own with
// a small grid moves the same bytes over the bus from a few CUs.
struct MappedBuf {
    void* host = nullptr;
    void* dev = nullptr;
};
struct MappedPool {
    std::mutex m;
    std::vector<MappedBuf> free_;
    MappedBuf get() {
        {
            std::lock_guard<std::mutex> g(m);
            if (!free_.empty()) {
                const MappedBuf b = free_.back();
                free_.pop_back();
                return b;
            }
        }
        MappedBuf b;
        BPE_HIP(hipHostMalloc(&b.host, kStageChunk, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
        const hipError_t e = hipHostGetDevicePointer(&b.dev, b.host, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(b.host);
            BPE_HIP(e);
        }
        return b;
    }
    void put(const MappedBuf& b) {
        std::lock_guard<std::mutex> g(m);
        free_.push_back(b);
    }
};
MappedPool& mapped_pool() {
    static MappedPool* p = new MappedPool;   // never freed: lives as long as the process
    return *p;
}

// device bytes -> a mapped host buffer: 16-byte loads and stores when both ends allow
__global__ void __launch_bounds__(256) k_to_host(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, size_t n) {
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
// workgroups per device-to-host chunk copy by k_to_host (BPE355_D2H_WG); 0, the default:
// hipMemcpyAsync.  16 workgroups moved encode_file's ids at ~18 GB/s against HIP's ~34 (r04u:
// 581-670 vs 383-421 ms per 11.9 GB call), so the knob stays for A/B only.
int d2h_wg() {   // read per call, so a test can switch it
    int n = 0;
    if (const char* e = std::getenv("BPE355_D2H_WG")) n = std::atoi(e);
    return std::max(0, std::min(n, 1024));
}

// Device buffers for the corpus, kept across training calls (per device, checked out by one
// call at a time): a fresh multi-GB allocation per call costs tens of ms (the driver clears it).
struct CorpusBuf {
    DevBuf<uint8_t> b;
    int dev = -1;
};
struct CorpusCache {
    std::mutex m;
    std::vector<std::unique_ptr<CorpusBuf>> free_;
};
CorpusCache& corpus_cache() {
    static CorpusCache* c = new CorpusCache;   // lives as long as the process
    return *c;
}
std::unique_ptr<CorpusBuf> corpus_take(size_t n) {
    int dev = 0;
    BPE_HIP(hipGetDevice(&dev));
    std::unique_ptr<CorpusBuf> x;
    {
        std::lock_guard<std::mutex> g(corpus_cache().m);
        auto& f = corpus_cache().free_;
        for (size_t i = 0; i < f.size(); ++i)
            if (f[i]->dev == dev) {   // this device's buffer: reuse it if it is large enough
                x = std::move(f[i]);
                f.erase(f.begin() + i);
                break;
            }
    }
    if (x && x->b.n >= n) return x;
    if (!x) x = std::make_unique<CorpusBuf>();
    x->b.release();
    x->b.alloc(n);
    x->dev = dev;
    return x;
}
void corpus_give(std::unique_ptr<CorpusBuf> x) {
    std::lock_guard<std::mutex> g(corpus_cache().m);
    corpus_cache().free_.push_back(std::move(x));
}

[[noreturn]] void io_error(int en, const std::string& what) {
    throw Error{BPE_E_IO, what + ": " + std::strerror(en), en};
}

}  // namespace

size_t corpus_release(int dev) {
    std::vector<std::unique_ptr<CorpusBuf>> drop;
    size_t bytes = 0;
    {
        std::lock_guard<std::mutex> g(corpus_cache().m);
        auto& f = corpus_cache().free_;
        for (size_t i = 0; i < f.size();)
            if (dev < 0 || f[i]->dev == dev) {
                bytes += f[i]->b.bytes();
                drop.push_back(std::move(f[i]));
                f.erase(f.begin() + i);
            } else {
                ++i;
            }
    }
    if (drop.empty()) return bytes;
    int cur = 0;
    BPE_HIP(hipGetDevice(&cur));
    for (auto& x : drop) {   // hipFree outside the lock, on the buffer's own device
        (void)hipSetDevice(x->dev);
        x->b.release();
    }
    BPE_HIP(hipSetDevice(cur));
    return bytes;
}

// Reader threads and DMA streams of one transfer.  Measured on MI355X boxes with a page-cache-warm
// 11.9 GB file (tools/microbench/numa_ab.hip, profiles/r03/e_load_ab.txt): DMA alone runs at
// 50-52 GB/s on 1-2 streams but 37 GB/s on 16; pread alone at 45 GB/s on 16 threads; together,
// 16 readers each with its own stream 34-38 GB/s, 8 readers feeding 2 shared streams 46-47 GB/s.
// More than 16 readers is slower (24: 30 GB/s, 32: 24 GB/s), as is the NUMA binding of the
// staging buffers (no difference).
int io_threads() {
    static const int t = [] {
        int n = 8;
        if (const char* e = std::getenv("BPE355_IO_THREADS")) n = std::atoi(e);
        return std::max(1, std::min(n, 16));   // a GPU's share of the host is 16 cores
    }();
    return t;
}

static int dma_streams() {
    static const int t = [] {
        int n = 2;
        if (const char* e = std::getenv("BPE355_DMA_STREAMS")) n = std::atoi(e);
        return std::max(1, std::min(n, 16));
    }();
    return t;
}

namespace {
// the DMA streams the reader threads of one transfer share (thread t copies on stream t % n): a
// few deep queues keep the copy engines busier than one queue per thread
struct DmaStreams {
    std::vector<hipStream_t> s;
    // on `device` (the calling thread's current device is kept); low_priority: the least stream
    // priority the device offers
    DmaStreams(int device, int n, bool low_priority = false) {
        int cur = 0;
        BPE_HIP(hipGetDevice(&cur));
        BPE_HIP(hipSetDevice(device));
        s.resize(n, nullptr);
        int least = 0, greatest = 0;
        if (low_priority) BPE_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        hipError_t e = hipSuccess;
        for (auto& x : s)
            if (e == hipSuccess)
                e = low_priority ? hipStreamCreateWithPriority(&x, hipStreamNonBlocking, least)
                                 : hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
        BPE_HIP(hipSetDevice(cur));
        if (e != hipSuccess) {
            for (auto& x : s)
                if (x) (void)hipStreamDestroy(x);
            BPE_HIP(e);
        }
    }
    ~DmaStreams() {
        for (auto& x : s)
            if (x) {
                (void)hipStreamSynchronize(x);
                (void)hipStreamDestroy(x);
            }
    }
    hipStream_t pick(int t) const { return s[(size_t)t % s.size()]; }
};

// The copy streams of one direction on one device, created on first use and kept for the
// process (never destroyed: streams outlive the calls that use them, and a stream torn down at
// exit can outlive the runtime).  encode_file stages a slab and copies a region out per call of
// stage_to_device / device_to_host; streams made and destroyed per call cost a round trip each,
// and the two directions keep separate streams so that host-to-device and device-to-host copies
// run side by side.
// Index (device, dir, priority).  BPE355_D2H_PRIO is read per call, so its A/B switches between
// two sets of streams within one process.
struct DmaCache {
    std::mutex m;
    std::vector<DmaStreams*> made;
};
DmaCache& dma_cache() {
    static DmaCache* c = new DmaCache;   // lives as long as the process
    return *c;
}
const DmaStreams& cached_dma(int device, int dir) {
    // device-to-host copies run at the least priority: HIP serves them with a copy kernel, whose
    // workgroups should yield the CUs to the encode beside it (BPE355_D2H_PRIO=0: normal priority)
    const char* pe = std::getenv("BPE355_D2H_PRIO");
    const bool low = dir == 1 && !(pe && pe[0] == '0');
    DmaCache& c = dma_cache();
    std::lock_guard<std::mutex> g(c.m);
    const size_t i = (size_t)device * 4 + (size_t)dir * 2 + (low ? 1 : 0);
    if (c.made.size() <= i) c.made.resize(i + 1, nullptr);
    if (!c.made[i]) c.made[i] = new DmaStreams(device, dma_streams(), low);
    return *c.made[i];
}
}  // namespace

// ------------------------------------------------------------------ sources
Source Source::open_path(const char* path) {
    Source s;
    s.name = path;
    s.fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (s.fd < 0) io_error(errno, std::string("cannot open ") + path);
    struct stat st;
    if (::fstat(s.fd, &st) != 0) io_error(errno, std::string("cannot stat ") + path);
    if (S_ISDIR(st.st_mode)) io_error(EISDIR, std::string("cannot read ") + path);
    if (S_ISREG(st.st_mode) && st.st_size > 0) {
        s.size = (size_t)st.st_size;
        return s;
    }
    // a pipe, FIFO, character device or /proc file (st_size 0 or meaningless): read to EOF
    std::vector<uint8_t>& b = s.owned;
    size_t n = 0;
    for (;;) {
        if (b.size() - n < (1u << 20)) b.resize(std::max<size_t>(2 * b.size(), n + (4u << 20)));
        const ssize_t r = ::read(s.fd, b.data() + n, b.size() - n);
        if (r < 0) {
            if (errno == EINTR) continue;
            io_error(errno, std::string("cannot read ") + path);
        }
        if (r == 0) break;
        n += (size_t)r;
    }
    b.resize(n);
    s.mem = b.data();
    s.size = n;
    ::close(s.fd);
    s.fd = -1;
    return s;
}

Source Source::memory(const uint8_t* p, size_t n) {
    Source s;
    s.mem = p;
    s.size = n;
    s.name = "<buffer>";
    return s;
}

Source::~Source() {
    if (fd >= 0) ::close(fd);
}

void Source::read(size_t off, size_t len, uint8_t* dst) const {
    if (mem) {
        std::memcpy(dst, mem + off, len);
        return;
    }
    size_t got = 0;
    while (got < len) {
        const ssize_t r = ::pread(fd, dst + got, len - got, (off_t)(off + got));
        if (r < 0) {
            if (errno == EINTR) continue;
            io_error(errno, "cannot read " + name);
        }
        if (r == 0) io_error(EIO, "short read on " + name + " (file truncated while reading?)");
        got += (size_t)r;
    }
}

// ------------------------------------------------------------------ slabs
std::vector<size_t> slab_cuts(const Source& src, int g) {
    std::vector<size_t> cut(g + 1, 0);
    cut[g] = src.size;
    std::vector<uint8_t> win;
    for (int r = 1; r < g; ++r) {
        const size_t want = src.size / g * r;
        size_t c = cut[r - 1];
        // look back from the nominal point in growing windows for a safe split
        for (size_t w = 1u << 16; w <= (64u << 20); w <<= 2) {
            const size_t lo = want > w ? want - w : 0;
            const size_t hi = std::min(src.size, want + 2);
            if (hi <= lo + 2) break;
            win.resize(hi - lo);
            src.read(lo, hi - lo, win.data());
            const size_t p = bpe_safe_split(win.data(), win.size(), want - lo);
            if (p > 0 && lo + p > cut[r - 1]) { c = lo + p; break; }
            if (lo == 0) break;
        }
        cut[r] = c;   // no safe point: this slab is empty and the previous one takes the text
    }
    return cut;
}

// ------------------------------------------------------------------ file -> HBM
void stage_to_device(const Source& src, size_t off, size_t len, uint8_t* d_dst, int device, int threads) {
    if (len == 0) return;
    const size_t chunks = (len + kStageChunk - 1) / kStageChunk;
    const int t_n = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, chunks));
    std::atomic<size_t> next{0};
    std::vector<std::exception_ptr> errs(t_n);
    const DmaStreams& dma = cached_dma(device, 0);
    auto work = [&](int t) {
        const hipStream_t s = dma.pick(t);
        void* buf[2] = {nullptr, nullptr};
        hipEvent_t ev[2] = {nullptr, nullptr};
        bool busy[2] = {false, false};
        try {
            BPE_HIP(hipSetDevice(device));
            for (int k = 0; k < 2; ++k) {
                buf[k] = pool().get();
                BPE_HIP(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
            }
            for (int k = 0;; k ^= 1) {
                const size_t i = next.fetch_add(1);
                if (i >= chunks) break;
                if (busy[k]) BPE_HIP(hipEventSynchronize(ev[k]));   // its previous DMA is done
                const size_t lo = i * kStageChunk, n = std::min(kStageChunk, len - lo);
                src.read(off + lo, n, static_cast<uint8_t*>(buf[k]));
                BPE_HIP(hipMemcpyAsync(d_dst + lo, buf[k], n, hipMemcpyHostToDevice, s));
                BPE_HIP(hipEventRecord(ev[k], s));
                busy[k] = true;
            }
        } catch (...) {
            errs[t] = std::current_exception();
            next.store(chunks);   // the others stop after their current chunk
            (void)hipStreamSynchronize(s);
        }
        for (int k = 0; k < 2; ++k) {   // this thread's copies are done before its buffers go back
            if (busy[k]) (void)hipEventSynchronize(ev[k]);
            if (ev[k]) (void)hipEventDestroy(ev[k]);
            if (buf[k]) pool().put(buf[k]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < t_n; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
}

// ------------------------------------------------------------------ HBM -> host memory
// The reverse of stage_to_device: each thread DMAs a chunk into its pinned buffer, then copies it
// to the destination while its other buffer's DMA runs (a pageable destination is faulted in by
// many threads at once instead of by one copy).
void device_to_host(const uint8_t* d_src, size_t len, uint8_t* h_dst, int device, int threads) {
    if (len == 0) return;
    const size_t chunks = (len + kStageChunk - 1) / kStageChunk;
    const int t_n = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, chunks));
    std::atomic<size_t> next{0};
    std::vector<std::exception_ptr> errs(t_n);
    const DmaStreams& dma = cached_dma(device, 1);
    auto work = [&](int t) {
        const hipStream_t s = dma.pick(t);
        const int wg = d2h_wg();
        void* buf[2] = {nullptr, nullptr};
        MappedBuf mb[2];
        hipEvent_t ev[2] = {nullptr, nullptr};
        size_t pend[2] = {~(size_t)0, ~(size_t)0};   // chunk whose copy into buf[k] is in flight
        auto drain = [&](int k) {
            if (pend[k] == ~(size_t)0) return;
            BPE_HIP(hipEventSynchronize(ev[k]));
            const size_t lo = pend[k] * kStageChunk;
            std::memcpy(h_dst + lo, buf[k], std::min(kStageChunk, len - lo));
            pend[k] = ~(size_t)0;
        };
        try {
            BPE_HIP(hipSetDevice(device));
            for (int k = 0; k < 2; ++k) {
                if (wg) {
                    mb[k] = mapped_pool().get();
                    buf[k] = mb[k].host;
                } else {
                    buf[k] = pool().get();
                }
                BPE_HIP(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
            }
            for (int k = 0;; k ^= 1) {
                drain(k);
                const size_t i = next.fetch_add(1);
                if (i >= chunks) break;
                const size_t lo = i * kStageChunk, n = std::min(kStageChunk, len - lo);
                if (wg) {
                    hipLaunchKernelGGL(k_to_host, dim3(wg), dim3(256), 0, s, d_src + lo, static_cast<uint8_t*>(mb[k].dev), n);
                    BPE_HIP(hipGetLastError());
                } else {
                    BPE_HIP(hipMemcpyAsync(buf[k], d_src + lo, n, hipMemcpyDeviceToHost, s));
                }
                BPE_HIP(hipEventRecord(ev[k], s));
                pend[k] = i;
            }
            drain(0);
            drain(1);
        } catch (...) {
            errs[t] = std::current_exception();
            next.store(chunks);
            (void)hipStreamSynchronize(s);
        }
        for (int k = 0; k < 2; ++k) {   // no DMA into a buffer that goes back to the pool
            if (pend[k] != ~(size_t)0) (void)hipEventSynchronize(ev[k]);
            if (ev[k]) (void)hipEventDestroy(ev[k]);
            if (buf[k]) {
                if (wg) mapped_pool().put(mb[k]);
                else pool().put(buf[k]);
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < t_n; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
}

// ------------------------------------------------------------------ file -> HBM, counted on arrival
// The corpus is cut into segments at safe split points; a segment is validated and counted
// (into one word table) as soon as its chunks are in HBM: the stream waits on the chunks' copy
// events, so the host never blocks the device, and the count of segment k overlaps the copy of
// segment k + 1.  The same tokens and counts as one pass over the whole text (text.hip).
namespace {

struct ChunkTrack {
    std::vector<hipEvent_t> ev;
    std::vector<char> ready;
    std::mutex m;
    std::condition_variable cv;
    size_t prefix = 0;   // chunks 0 .. prefix-1 have their copy event recorded
    bool failed = false;
    explicit ChunkTrack(size_t n) : ev(n, nullptr), ready(n, 0) {
        for (auto& e : ev) BPE_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    ~ChunkTrack() {
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
    }
    void mark(size_t i) {
        std::lock_guard<std::mutex> g(m);
        ready[i] = 1;
        while (prefix < ready.size() && ready[prefix]) ++prefix;
        cv.notify_all();
    }
    void fail() {
        std::lock_guard<std::mutex> g(m);
        failed = true;
        cv.notify_all();
    }
    bool wait_prefix(size_t k) {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return prefix >= k || failed; });
        return !failed;
    }
};

size_t segment_bytes() {
    const char* e = std::getenv("BPE355_SEG_MB");   // experiment / test knob
    return (size_t)(e ? std::max(1, std::atoi(e)) : 256) << 20;   // 256/512/1024 MB: 690/720/790 ms steps
}

// safe cut points splitting src[off, off + len) into segments of ~seg bytes (relative to off)
std::vector<size_t> segment_cuts(const Source& src, size_t off, size_t len, size_t seg) {
    std::vector<size_t> cut{0};
    std::vector<uint8_t> win(1u << 16);
    for (size_t want = seg; want + seg / 2 < len; want += seg) {
        const size_t lo = want - std::min(want, win.size() - 2);
        const size_t hi = want + 2;
        src.read(off + lo, hi - lo, win.data());
        const size_t p = bpe_safe_split(win.data(), hi - lo, want - lo);
        if (p > 0 && lo + p > cut.back()) cut.push_back(lo + p);
    }
    cut.push_back(len);
    return cut;
}

}  // namespace

bool load_and_count(const Source& src, size_t off, size_t len, uint8_t* d_dst, int device, int threads,
                    hipStream_t stream, Prepared& pre) {
    const auto t0 = std::chrono::steady_clock::now();
    const std::vector<size_t> cut = segment_cuts(src, off, len, segment_bytes());
    const size_t chunks = (len + kStageChunk - 1) / kStageChunk;
    ChunkTrack track(chunks);
    const int t_n = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, chunks));
    std::atomic<size_t> next{0};
    std::vector<std::exception_ptr> errs(t_n);
    DmaStreams dma(device, dma_streams());
    auto reader = [&](int t) {
        const hipStream_t s = dma.pick(t);
        void* buf[2] = {nullptr, nullptr};
        size_t last[2] = {~(size_t)0, ~(size_t)0};
        try {
            BPE_HIP(hipSetDevice(device));
            for (int k = 0; k < 2; ++k) buf[k] = pool().get();
            for (int k = 0;; k ^= 1) {
                const size_t i = next.fetch_add(1);
                if (i >= chunks) break;
                if (last[k] != ~(size_t)0) BPE_HIP(hipEventSynchronize(track.ev[last[k]]));
                const size_t lo = i * kStageChunk, n = std::min(kStageChunk, len - lo);
                src.read(off + lo, n, static_cast<uint8_t*>(buf[k]));
                BPE_HIP(hipMemcpyAsync(d_dst + lo, buf[k], n, hipMemcpyHostToDevice, s));
                BPE_HIP(hipEventRecord(track.ev[i], s));
                last[k] = i;
                track.mark(i);
            }
        } catch (...) {
            errs[t] = std::current_exception();
            next.store(chunks);
            track.fail();
            (void)hipStreamSynchronize(s);
        }
        for (int k = 0; k < 2; ++k) {   // this thread's copies are done before its buffers go back
            if (last[k] != ~(size_t)0) (void)hipEventSynchronize(track.ev[last[k]]);
            if (buf[k]) pool().put(buf[k]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < t_n; ++t) th.emplace_back(reader, t);
    // enqueue each segment's validation and count behind its chunks' copies
    ValidatePass vp;
    CountPass cp;
    bool ok = true;
    const char* ae = std::getenv("BPE355_AGG_SEGS");   // segments between partial aggregations (0: off)
    const size_t agg_every = ae ? (size_t)std::max(0, std::atoi(ae)) : 4;
    try {
        vp.begin(d_dst, len, stream);
        cp.begin(d_dst, len, CountPass::initial_cap(len), stream, timing_enabled());
        cp.gate = vp.flags.p;   // counts only text whose validation (earlier on the stream) passed
        size_t waited = 0;
        for (size_t k = 0; k + 1 < cut.size(); ++k) {
            const size_t need = (cut[k + 1] + kStageChunk - 1) / kStageChunk;
            if (!track.wait_prefix(need)) { ok = false; break; }
            for (; waited < need; ++waited) BPE_HIP(hipStreamWaitEvent(stream, track.ev[waited], 0));
            vp.range(cut[k], cut[k + 1]);
            cp.range(cut[k], cut[k + 1]);
            // the GPU waits on PCIe here: aggregate the record pages completed so far
            if (agg_every > 0 && (k + 1) % agg_every == 0 && k + 2 < cut.size()) cp.partial();
        }
    } catch (...) {
        track.fail();
        next.store(chunks);
        for (auto& x : th) x.join();
        throw;
    }
    for (auto& x : th) x.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
    BPE_REQUIRE(ok, BPE_E_IO, "corpus load failed");
    const double load_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    unsigned long long bad = 0;
    bool cr = false;
    vp.finish(&bad, &cr);
    if (bad != ~0ULL)
        throw Error{BPE_E_UTF8, "'utf-8' codec can't decode byte at position " + std::to_string(bad)};
    if (cr) return false;   // universal newlines change the text: the caller prepares it whole
    if (!cp.finish()) {     // the word table overflowed: recount the (now resident) text whole
        float kms = 0;
        count_words(d_dst, len, cp.wc, stream, timing_enabled() ? &kms : nullptr);
        cp.kernel_ms += kms;
    }
    pre.text = d_dst;
    pre.n = len;
    pre.wc = std::move(cp.wc);
    pre.count_kernel_ms = (float)cp.kernel_ms;
    pre.t_prepare_ms = 0;
    pre.t_count_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() - load_ms;
    pre.load_ms = load_ms;
    return true;
}

// ------------------------------------------------------------------ trainers
// test knob BPE355_INPROC_RANKS=1: the multi-device driver's ranks talk through an in-process
// communicator and may share devices, so its slab / exchange / error paths run on one GPU
bool inproc_ranks() { return std::getenv("BPE355_INPROC_RANKS") != nullptr; }

std::vector<int> pick_devices(int n_gpus) {
    int cur = 0, n = 0;
    BPE_HIP(hipGetDevice(&cur));
    BPE_HIP(hipGetDeviceCount(&n));
    BPE_REQUIRE(n > 0, BPE_E_HIP, "no HIP device visible");
    const int want = n_gpus <= 0 ? n : n_gpus;
    BPE_REQUIRE(want <= n || inproc_ranks(), BPE_E_ARG,
                "n_gpus = " + std::to_string(n_gpus) + " but only " + std::to_string(n) + " devices are visible");
    std::vector<int> d;
    for (int i = 0; i < want; ++i) d.push_back((cur + i) % n);   // the caller's device first
    return d;
}

void train_source(const Source& src, int vocab_size, const std::vector<std::string>& specials, int n_gpus,
                  TrainOutput& out) {
    const auto t0 = std::chrono::steady_clock::now();
    const std::vector<int> dev = pick_devices(n_gpus);
    const int g = (int)dev.size();
    if (g == 1) {
        static const bool dtrace = std::getenv("BPE355_DRIVE_TRACE") != nullptr;
        auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
        hipStream_t s = nullptr;
        BPE_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        struct SGuard { hipStream_t s; ~SGuard() { (void)hipStreamDestroy(s); } } sg{s};
        std::unique_ptr<CorpusBuf> d = corpus_take(std::max<size_t>(src.size, 1));
        const double a_ms = ms();
        Prepared pre;
        const bool counted = load_and_count(src, 0, src.size, d->b.p, dev[0], io_threads(), s, pre);
        const double load_ms = counted ? a_ms + pre.load_ms : ms();
        const double before_train = ms();
        train_on_device(d->b.p, src.size, vocab_size, specials, nullptr, s, out, TrainOpts{}, counted ? &pre : nullptr);
        if (dtrace) {
            const double tr = ms();
            std::fprintf(stderr, "[bpe355 drive] alloc %.1f stage %.1f train %.1f ms\n", a_ms, load_ms - a_ms,
                         tr - load_ms);
        }
        corpus_give(std::move(d));
        out.stats.t_load_ms = load_ms;
        out.stats.t_total_ms += before_train;
        out.stats.n_gpus = 1;
        return;
    }
    const std::vector<size_t> cut = slab_cuts(src, g);
    const bool inproc = inproc_ranks();
    uint8_t id[128] = {};
    std::shared_ptr<void> group;
    if (inproc) group = make_inproc_group();
    else BPE_REQUIRE(bpe_comm_unique_id(id) == BPE_OK, BPE_E_RCCL, "ncclGetUniqueId failed");
    std::vector<TrainOutput> outs(g);
    std::vector<std::exception_ptr> errs(g);
    std::vector<double> load_ms(g, 0);
    const int per = std::max(2, io_threads() / g);
    auto work = [&](int r) {
        try {
            BPE_HIP(hipSetDevice(dev[r]));
            hipStream_t s = nullptr;
            BPE_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            struct SGuard { hipStream_t s; ~SGuard() { (void)hipStreamDestroy(s); } } sg{s};
            const size_t len = cut[r + 1] - cut[r];
            std::unique_ptr<CorpusBuf> dbuf = corpus_take(std::max<size_t>(len, 1));
            uint8_t* const d = dbuf->b.p;
            TrainOpts opt;
            opt.slab_offset = cut[r];
            // every rank holds the union and one trains on it; per-round exchange: all of them
            opt.merge_loop = r == 0 || per_round_exchange();
            Prepared pre;
            bool counted = false;
            try {
                counted = load_and_count(src, cut[r], len, d, dev[r], per, s, pre);
            } catch (const Error& e) {
                opt.pending = e;   // reported by all ranks together, before any collective
                opt.has_pending = true;
            }
            load_ms[r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            auto comm = inproc ? make_inproc_comm(group, g, r, dev[r]) : make_rccl_comm(id, g, r, dev[r]);
            train_on_device(d, len, vocab_size, specials, comm.get(), s, outs[r], opt, counted ? &pre : nullptr);
            BPE_HIP(hipStreamSynchronize(s));
            corpus_give(std::move(dbuf));
        } catch (...) {
            errs[r] = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    for (int r = 1; r < g; ++r) th.emplace_back(work, r);
    work(0);
    for (auto& x : th) x.join();
    for (auto& e : errs)
        if (e) std::rethrow_exception(e);
    if (per_round_exchange())   // every rank ran the replicated argmax: they must agree exactly
        for (int r = 1; r < g; ++r)
            BPE_REQUIRE(outs[r].merges == outs[0].merges, BPE_E_RCCL,
                        "rank " + std::to_string(r) + " chose different merges than rank 0");
    out = std::move(outs[0]);
    out.stats.t_load_ms = *std::max_element(load_ms.begin(), load_ms.end());
    out.stats.t_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    out.stats.n_gpus = g;
    int64_t nb = 0;
    for (auto& o : outs) nb += o.stats.n_bytes;
    out.stats.n_bytes = nb;
}

void train_source_comm(const Source& src, bool split, int vocab_size, const std::vector<std::string>& specials,
                       Comm* comm, TrainOutput& out) {
    const auto t0 = std::chrono::steady_clock::now();
    int dev = 0;
    BPE_HIP(hipGetDevice(&dev));
    size_t lo = 0, hi = src.size;
    if (split && comm && comm->nranks > 1) {
        const std::vector<size_t> cut = slab_cuts(src, comm->nranks);
        lo = cut[comm->rank];
        hi = cut[comm->rank + 1];
    }
    hipStream_t s = nullptr;
    BPE_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct SGuard { hipStream_t s; ~SGuard() { (void)hipStreamDestroy(s); } } sg{s};
    std::unique_ptr<CorpusBuf> dbuf = corpus_take(std::max<size_t>(hi - lo, 1));
    uint8_t* const d = dbuf->b.p;
    TrainOpts opt;
    opt.slab_offset = lo;
    Prepared pre;
    bool counted = false;
    try {
        counted = load_and_count(src, lo, hi - lo, d, dev, io_threads(), s, pre);
    } catch (const Error& e) {
        if (!comm || comm->nranks == 1) throw;
        opt.pending = e;
        opt.has_pending = true;
    }
    const double before_train = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    train_on_device(d, hi - lo, vocab_size, specials, comm, s, out, opt, counted ? &pre : nullptr);
    corpus_give(std::move(dbuf));
    out.stats.t_load_ms = counted ? pre.load_ms : before_train;
    out.stats.t_total_ms += before_train;
    out.stats.n_gpus = comm ? comm->nranks : 1;
}

}  // namespace bpe
