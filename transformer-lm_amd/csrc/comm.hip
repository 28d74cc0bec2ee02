// Communicators for the sharded trainer: one process per GPU, corpus slabs per rank.  The
// default exchange is one all-gather of the ranks' unique-word tables (exchange.hip); the
// per-round exchange (BPE355_EXCHANGE=rounds) is one sum all-reduce of the pair deltas per
// merge round (and once of the initial byte-pair histogram).  RCCL over xGMI in production; a host-staged variant lets the sharded path be
// exercised by several processes that share one GPU (tests).
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <memory>
#include <vector>

#include "internal.h"

namespace bpe {

namespace {

#define BPE_NCCL(expr)                                                                       \
    do {                                                                                     \
        ncclResult_t r_ = (expr);                                                            \
        if (r_ != ncclSuccess)                                                               \
            throw Error{BPE_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)};     \
    } while (0)

struct RcclComm final : Comm {
    ncclComm_t comm = nullptr;
    RcclComm(const uint8_t id[128], int n, int r, int dev) {
        nranks = n;
        rank = r;
        device = dev;
        BPE_HIP(hipSetDevice(dev));
        ncclUniqueId uid;
        static_assert(sizeof(uid.internal) == 128, "ncclUniqueId size");
        std::memcpy(uid.internal, id, 128);
        BPE_NCCL(ncclCommInitRank(&comm, n, uid, r));
    }
    ~RcclComm() override {
        if (comm) (void)ncclCommDestroy(comm);
    }
    void allreduce_i64(int64_t* d_buf, size_t count, hipStream_t stream) override {
        if (count == 0) return;
        BPE_NCCL(ncclAllReduce(d_buf, d_buf, count, ncclInt64, ncclSum, comm, stream));
    }
    void allgather_bytes(const void* d_send, size_t bytes, void* d_recv, hipStream_t stream) override {
        if (bytes == 0) return;
        BPE_NCCL(ncclAllGather(d_send, d_recv, bytes, ncclUint8, comm, stream));
    }
    // one grouped send/recv per peer over xGMI (the own share is a device copy)
    void alltoallv_bytes(const void* d_send, const size_t* soff, const size_t* scnt, void* d_recv,
                         const size_t* roff, const size_t* rcnt, hipStream_t stream) override {
        const uint8_t* snd = static_cast<const uint8_t*>(d_send);
        uint8_t* rcv = static_cast<uint8_t*>(d_recv);
        if (scnt[rank])
            BPE_HIP(hipMemcpyAsync(rcv + roff[rank], snd + soff[rank], scnt[rank], hipMemcpyDeviceToDevice, stream));
        BPE_NCCL(ncclGroupStart());
        for (int p = 0; p < nranks; ++p) {
            if (p == rank) continue;
            if (scnt[p]) BPE_NCCL(ncclSend(snd + soff[p], scnt[p], ncclUint8, p, comm, stream));
            if (rcnt[p]) BPE_NCCL(ncclRecv(rcv + roff[p], rcnt[p], ncclUint8, p, comm, stream));
        }
        BPE_NCCL(ncclGroupEnd());
    }
};

struct HostComm final : Comm {
    bpe_host_allreduce_fn fn;
    void* ctx;
    std::vector<int64_t> buf;
    HostComm(bpe_host_allreduce_fn f, void* c, int n, int r, int dev) : fn(f), ctx(c) {
        nranks = n;
        rank = r;
        device = dev;
    }
    void allreduce_i64(int64_t* d_buf, size_t count, hipStream_t stream) override {
        if (count == 0) return;
        buf.resize(count);
        BPE_HIP(hipMemcpyAsync(buf.data(), d_buf, count * 8, hipMemcpyDeviceToHost, stream));
        BPE_HIP(hipStreamSynchronize(stream));
        BPE_REQUIRE(fn(ctx, buf.data(), count) == 0, BPE_E_RCCL, "host all-reduce callback failed");
        BPE_HIP(hipMemcpyAsync(d_buf, buf.data(), count * 8, hipMemcpyHostToDevice, stream));
        BPE_HIP(hipStreamSynchronize(stream));
    }
};

// Ranks that are threads of one process (tests of the multi-device driver on a one-GPU box:
// several ranks may share a device, which RCCL refuses).  A generation-counted barrier: the sum
// of an operation is published when the last rank arrives; a rank cannot start the next
// operation's sum before every rank has taken this one's result, because that needs them all.
struct InProcShared {
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<int64_t> acc, result;
    std::vector<uint8_t> gather;   // all-gather: rank r's segment at r * bytes
    int g_entered = 0, g_readers = 0;
    // all-to-all: every rank's whole send buffer and its offsets / sizes per destination
    std::vector<std::vector<uint8_t>> a2a;
    std::vector<std::vector<size_t>> a2a_off, a2a_cnt;
    // a rank left a collective with an error: every rank waiting in (or later entering) one
    // throws instead of waiting for it forever
    bool failed = false;
};

struct InProcComm final : Comm {
    std::shared_ptr<InProcShared> sh;
    std::vector<int64_t> h;
    InProcComm(std::shared_ptr<InProcShared> s, int n, int r, int dev) : sh(std::move(s)) {
        nranks = n;
        rank = r;
        device = dev;
    }
    // runs op; any exception it throws marks the group failed (waking every waiter) and goes on
    template <class Op>
    void guarded(const Op& op) {
        try {
            op();
        } catch (...) {
            {
                std::lock_guard<std::mutex> g(sh->m);
                sh->failed = true;
            }
            sh->cv.notify_all();
            throw;
        }
    }
    void check_failed() const {   // sh->m held
        BPE_REQUIRE(!sh->failed, BPE_E_RCCL, "in-process collective: another rank failed");
    }
    void allreduce_i64(int64_t* d_buf, size_t count, hipStream_t stream) override {
        if (count == 0) return;
        guarded([&] {
            h.resize(count);
            BPE_HIP(hipMemcpyAsync(h.data(), d_buf, count * 8, hipMemcpyDeviceToHost, stream));
            BPE_HIP(hipStreamSynchronize(stream));
            {
                std::unique_lock<std::mutex> lk(sh->m);
                check_failed();
                const uint64_t g = sh->gen;
                if (sh->arrived == 0) sh->acc.assign(count, 0);
                BPE_REQUIRE(sh->acc.size() == count, BPE_E_RCCL, "in-process all-reduce: ranks disagree on the size");
                for (size_t i = 0; i < count; ++i) sh->acc[i] += h[i];
                if (++sh->arrived == nranks) {
                    sh->result.swap(sh->acc);
                    sh->arrived = 0;
                    ++sh->gen;
                    sh->cv.notify_all();
                } else {
                    sh->cv.wait(lk, [&] { return sh->gen != g || sh->failed; });
                    check_failed();
                }
                h = sh->result;
            }
            BPE_HIP(hipMemcpyAsync(d_buf, h.data(), count * 8, hipMemcpyHostToDevice, stream));
            BPE_HIP(hipStreamSynchronize(stream));
        });
    }
    // ncclAllGather's contract: every rank copies its segment into one shared host buffer, and
    // after the last rank arrives each one copies the whole buffer back (no zero-padded sum)
    void allgather_bytes(const void* d_send, size_t bytes, void* d_recv, hipStream_t stream) override {
        if (bytes == 0) return;
        guarded([&] {
            std::unique_lock<std::mutex> lk(sh->m);
            // a rank done with the previous gather may not reset the buffer others still read
            sh->cv.wait(lk, [&] { return sh->g_readers == 0 || sh->failed; });
            check_failed();
            const uint64_t g = sh->gen;
            if (sh->g_entered == 0) sh->gather.assign((size_t)nranks * bytes, 0);
            BPE_REQUIRE(sh->gather.size() == (size_t)nranks * bytes, BPE_E_RCCL,
                        "in-process all-gather: ranks disagree on the size");
            ++sh->g_entered;
            uint8_t* mine = sh->gather.data() + (size_t)rank * bytes;
            lk.unlock();   // the copies of the ranks' own segments run concurrently
            BPE_HIP(hipMemcpyAsync(mine, d_send, bytes, hipMemcpyDeviceToHost, stream));
            BPE_HIP(hipStreamSynchronize(stream));
            lk.lock();
            check_failed();
            if (++sh->arrived == nranks) {
                sh->arrived = 0;
                sh->g_entered = 0;
                sh->g_readers = nranks;
                ++sh->gen;
                sh->cv.notify_all();
            } else {
                sh->cv.wait(lk, [&] { return sh->gen != g || sh->failed; });
                check_failed();
            }
            const uint8_t* all = sh->gather.data();
            lk.unlock();
            BPE_HIP(hipMemcpyAsync(d_recv, all, (size_t)nranks * bytes, hipMemcpyHostToDevice, stream));
            BPE_HIP(hipStreamSynchronize(stream));
            lk.lock();
            --sh->g_readers;
            sh->cv.notify_all();
        });
    }
    // every rank stages its send buffer in host memory; after the last one arrives each copies
    // its share of every rank's buffer (rank q's bytes for this rank) back to its device
    void alltoallv_bytes(const void* d_send, const size_t* soff, const size_t* scnt, void* d_recv,
                         const size_t* roff, const size_t* rcnt, hipStream_t stream) override {
        guarded([&] {
            size_t total = 0;
            for (int p = 0; p < nranks; ++p) total = std::max(total, soff[p] + scnt[p]);
            std::unique_lock<std::mutex> lk(sh->m);
            sh->cv.wait(lk, [&] { return sh->g_readers == 0 || sh->failed; });
            check_failed();
            const uint64_t g = sh->gen;
            if (sh->g_entered == 0) {
                sh->a2a.assign(nranks, {});
                sh->a2a_off.assign(nranks, {});
                sh->a2a_cnt.assign(nranks, {});
            }
            ++sh->g_entered;
            std::vector<uint8_t>& mine = sh->a2a[rank];
            sh->a2a_off[rank].assign(soff, soff + nranks);
            sh->a2a_cnt[rank].assign(scnt, scnt + nranks);
            lk.unlock();
            mine.resize(total);
            if (total) BPE_HIP(hipMemcpyAsync(mine.data(), d_send, total, hipMemcpyDeviceToHost, stream));
            BPE_HIP(hipStreamSynchronize(stream));
            lk.lock();
            check_failed();
            if (++sh->arrived == nranks) {
                sh->arrived = 0;
                sh->g_entered = 0;
                sh->g_readers = nranks;
                ++sh->gen;
                sh->cv.notify_all();
            } else {
                sh->cv.wait(lk, [&] { return sh->gen != g || sh->failed; });
                check_failed();
            }
            lk.unlock();
            for (int q = 0; q < nranks; ++q) {
                const size_t c = sh->a2a_cnt[q][rank];
                BPE_REQUIRE(c == rcnt[q], BPE_E_RCCL, "in-process all-to-all: ranks disagree on a size");
                if (c)
                    BPE_HIP(hipMemcpyAsync(static_cast<uint8_t*>(d_recv) + roff[q], sh->a2a[q].data() + sh->a2a_off[q][rank],
                                           c, hipMemcpyHostToDevice, stream));
            }
            BPE_HIP(hipStreamSynchronize(stream));
            lk.lock();
            --sh->g_readers;
            sh->cv.notify_all();
        });
    }
};

}  // namespace

std::shared_ptr<void> make_inproc_group() { return std::make_shared<InProcShared>(); }
std::unique_ptr<Comm> make_inproc_comm(const std::shared_ptr<void>& group, int nranks, int rank, int device) {
    return std::make_unique<InProcComm>(std::static_pointer_cast<InProcShared>(group), nranks, rank, device);
}

std::unique_ptr<Comm> make_rccl_comm(const uint8_t id[128], int nranks, int rank, int device) {
    return std::make_unique<RcclComm>(id, nranks, rank, device);
}
std::unique_ptr<Comm> make_host_comm(bpe_host_allreduce_fn fn, void* ctx, int nranks, int rank,
                                     int device) {
    return std::make_unique<HostComm>(fn, ctx, nranks, rank, device);
}

}  // namespace bpe

extern "C" int bpe_comm_unique_id(uint8_t id_out[128]) {
    if (!id_out) return BPE_E_ARG;
    ncclUniqueId uid;
    const ncclResult_t r = ncclGetUniqueId(&uid);
    if (r != ncclSuccess) {
        bpe::set_error(BPE_E_RCCL, ncclGetErrorString(r));
        return BPE_E_RCCL;
    }
    std::memcpy(id_out, uid.internal, 128);
    return BPE_OK;
}
