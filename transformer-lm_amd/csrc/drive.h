// Host driver of train_bpe(path) (drive.hip): parallel file -> HBM staging, slab cutting and
// the multi-device trainer.
#pragma once

#include <string>
#include <vector>

#include "internal.h"

namespace bpe {

// Bytes of a corpus: a regular file (read with pread by many threads) or host memory (a pipe
// or FIFO is read to EOF first).
struct Source {
    int fd = -1;
    const uint8_t* mem = nullptr;
    size_t size = 0;
    std::string name;
    std::vector<uint8_t> owned;
    static Source open_path(const char* path);   // throws Error{BPE_E_IO} with errno
    static Source memory(const uint8_t* p, size_t n);
    Source() = default;
    Source(Source&& o) noexcept
        : fd(o.fd), mem(o.mem), size(o.size), name(std::move(o.name)), owned(std::move(o.owned)) {
        o.fd = -1;
        if (!owned.empty()) mem = owned.data();
    }
    Source(const Source&) = delete;
    ~Source();
    void read(size_t off, size_t len, uint8_t* dst) const;
};

int io_threads();
// g + 1 cut points [0, c1, ..., size] at safe split points
std::vector<size_t> slab_cuts(const Source& src, int g);
// src[off, off + len) -> d_dst on `device`, through pinned staging, `threads` readers
void stage_to_device(const Source& src, size_t off, size_t len, uint8_t* d_dst, int device, int threads);
// d_src[0, len) on `device` -> host memory h_dst (pageable), through pinned staging, `threads` copiers
void device_to_host(const uint8_t* d_src, size_t len, uint8_t* h_dst, int device, int threads);
// src[off, off + len) -> d_dst, validated and counted segment by segment as it arrives
// (false: the text holds a \r, so the caller must apply universal newlines and count it whole)
bool load_and_count(const Source& src, size_t off, size_t len, uint8_t* d_dst, int device, int threads,
                    hipStream_t stream, Prepared& pre);
std::vector<int> pick_devices(int n_gpus);
// train_bpe over the whole source on n_gpus devices of this process (<= 0: all visible)
void train_source(const Source& src, int vocab_size, const std::vector<std::string>& specials, int n_gpus,
                  TrainOutput& out);
// one rank of a multi-process job: the source is this rank's slab, or (split) the whole corpus
// of which this rank reads its share
void train_source_comm(const Source& src, bool split, int vocab_size, const std::vector<std::string>& specials,
                       Comm* comm, TrainOutput& out);
// bpe_release_device_memory: the corpus buffers kept for `dev` (< 0: every device) go back to the
// device allocator; returns the bytes freed.  Buffers a running call holds are not touched, and the
// cached copy streams are kept for the process (a concurrent transfer may be using them)
size_t corpus_release(int dev);

}  // namespace bpe
