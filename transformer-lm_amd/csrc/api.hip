// C ABI of libbpe355 (include/bpe355.h): argument checking, error codes, result objects.
#include <dlfcn.h>
#include <hip/hip_version.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <string>
#include <vector>

#include "count.h"
#include "drive.h"
#include "internal.h"

namespace bpe {

namespace {
thread_local std::string g_err;
thread_local int g_errno = 0;
bool g_timing = false;

struct DeviceGuard {
    // make sure a gfx950 device is present; there is no CPU fallback
    static void require() {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
            throw Error{BPE_E_HIP, "no HIP device visible (libbpe355 needs an MI355X / gfx950 GPU)"};
    }
};

template <class F>
int guarded(F&& f) {
    try {
        f();
        g_err.clear();
        return BPE_OK;
    } catch (const Error& e) {
        g_err = e.msg;
        g_errno = e.sys_errno;
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "host allocation failed";
        return BPE_E_NOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return BPE_E_ARG;
    }
}

std::vector<std::string> to_specials(const char* const* specials, int n) {
    BPE_REQUIRE(n >= 0 && (n == 0 || specials), BPE_E_ARG, "bad special token list");
    std::vector<std::string> v;
    for (int i = 0; i < n; ++i) {
        BPE_REQUIRE(specials[i], BPE_E_ARG, "null special token");
        v.emplace_back(specials[i]);
    }
    return v;
}

struct StreamHolder {
    hipStream_t s = nullptr;
    bool own = false;
    explicit StreamHolder(void* user) {
        if (user) {
            s = (hipStream_t)user;
        } else {
            BPE_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            own = true;
        }
    }
    ~StreamHolder() {
        if (own && s) (void)hipStreamDestroy(s);
    }
};

void put_u32(std::string& b, uint32_t v) { b.append(reinterpret_cast<const char*>(&v), 4); }

}  // namespace

void set_error(int, const std::string& msg, int sys_errno) {
    g_err = msg;
    g_errno = sys_errno;
}
bool timing_enabled() { return g_timing; }

}  // namespace bpe

struct bpe_result {
    std::vector<std::pair<std::string, std::string>> merges;   // byte pairs, in order
    std::vector<std::string> vocab;                            // id order
    std::vector<uint32_t> merge_ids;     // (a, b, a, b, ...) as vocab ids (empty: unavailable)
    int64_t n_merges = 0, n_vocab = 0;
    bpe_train_stats stats{};
    // the byte views, built on first request (the Python shim asks only for the vocab's flat
    // records and the merge ids): blobs, and (lengths, concatenated bytes) records to slice
    mutable std::once_flag once_mblob, once_vblob, once_flat[2];
    mutable std::string merges_blob, vocab_blob;
    mutable std::vector<uint32_t> flat_len[2];   // 0: merges (a, b, a, b, ...), 1: vocab in id order
    mutable std::string flat_bytes[2];
};

struct bpe_comm {
    std::unique_ptr<bpe::Comm> impl;
};

namespace bpe {
std::unique_ptr<Comm> make_rccl_comm(const uint8_t id[128], int nranks, int rank, int device);
std::unique_ptr<Comm> make_host_comm(bpe_host_allreduce_fn fn, void* ctx, int nranks, int rank,
                                     int device);
}  // namespace bpe

namespace {

// Vocab(special_tokens) + add_token per merge (reference models/tokenizer/vocab.py:2-34)
void finish_result(bpe::TrainOutput& out, const std::vector<std::string>& specials, bpe_result* r) {
    // the vocab in id order: a token whose bytes are already there is not added again
    // (vocab.py:29); every container sized up front (no rehash, and the vector never moves, so
    // the views the index keeps into its strings stay valid)
    const size_t cap = specials.size() + 256 + out.merges.size();
    std::vector<std::string> toks;
    toks.reserve(cap);
    std::unordered_map<std::string_view, uint32_t> id_of;
    id_of.reserve(2 * cap);
    auto add = [&](std::string s) {
        if (id_of.count(s)) return;
        toks.push_back(std::move(s));
        id_of.emplace(toks.back(), (uint32_t)(toks.size() - 1));
    };
    for (const auto& s : specials) add(s);
    for (int b = 0; b < 256; ++b) add(std::string(1, (char)b));
    for (const auto& m : out.merges) add(m.first + m.second);
    r->n_merges = (int64_t)out.merges.size();
    r->n_vocab = (int64_t)toks.size();
    r->merge_ids.reserve(2 * out.merges.size());
    for (const auto& m : out.merges) {
        const auto ia = id_of.find(m.first), ib = id_of.find(m.second);   // (a part is always a token)
        if (ia == id_of.end() || ib == id_of.end()) { r->merge_ids.clear(); break; }
        r->merge_ids.push_back(ia->second);
        r->merge_ids.push_back(ib->second);
    }
    id_of.clear();   // (views into toks: dropped before toks moves)
    r->merges = std::move(out.merges);
    r->vocab = std::move(toks);
    r->stats = out.stats;
}

int train_common(const uint8_t* d_data, size_t n, int vocab_size, const char* const* specials,
                 int n_specials, bpe_comm* comm, void* stream, bpe_result** out) {
    return bpe::guarded([&] {
        BPE_REQUIRE(out, BPE_E_ARG, "out is NULL");
        *out = nullptr;
        bpe::DeviceGuard::require();
        auto sp = bpe::to_specials(specials, n_specials);
        bpe::StreamHolder sh(stream);
        bpe::TrainOutput to;
        bpe::train_on_device(d_data, n, vocab_size, sp, comm ? comm->impl.get() : nullptr, sh.s, to);
        auto r = std::make_unique<bpe_result>();
        finish_result(to, sp, r.get());
        *out = r.release();
    });
}

}  // namespace

extern "C" {

int bpe_abi_version(void) { return BPE355_ABI_VERSION; }

int bpe_runtime_info(int* compiled_hip_version, int* runtime_hip_version, char* runtime_path, size_t cap) {
    if (compiled_hip_version) *compiled_hip_version = HIP_VERSION;
    int rv = 0;
    const hipError_t e = hipRuntimeGetVersion(&rv);
    if (runtime_hip_version) *runtime_hip_version = e == hipSuccess ? rv : 0;
    if (runtime_path && cap) {
        runtime_path[0] = '\0';
        Dl_info di{};
        if (dladdr(reinterpret_cast<void*>(&hipRuntimeGetVersion), &di) && di.dli_fname)
            std::snprintf(runtime_path, cap, "%s", di.dli_fname);
    }
    return e == hipSuccess ? BPE_OK : BPE_E_HIP;
}
const char* bpe_last_error(void) { return bpe::g_err.c_str(); }
int bpe_last_errno(void) { return bpe::g_errno; }
void bpe_set_timing(int enable) { bpe::g_timing = enable != 0; }

int bpe_release_device_memory(int device, size_t* freed_bytes) {
    return bpe::guarded([&] {
        if (freed_bytes) *freed_bytes = 0;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        BPE_REQUIRE(device < n, BPE_E_ARG, "device " + std::to_string(device) + " is not visible");
        size_t b = bpe::corpus_release(device);
        b += bpe::scratch_release(device);
        // the copy streams stay: they hold no HBM to speak of, and a transfer of another thread
        // (encode_file, train_bpe) may be using them right now (drive.hip, DmaCache)
        if (freed_bytes) *freed_bytes = b;
    });
}

int bpe_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int k = 0;
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) == hipSuccess && std::strncmp(p.gcnArchName, "gfx950", 6) == 0) ++k;
    }
    return k;
}

int bpe_train_device(const uint8_t* d_data, size_t n, int vocab_size, const char* const* specials,
                     int n_specials, bpe_comm* comm, void* hip_stream, bpe_result** out) {
    if (n && !d_data) return bpe::guarded([] { throw bpe::Error{BPE_E_ARG, "data is NULL"}; });
    return train_common(d_data, n, vocab_size, specials, n_specials, comm, hip_stream, out);
}

int bpe_train_buffer(const uint8_t* data, size_t n, int vocab_size, const char* const* specials,
                     int n_specials, bpe_comm* comm, bpe_result** out) {
    return bpe::guarded([&] {
        BPE_REQUIRE(out, BPE_E_ARG, "out is NULL");
        *out = nullptr;
        BPE_REQUIRE(!n || data, BPE_E_ARG, "data is NULL");
        bpe::DeviceGuard::require();
        auto sp = bpe::to_specials(specials, n_specials);
        const bpe::Source src = bpe::Source::memory(data, n);
        bpe::TrainOutput to;
        if (comm) bpe::train_source_comm(src, false, vocab_size, sp, comm->impl.get(), to);
        else bpe::train_source(src, vocab_size, sp, 1, to);
        auto r = std::make_unique<bpe_result>();
        finish_result(to, sp, r.get());
        *out = r.release();
    });
}

int bpe_train_buffer_gpus(const uint8_t* data, size_t n, int vocab_size, const char* const* specials,
                          int n_specials, int n_gpus, bpe_result** out) {
    return bpe::guarded([&] {
        BPE_REQUIRE(out, BPE_E_ARG, "out is NULL");
        *out = nullptr;
        BPE_REQUIRE(!n || data, BPE_E_ARG, "data is NULL");
        bpe::DeviceGuard::require();
        auto sp = bpe::to_specials(specials, n_specials);
        const bpe::Source src = bpe::Source::memory(data, n);
        bpe::TrainOutput to;
        bpe::train_source(src, vocab_size, sp, n_gpus, to);
        auto r = std::make_unique<bpe_result>();
        finish_result(to, sp, r.get());
        *out = r.release();
    });
}

int bpe_train_file(const char* path, int vocab_size, const char* const* specials, int n_specials,
                   int n_gpus, bpe_result** out) {
    return bpe::guarded([&] {
        BPE_REQUIRE(out, BPE_E_ARG, "out is NULL");
        *out = nullptr;
        BPE_REQUIRE(path, BPE_E_ARG, "path is NULL");
        auto sp = bpe::to_specials(specials, n_specials);
        const bpe::Source src = bpe::Source::open_path(path);   // FileNotFoundError before any GPU check
        bpe::DeviceGuard::require();
        bpe::TrainOutput to;
        bpe::train_source(src, vocab_size, sp, n_gpus, to);
        auto r = std::make_unique<bpe_result>();
        finish_result(to, sp, r.get());
        *out = r.release();
    });
}

int bpe_train_file_comm(const char* path, int vocab_size, const char* const* specials, int n_specials,
                        bpe_comm* comm, int split, bpe_result** out) {
    return bpe::guarded([&] {
        BPE_REQUIRE(out, BPE_E_ARG, "out is NULL");
        *out = nullptr;
        BPE_REQUIRE(path, BPE_E_ARG, "path is NULL");
        auto sp = bpe::to_specials(specials, n_specials);
        const bpe::Source src = bpe::Source::open_path(path);
        bpe::DeviceGuard::require();
        bpe::TrainOutput to;
        bpe::train_source_comm(src, split != 0, vocab_size, sp, comm ? comm->impl.get() : nullptr, to);
        auto r = std::make_unique<bpe_result>();
        finish_result(to, sp, r.get());
        *out = r.release();
    });
}

int bpe_word_counts(const uint8_t* data, size_t n, const char* const* specials, int n_specials,
                    uint8_t** blob, size_t* blob_n) {
    return bpe::guarded([&] {
        BPE_REQUIRE(blob && blob_n, BPE_E_ARG, "blob is NULL");
        *blob = nullptr;
        *blob_n = 0;
        BPE_REQUIRE(!n || data, BPE_E_ARG, "data is NULL");
        bpe::DeviceGuard::require();
        auto sp = bpe::to_specials(specials, n_specials);
        bpe::StreamHolder sh(nullptr);
        bpe::DevBuf<uint8_t> d(std::max<size_t>(n, 1)), scratch;
        if (n) BPE_HIP(hipMemcpyAsync(d.p, data, n, hipMemcpyHostToDevice, sh.s));
        size_t tn = 0;
        const uint8_t* text = bpe::prepare_text(d.p, n, scratch, &tn, sh.s);
        bpe::WordCounts wc;
        bpe::count_words(text, tn, wc, sh.s, nullptr);
        // the table as the merge loop's word collection reads it (k_collect_words): inline keys
        // hold len and bytes, the others len << 40 | offset + 1 of the first occurrence
        std::vector<unsigned long long> kv(2 * wc.cap), pos(wc.cap);
        std::string t(tn, '\0');
        BPE_HIP(hipMemcpyAsync(kv.data(), wc.kv.p, kv.size() * 8, hipMemcpyDeviceToHost, sh.s));
        BPE_HIP(hipMemcpyAsync(pos.data(), wc.pos.p, pos.size() * 8, hipMemcpyDeviceToHost, sh.s));
        if (tn) BPE_HIP(hipMemcpyAsync(&t[0], text, tn, hipMemcpyDeviceToHost, sh.s));
        BPE_HIP(hipStreamSynchronize(sh.s));
        std::unordered_set<std::string> skip(sp.begin(), sp.end());
        std::string out;
        for (size_t i = 0; i < wc.cap; ++i) {
            const unsigned long long k = kv[2 * i];
            if (!k) continue;
            const bool inl = (k >> 63) != 0;
            const size_t len = inl ? (size_t)((k >> 56) & 0x7f) : (size_t)(k >> 40);
            const size_t off = inl ? (size_t)pos[i] : (size_t)((k & ((1ULL << 40) - 1)) - 1);
            const std::string w = t.substr(off, len);
            if (skip.count(w)) continue;
            bpe::put_u32(out, (uint32_t)len);
            out += w;
            const unsigned long long c = kv[2 * i + 1];
            out.append(reinterpret_cast<const char*>(&c), 8);
        }
        *blob = static_cast<uint8_t*>(std::malloc(std::max<size_t>(out.size(), 1)));
        BPE_REQUIRE(*blob, BPE_E_NOMEM, "host allocation failed");
        std::memcpy(*blob, out.data(), out.size());
        *blob_n = out.size();
    });
}

void bpe_blob_free(uint8_t* blob) { std::free(blob); }

size_t bpe_result_flat(const bpe_result* r, int which, const uint32_t** lens, const uint8_t** bytes,
                       size_t* n_bytes) {
    if (!r || which < 0 || which > 1 || !lens || !bytes || !n_bytes) return 0;
    std::call_once(r->once_flat[which], [&] {
        std::vector<uint32_t>& L = r->flat_len[which];
        std::string& B = r->flat_bytes[which];
        size_t nb = 0;
        if (which == 0) {
            for (const auto& m : r->merges) nb += m.first.size() + m.second.size();
            L.reserve(2 * r->merges.size());
            B.reserve(nb);
            for (const auto& m : r->merges) {
                L.push_back((uint32_t)m.first.size());
                L.push_back((uint32_t)m.second.size());
                B += m.first;
                B += m.second;
            }
        } else {
            for (const auto& t : r->vocab) nb += t.size();
            L.reserve(r->vocab.size());
            B.reserve(nb);
            for (const auto& t : r->vocab) {
                L.push_back((uint32_t)t.size());
                B += t;
            }
        }
    });
    *lens = r->flat_len[which].data();
    *bytes = reinterpret_cast<const uint8_t*>(r->flat_bytes[which].data());
    *n_bytes = r->flat_bytes[which].size();
    return r->flat_len[which].size();
}

size_t bpe_result_merge_ids(const bpe_result* r, const uint32_t** ids) {
    if (!r || !ids || r->merge_ids.size() != 2 * (size_t)r->n_merges) return 0;
    *ids = r->merge_ids.data();
    return (size_t)r->n_merges;
}

int64_t bpe_result_n_merges(const bpe_result* r) { return r ? r->n_merges : -1; }
int64_t bpe_result_n_vocab(const bpe_result* r) { return r ? r->n_vocab : -1; }
size_t bpe_result_merges_blob(const bpe_result* r, const uint8_t** data) {
    if (!r || !data) return 0;
    std::call_once(r->once_mblob, [&] {
        for (const auto& m : r->merges) {
            bpe::put_u32(r->merges_blob, (uint32_t)m.first.size());
            r->merges_blob += m.first;
            bpe::put_u32(r->merges_blob, (uint32_t)m.second.size());
            r->merges_blob += m.second;
        }
    });
    *data = reinterpret_cast<const uint8_t*>(r->merges_blob.data());
    return r->merges_blob.size();
}
size_t bpe_result_vocab_blob(const bpe_result* r, const uint8_t** data) {
    if (!r || !data) return 0;
    std::call_once(r->once_vblob, [&] {
        for (const auto& t : r->vocab) {
            bpe::put_u32(r->vocab_blob, (uint32_t)t.size());
            r->vocab_blob += t;
        }
    });
    *data = reinterpret_cast<const uint8_t*>(r->vocab_blob.data());
    return r->vocab_blob.size();
}
int bpe_result_stats(const bpe_result* r, bpe_train_stats* out) {
    if (!r || !out) return BPE_E_ARG;
    *out = r->stats;
    return BPE_OK;
}
void bpe_result_free(bpe_result* r) { delete r; }

int bpe_comm_unique_id(uint8_t id_out[128]);
int bpe_comm_init(const uint8_t id[128], int nranks, int rank, int device, bpe_comm** out) {
    return bpe::guarded([&] {
        BPE_REQUIRE(out && id && nranks >= 1 && rank >= 0 && rank < nranks, BPE_E_ARG, "bad comm args");
        auto c = std::make_unique<bpe_comm>();
        c->impl = bpe::make_rccl_comm(id, nranks, rank, device);
        *out = c.release();
    });
}
int bpe_comm_init_host(bpe_host_allreduce_fn fn, void* ctx, int nranks, int rank, int device,
                       bpe_comm** out) {
    return bpe::guarded([&] {
        BPE_REQUIRE(out && fn && nranks >= 1 && rank >= 0 && rank < nranks, BPE_E_ARG, "bad comm args");
        auto c = std::make_unique<bpe_comm>();
        c->impl = bpe::make_host_comm(fn, ctx, nranks, rank, device);
        *out = c.release();
    });
}
void bpe_comm_free(bpe_comm* comm) { delete comm; }

size_t bpe_safe_split(const uint8_t* data, size_t n, size_t pos) {
    auto ascii_nonspace = [](uint8_t b) { return b < 0x80 && b != 0x20 && (b < 0x09 || b > 0x0D); };
    if (!data || n < 3) return 0;
    if (pos > n - 2) pos = n - 2;
    for (size_t p = pos; p >= 1; --p)
        if (data[p] == 0x20 && ascii_nonspace(data[p - 1]) && ascii_nonspace(data[p + 1])) return p;
    return 0;
}

}  // extern "C"
