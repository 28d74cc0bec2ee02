// Device-wide scans, sorts and selections on rocPRIM (AMD's own primitives library; no CUB-shaped
// layer): exclusive prefix sums for offsets, the posting index's radix sort, the newline filter.
// Each call sizes its temporary storage with a first rocPRIM call and reuses a caller's buffer
// when one is given (grow-only), else allocates one for the call.
#pragma once

#include <rocprim/block/block_scan.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include <algorithm>

#include "bpe_common.h"

namespace bpe {

// out[i] = in[0] + ... + in[i - 1], i < n
template <class T>
void exclusive_sum(const T* in, T* out, size_t n, hipStream_t s, DevBuf<uint8_t>* keep = nullptr) {
    if (n == 0) return;
    DevBuf<uint8_t> local;
    DevBuf<uint8_t>& tmp = keep ? *keep : local;
    size_t tb = 0;
    BPE_HIP(rocprim::exclusive_scan(nullptr, tb, in, out, T(0), n, rocprim::plus<T>(), s));
    tmp.reserve(std::max<size_t>(tb, 1));
    BPE_HIP(rocprim::exclusive_scan(tmp.p, tb, in, out, T(0), n, rocprim::plus<T>(), s));
}

// (keys, values) sorted by the key bits [0, end_bit), stable
template <class K, class V>
void radix_sort_pairs(const K* kin, K* kout, const V* vin, V* vout, size_t n, unsigned end_bit, hipStream_t s,
                      DevBuf<uint8_t>* keep = nullptr) {
    if (n == 0) return;
    DevBuf<uint8_t> local;
    DevBuf<uint8_t>& tmp = keep ? *keep : local;
    size_t tb = 0;
    BPE_HIP(rocprim::radix_sort_pairs(nullptr, tb, kin, kout, vin, vout, n, 0u, end_bit, s));
    tmp.reserve(std::max<size_t>(tb, 1));
    BPE_HIP(rocprim::radix_sort_pairs(tmp.p, tb, kin, kout, vin, vout, n, 0u, end_bit, s));
}

// keys sorted by the bits [0, end_bit)
template <class K>
void radix_sort_keys(const K* kin, K* kout, size_t n, unsigned end_bit, hipStream_t s, DevBuf<uint8_t>* keep = nullptr) {
    if (n == 0) return;
    DevBuf<uint8_t> local;
    DevBuf<uint8_t>& tmp = keep ? *keep : local;
    size_t tb = 0;
    BPE_HIP(rocprim::radix_sort_keys(nullptr, tb, kin, kout, n, 0u, end_bit, s));
    tmp.reserve(std::max<size_t>(tb, 1));
    BPE_HIP(rocprim::radix_sort_keys(tmp.p, tb, kin, kout, n, 0u, end_bit, s));
}

// out = the in[i] with flags[i] != 0, in order; *d_count = how many (device)
template <class T, class F, class C>
void select_flagged(const T* in, const F* flags, T* out, C* d_count, size_t n, hipStream_t s) {
    DevBuf<uint8_t> tmp;
    size_t tb = 0;
    BPE_HIP(rocprim::select(nullptr, tb, in, flags, out, d_count, n, s));
    tmp.reserve(std::max<size_t>(tb, 1));
    BPE_HIP(rocprim::select(tmp.p, tb, in, flags, out, d_count, n, s));
}

}  // namespace bpe
