// Host evaluation of the byte-parallel token-start predicate (tokstart.h), block by block exactly
// as the device counter evaluates it, for the CPU tests that check it against the serial scanner
// and the oracle (tests/test_tokstart.py).  Test support: no product path calls it.
#include <cstring>

#include "internal.h"
#include "tokstart.h"

namespace bpe {
namespace hosttab {
#define BPE_UCTAB static const
#include "uniclass_tables.inc"
#undef BPE_UCTAB
struct Tab {
    static unsigned page(unsigned i) { return BPE_UC_PAGE[i]; }
    static unsigned bits(unsigned pg, unsigned i) { return BPE_UC_BITS[pg][i]; }
    static int cls(uint32_t cp) { return uc_class<Tab>(cp); }
};
}  // namespace hosttab
}  // namespace bpe

namespace {
struct HostWin {
    const uint8_t* b;
    uint32_t byte(int j) const { return b[j]; }
    uint32_t dword(int k) const {
        return (uint32_t)b[4 * k] | ((uint32_t)b[4 * k + 1] << 8) | ((uint32_t)b[4 * k + 2] << 16) |
               ((uint32_t)b[4 * k + 3] << 24);
    }
};
}  // namespace

// flags[i] = 1 when a pre-token of text[0..n) begins at byte i (n >= 1: flags[0] = 1)
extern "C" int bpe_pretok_starts_host(const uint8_t* text, size_t n, uint8_t* flags) {
    if ((!text && n) || !flags) return BPE_E_ARG;
    for (size_t o = 0; o < n; o += 64) {
        uint8_t w[bpe::kStartWin];
        for (int j = 0; j < bpe::kStartWin; ++j) {
            const long long p = (long long)o - bpe::kStartPre + j;
            w[j] = p < 0 ? '\n' : (p < (long long)n ? text[p] : 0);
        }
        const long long vhi = (long long)n - ((long long)o - bpe::kStartPre);
        uint64_t m = bpe::token_starts64<bpe::hosttab::Tab>(HostWin{w}, (int)(vhi > bpe::kStartWin ? bpe::kStartWin : vhi));
        if (o == 0) m |= 1;   // the text start
        for (int k = 0; k < 64 && o + k < n; ++k) flags[o + k] = (uint8_t)((m >> k) & 1);
    }
    return BPE_OK;
}
