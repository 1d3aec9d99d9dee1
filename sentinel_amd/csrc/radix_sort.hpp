#pragma once
#include "common.hpp"

namespace sga {

// 16-byte payload carried through the sort: original index, timestamp offset,
// acquire count with the prioritized flag in bit 31, and the low 32 bits of the
// request's window-bucket index (t / windowLengthInMs of its rule).
struct alignas(16) Payload {
    uint32_t idx;
    uint32_t ts_off;
    uint32_t acq_prio;
    uint32_t bucket;
};

constexpr int kMaxDigitBits = 11;

struct RadixScratch {
    uint32_t *ghist = nullptr;      // look-back mode: kRadixMaxPasses x 2048 digit totals + tile counters
    uint32_t *err = nullptr;        // look-back mode: error flag (a look-back gave up)
    uint32_t *hist = nullptr;       // radix_hist_entries(n, bits)
    uint32_t *hist_scan = nullptr;  // same size
    uint32_t *partial = nullptr;    // scan_partials_needed(hist entries)
};

size_t radix_tiles(size_t n);
size_t radix_hist_entries(size_t n, int bits);
size_t scan_partials_needed(size_t n);
void exclusive_scan_u32(const uint32_t *in, uint32_t *out, size_t n, uint32_t *partial, hipStream_t s);

// Stable sort by the low `bits` bits of keys.  Returns the number of passes;
// the sorted data is in (keys, pay) when it is even, in the alt buffers when odd.
int radix_sort_pairs(uint32_t *keys, Payload *pay, uint32_t *keys_alt, Payload *pay_alt, size_t n, int bits,
                     RadixScratch &sc, hipStream_t s);

// Stable LSD sort of u64 elements by their bits [key_shift, key_shift + bits), tiles of
// radix64_tile() elements, radix64_digit_bits(bits) bits per pass.  When hist0_ready, the
// first pass's per-tile digit histogram (digit-major: hist[d * ntiles + tile]) is already in
// sc.hist.  Returns the number of passes: the result is in `a` when even, in `alt` when odd.
constexpr int kRadix64Tile = 4096;
constexpr int kRadixMaxPasses = 3;
constexpr size_t kRadixGhistWords = kRadixMaxPasses * 2048 + 64;
// 1 when the u64 sort runs single-pass look-back sweeps (SGA_RADIX_MODE=0): the producer of the
// elements then counts every pass's global digit totals into sc.ghist (zeroed first).
int radix64_lookback();
int radix64_digit_bits(int bits);
size_t radix64_tiles(size_t n);
int radix_sort_u64(uint64_t *a, uint64_t *alt, size_t n, int key_shift, int bits, RadixScratch &sc, hipStream_t s,
                   bool hist0_ready);
// Same sort, pass 0 reading a segmented producer buffer: each tile is 4 segments of 1024 slots,
// segment w of tile t holds tile_n0[4 t + w] elements from its start (arrival order);
// dn = total element count on the device.  `src` is only read.  Pass p
// writes `a` when p is even, `alt` when odd: the result is in `a` when the pass count is odd.
int radix_sort_u64_tiled(const uint64_t *src, const uint32_t *tile_n0, const uint32_t *dn, uint64_t *a,
                         uint64_t *alt, size_t n, int key_shift, int bits, RadixScratch &sc, hipStream_t s,
                         bool hist0_ready);

}  // namespace sga
