// Shared helpers for the MI355X admission engine (gfx950, HIP).
// Java numeric semantics are restated here for device code (independently of
// the oracle): JLS 5.1.3 narrowing casts, Math.round, Math.nextUp.
// All translation units are compiled with -ffp-contract=off so double
// expressions round exactly like the JVM (no FMA contraction).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#define SGA_HD __host__ __device__ __forceinline__

namespace sga {

constexpr int64_t kAbsent = INT64_MIN;  // "array.get(idx) == null" for a window slot

SGA_HD int32_t j_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d;
}

SGA_HD int64_t j_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

// Math.round(double): nearest long, ties toward +infinity, NaN -> 0, saturating.
SGA_HD int64_t j_round(double a) {
    uint64_t bits = (uint64_t)__builtin_bit_cast(int64_t, a);
    int64_t biased_exp = (int64_t)((bits & 0x7FF0000000000000ULL) >> 52);
    int64_t shift = 1074 - biased_exp;
    if (shift >= 0 && shift < 64) {
        int64_t r = (int64_t)((bits & 0x000FFFFFFFFFFFFFULL) | 0x0010000000000000ULL);
        if ((int64_t)bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    if (shift >= 64) return 0;
    return j_d2l(a);
}

// Math.nextUp(double)
SGA_HD double j_next_up(double d) {
    if (d != d) return d;
    int64_t b = __builtin_bit_cast(int64_t, d);
    if (b == 0x7FF0000000000000LL) return d;  // +inf
    if (d == 0.0) return __builtin_bit_cast(double, (int64_t)1);  // +MIN_VALUE for +0/-0
    b += (b >= 0) ? 1 : -1;
    return __builtin_bit_cast(double, b);
}

SGA_HD uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

SGA_HD uint64_t hash_flow_id(int64_t id) { return splitmix64((uint64_t)id ^ 0x5EB7F00DULL); }

}  // namespace sga

struct sga_error_sink {
    std::string msg;
};

#define SGA_HIP_CHECK(expr)                                                                        \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) {                                                                    \
            throw sga::HipError(std::string(#expr) + ": " + hipGetErrorString(_e), __FILE__, __LINE__); \
        }                                                                                          \
    } while (0)

namespace sga {
struct HipError {
    std::string what;
    HipError(std::string w, const char *f, int l) : what(std::move(w) + " @" + f + ":" + std::to_string(l)) {}
};

// Minimal owning device buffer.
// Page-locked host staging (one DMA per direction for small batches).
struct PinnedBuf {
    uint8_t *p = nullptr;
    size_t n = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf &) = delete;
    PinnedBuf &operator=(const PinnedBuf &) = delete;
    ~PinnedBuf() { release(); }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t bytes) {
        release();
        SGA_HIP_CHECK(hipHostMalloc((void **)&p, bytes, hipHostMallocDefault));
        n = bytes;
    }
};

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        release();
        if (count == 0) return;
        SGA_HIP_CHECK(hipMalloc((void **)&p, count * sizeof(T)));
        n = count;
    }
    // grow preserving contents (stream-ordered copy); fill is done by caller
    void grow(size_t count, hipStream_t s) {
        if (count <= n) return;
        T *q = nullptr;
        SGA_HIP_CHECK(hipMalloc((void **)&q, count * sizeof(T)));
        if (p && n) SGA_HIP_CHECK(hipMemcpyAsync(q, p, n * sizeof(T), hipMemcpyDeviceToDevice, s));
        SGA_HIP_CHECK(hipStreamSynchronize(s));
        if (p) (void)hipFree(p);
        p = q;
        n = count;
    }
    size_t bytes() const { return n * sizeof(T); }
};
// ---- wave64 scans on DPP (VALU lane moves: no LDS round trip per step, unlike __shfl_up).
// Hillis-Steele inside each 16-lane row (row_shr 1, 2, 4, 8), then row 0's / row 2's totals into
// rows 1 / 3 (row_bcast:15) and the first half's total into rows 2 and 3 (row_bcast:31).  Lanes whose
// source is outside the row, or whose row is masked off, read `old` = the identity.
namespace dpp {
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int64_t mov64(int64_t old, int64_t v) {
    const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)old, (int)(uint32_t)v, kCtrl, kRowMask, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)((uint64_t)old >> 32), (int)(uint32_t)((uint64_t)v >> 32),
                                               kCtrl, kRowMask, 0xf, false);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
}  // namespace dpp

namespace dpp {
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int mov32(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, kCtrl, kRowMask, 0xf, false);
}
}  // namespace dpp

// inclusive prefix max / min of an int64 over the wave (lane order)
__device__ __forceinline__ int64_t wave_incl_max_i64(int64_t v) {
    v = max(v, dpp::mov64<0x111, 0xf>(INT64_MIN, v));
    v = max(v, dpp::mov64<0x112, 0xf>(INT64_MIN, v));
    v = max(v, dpp::mov64<0x114, 0xf>(INT64_MIN, v));
    v = max(v, dpp::mov64<0x118, 0xf>(INT64_MIN, v));
    v = max(v, dpp::mov64<0x142, 0xa>(INT64_MIN, v));
    v = max(v, dpp::mov64<0x143, 0xc>(INT64_MIN, v));
    return v;
}
__device__ __forceinline__ int64_t wave_incl_min_i64(int64_t v) {
    v = min(v, dpp::mov64<0x111, 0xf>(INT64_MAX, v));
    v = min(v, dpp::mov64<0x112, 0xf>(INT64_MAX, v));
    v = min(v, dpp::mov64<0x114, 0xf>(INT64_MAX, v));
    v = min(v, dpp::mov64<0x118, 0xf>(INT64_MAX, v));
    v = min(v, dpp::mov64<0x142, 0xa>(INT64_MAX, v));
    v = min(v, dpp::mov64<0x143, 0xc>(INT64_MAX, v));
    return v;
}

// segmented inclusive sum of two int32 counters (a head flag starts a new segment at its lane)
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void segsum2_step(int &a, int &b, int &hd) {
    const int ya = dpp::mov32<kCtrl, kRowMask>(0, a), yb = dpp::mov32<kCtrl, kRowMask>(0, b);
    const int yh = dpp::mov32<kCtrl, kRowMask>(0, hd);
    if (!hd) {
        a += ya;
        b += yb;
    }
    hd |= yh;
}
__device__ __forceinline__ void wave_incl_segsum2(int &a, int &b, int &hd) {
    segsum2_step<0x111, 0xf>(a, b, hd);
    segsum2_step<0x112, 0xf>(a, b, hd);
    segsum2_step<0x114, 0xf>(a, b, hd);
    segsum2_step<0x118, 0xf>(a, b, hd);
    segsum2_step<0x142, 0xa>(a, b, hd);
    segsum2_step<0x143, 0xc>(a, b, hd);
}

// whole-wave reductions through DPP row shifts and row broadcasts (no LDS permutes): the inclusive scan's
// lane 63, read as a wave-uniform value.  Every lane of the wave must be active.
template <class Op>
__device__ __forceinline__ uint32_t wave_reduce_u32(uint32_t v, uint32_t id, Op op) {
    int x = (int)v;
    x = (int)op((uint32_t)x, (uint32_t)dpp::mov32<0x111, 0xf>((int)id, x));
    x = (int)op((uint32_t)x, (uint32_t)dpp::mov32<0x112, 0xf>((int)id, x));
    x = (int)op((uint32_t)x, (uint32_t)dpp::mov32<0x114, 0xf>((int)id, x));
    x = (int)op((uint32_t)x, (uint32_t)dpp::mov32<0x118, 0xf>((int)id, x));
    x = (int)op((uint32_t)x, (uint32_t)dpp::mov32<0x142, 0xa>((int)id, x));
    x = (int)op((uint32_t)x, (uint32_t)dpp::mov32<0x143, 0xc>((int)id, x));
    return (uint32_t)__builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    return wave_reduce_u32(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return wave_reduce_u32(v, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
    return wave_reduce_u32(v, 0u, [](uint32_t a, uint32_t b) { return a | b; });
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    return wave_reduce_u32(v, 0xFFFFFFFFu, [](uint32_t a, uint32_t b) { return a < b ? a : b; });
}

// inclusive prefix sum of an int64 over the wave (lane order)
__device__ __forceinline__ int64_t wave_incl_sum_i64(int64_t v) {
    v += dpp::mov64<0x111, 0xf>(0, v);
    v += dpp::mov64<0x112, 0xf>(0, v);
    v += dpp::mov64<0x114, 0xf>(0, v);
    v += dpp::mov64<0x118, 0xf>(0, v);
    v += dpp::mov64<0x142, 0xa>(0, v);
    v += dpp::mov64<0x143, 0xc>(0, v);
    return v;
}

// inclusive max-plus scan: lane k ends with the composition of f_0 .. f_k, f_i(x) = max(x + A_i, B_i);
// (A1, B1) then (A2, B2) = (A1 + A2, max(B1 + A2, B2)); identity (0, kNegInf)
constexpr int64_t kMaxPlusNegInf = INT64_MIN / 4;
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void maxplus_step(int64_t &A, int64_t &B) {
    const int64_t a = dpp::mov64<kCtrl, kRowMask>(0, A), b = dpp::mov64<kCtrl, kRowMask>(kMaxPlusNegInf, B);
    B = max(b + A, B);
    A += a;
}
__device__ __forceinline__ void wave_incl_maxplus(int64_t &A, int64_t &B) {
    maxplus_step<0x111, 0xf>(A, B);
    maxplus_step<0x112, 0xf>(A, B);
    maxplus_step<0x114, 0xf>(A, B);
    maxplus_step<0x118, 0xf>(A, B);
    maxplus_step<0x142, 0xa>(A, B);
    maxplus_step<0x143, 0xc>(A, B);
}

// lane i <- lane i - 1 (lane 0 <- fill), whole wave (wave_shr:1)
__device__ __forceinline__ int64_t wave_shr1_i64(int64_t v, int64_t fill) { return dpp::mov64<0x138, 0xf>(fill, v); }

// one lane's value, wave-uniform (v_readlane)
__device__ __forceinline__ int64_t readlane_i64(int64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// whole-wave int64 sum / max / min (DPP scan, lane 63); every lane of the wave must be active
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) { return readlane_i64(wave_incl_sum_i64(v), 63); }
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) { return readlane_i64(wave_incl_max_i64(v), 63); }
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) { return readlane_i64(wave_incl_min_i64(v), 63); }
}  // namespace sga
