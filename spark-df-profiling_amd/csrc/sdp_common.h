// sdp_common.h -- device helpers shared by the libsdp kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include "../../include/sdp.h"

namespace sdp {

constexpr int WAVE = 64;
constexpr uint64_t KEY_NAN = 0xFFF8000000000000ull;   // key of the canonical NaN
constexpr uint64_t EMPTY64 = 0xFFFFFFFFFFFFFFFFull;

// ---- error plumbing (sdp_abi.cpp) -------------------------------------------
int set_error(int code, const char *fmt, ...);
int check_launch(const char *what);
bool aligned16(const void *p);

// fp64 min / max of operands that are never NaN: the bare v_min_f64 /
// v_max_f64.  fmin / fmax must quiet signalling NaNs first, so the compiler
// canonicalises every operand it cannot prove canonical (a loop-carried
// accumulator, a loaded value): up to three extra fp64 instructions per use.
__device__ __forceinline__ double dmin_nn(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double dmax_nn(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// ---- order-preserving keys (A.8: NaN above +inf, -0.0 == 0.0) ----------------
__host__ __device__ __forceinline__ uint64_t f64_key(double d) {
    uint64_t b;
    memcpy(&b, &d, 8);
    if (d == 0.0) b = 0;                       // -0.0 groups with 0.0
    if (d != d) b = 0x7FF8000000000000ull;     // one NaN
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
// f64_key of a non-NaN value: -0.0 becomes +0.0 by adding +0.0 (IEEE
// round-to-nearest; the kernels preserve denormals, so no other value
// changes), then the sign flip -- five VALU instead of the zero test's selects
__device__ __forceinline__ uint64_t f64_key_nn(double d) {
    const double z = d + 0.0;
    const uint64_t b = (uint64_t)__double_as_longlong(z);
    const uint64_t m = (uint64_t)((int64_t)b >> 63);
    return b ^ (m | 0x8000000000000000ull);
}
__host__ __device__ __forceinline__ double key_f64(uint64_t k) {
    uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    double d;
    memcpy(&d, &b, 8);
    return d;
}
__host__ __device__ __forceinline__ uint64_t i64_key(int64_t v) {
    return (uint64_t)v ^ 0x8000000000000000ull;
}
__host__ __device__ __forceinline__ int64_t key_i64(uint64_t k) {
    return (int64_t)(k ^ 0x8000000000000000ull);
}

// element traits: how a stored element becomes a double, an int64 and a key
template <typename T> struct Elem;
template <> struct Elem<double> {
    static constexpr bool is_float = true;
    __device__ static double d(double v) { return v; }
    __device__ static int64_t i(double) { return 0; }
    __device__ static uint64_t key(double v) { return f64_key(v); }
    __device__ static uint64_t key_nn(double v) { return f64_key_nn(v); }   // v not NaN
};
template <> struct Elem<float> {
    static constexpr bool is_float = true;
    __device__ static double d(float v) { return (double)v; }
    __device__ static int64_t i(float) { return 0; }
    __device__ static uint64_t key(float v) { return f64_key((double)v); }
    __device__ static uint64_t key_nn(float v) { return f64_key_nn((double)v); }
};
#define SDP_INT_ELEM(T)                                                          \
    template <> struct Elem<T> {                                                 \
        static constexpr bool is_float = false;                                  \
        __device__ static double d(T v) { return (double)(int64_t)v; }           \
        __device__ static int64_t i(T v) { return (int64_t)v; }                  \
        __device__ static uint64_t key(T v) { return i64_key((int64_t)v); }      \
        __device__ static uint64_t key_nn(T v) { return i64_key((int64_t)v); }   \
    };
// 32-bit order-preserving keys of 4-byte types (pass 1's inclusive window
// tests): key32 is monotone in the value and widen(key32) is the element's
// 64-bit key, so for valid (non-NaN) elements key64 < L  <=>  key32 < lower32(L)
// and key64 <= H  <=>  key32 <= upper32(H) (pass1_bounds32 below).
template <typename T> struct Key32 { static constexpr bool ok = false; };
template <> struct Key32<float> {
    static constexpr bool ok = true;
    __device__ static uint32_t key(float v) {            // v not NaN; -0.0 groups with 0.0
        const uint32_t b = v == 0.0f ? 0u : __float_as_uint(v);
        return (b >> 31) ? ~b : (b | 0x80000000u);
    }
    __device__ static uint32_t key_nn(float v) {         // key() by sign flip of v + 0.0f (-0.0 -> +0.0)
        const uint32_t b = __float_as_uint(v + 0.0f);
        const uint32_t m = (uint32_t)((int32_t)b >> 31);
        return b ^ (m | 0x80000000u);
    }
    // 64-bit key of the element with key k; keys below -inf's / above +inf's
    // (NaN patterns, never a valid element's) map to 0 / UINT64_MAX so that the
    // map stays monotone over all of [0, 2^32)
    __device__ static uint64_t widen(uint32_t k) {
        if (k < 0x007FFFFFu) return 0;
        if (k > 0xFF800000u) return EMPTY64;
        return widen_valid(k);
    }
    __device__ static uint64_t widen_valid(uint32_t k) {  // k of a non-NaN value
        const uint32_t b = (k >> 31) ? (k & 0x7FFFFFFFu) : ~k;
        const uint64_t d = (uint64_t)__double_as_longlong((double)__uint_as_float(b));
        return (d >> 63) ? ~d : (d | 0x8000000000000000ull);   // f64_key without the NaN / -0.0 cases
    }
};
template <> struct Key32<int32_t> {
    static constexpr bool ok = true;
    __device__ static uint32_t key(int32_t v) { return (uint32_t)v ^ 0x80000000u; }
    __device__ static uint32_t key_nn(int32_t v) { return key(v); }
    __device__ static uint64_t widen(uint32_t k) { return i64_key((int64_t)(int32_t)(k ^ 0x80000000u)); }
    __device__ static uint64_t widen_valid(uint32_t k) { return widen(k); }
};
template <> struct Key32<uint32_t> {
    static constexpr bool ok = true;
    __device__ static uint32_t key(uint32_t v) { return v; }
    __device__ static uint32_t key_nn(uint32_t v) { return v; }
    __device__ static uint64_t widen(uint32_t k) { return i64_key((int64_t)k); }
    __device__ static uint64_t widen_valid(uint32_t k) { return widen(k); }
};
// smallest k in [0, 2^32) with widen(k) >= L, or 2^32 when there is none (L
// above every 32-bit key's widening); reported apart, since 2^32 - 1 is itself
// a valid key (INT32_MAX, UINT32_MAX)
template <typename T>
__device__ __forceinline__ uint64_t key32_lower(uint64_t L) {
    uint64_t a = 0, b = 0x100000000ull;
    while (a < b) {
        const uint64_t mid = (a + b) >> 1;
        if (Key32<T>::widen((uint32_t)mid) >= L) b = mid; else a = mid + 1;
    }
    return a;
}

SDP_INT_ELEM(int64_t)
SDP_INT_ELEM(int32_t)
SDP_INT_ELEM(int16_t)
SDP_INT_ELEM(int8_t)
SDP_INT_ELEM(uint32_t)
SDP_INT_ELEM(uint16_t)
SDP_INT_ELEM(uint8_t)
#undef SDP_INT_ELEM

// 16-byte vector of T (one global_load_dwordx4 per lane)
template <typename T> struct alignas(16) Vec16 {
    static constexpr int N = 16 / sizeof(T);
    T v[N];
};

// Validity bits [idx, idx+cnt) of an Arrow bitmap (cnt <= 32), LSB = row idx.
__device__ __forceinline__ uint32_t valid_bits(const uint8_t *bm, int64_t bitoff, int64_t idx,
                                               int cnt) {
    // cnt <= 32 bits from bit bitoff + idx, branch-free: two dword loads from
    // the 4-byte-aligned base below bm (bitmaps carry >= 8 bytes of padding;
    // a sliced bitmap's base lies inside its parent) and one alignbit.  A byte
    // loop here put an s_waitcnt vmcnt(0) inside every tile load, which waited
    // for the prefetched next tile as well.
    if (bm == nullptr) return cnt >= 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u);
    // (pointer arithmetic, not an integer round trip, so the loads stay
    // global_load: a pointer rebuilt from an integer becomes a flat load, and
    // every flat result waits for all LDS traffic too)
    const uint32_t mis = (uint32_t)((uintptr_t)bm & 3u);
    const int64_t b = bitoff + idx + (int64_t)mis * 8;
    const uint32_t *wp = (const uint32_t *)(bm - mis) + (b >> 5);
    const uint32_t v = __builtin_amdgcn_alignbit(wp[1], wp[0], (uint32_t)(b & 31));
    return cnt >= 32 ? v : (v & ((1u << cnt) - 1u));
}
// Branch-free streaming of 16-byte vectors with their validity bits.  The
// loads of one vector (values + the two raw validity dwords) are issued with
// no condition (the index is clamped; vectors past the end get zero bits) and
// the bits are decoded only when used, so a tile's loads stay in flight while
// the previous tile is worked on (callers alternate two VecIn sets instead of
// copying one into the other, which would wait for the loads).
struct VBits {
    const uint32_t *base;       // 4-byte aligned base of the bitmap (the values when there is none)
    int64_t bit0;               // bit index of element 0 from base
    bool none;                  // no bitmap: every element valid
};
__device__ __forceinline__ VBits vbits_init(const uint8_t *bm, int64_t bitoff, const void *values) {
    VBits b;
    b.none = bm == nullptr;
    const uint8_t *p = b.none ? (const uint8_t *)values : bm;
    const uint32_t mis = (uint32_t)((uintptr_t)p & 3u);
    b.base = (const uint32_t *)(p - mis);
    b.bit0 = b.none ? 0 : bitoff + (int64_t)mis * 8;
    return b;
}
template <typename T>
struct VecIn {
    static constexpr int VPT = Vec16<T>::N;
    Vec16<T> v;
    uint32_t w0, w1, sh;
    bool in;
    // vector vi of the column (nvec >= 1 whole vectors)
    // (global address space: a column pointer read from a task table in memory
    // is generic, and a flat load also counts against the LDS wait counter)
    __device__ __forceinline__ void load(const Vec16<T> *vals, const VBits &vb, int64_t vi, int64_t nvec) {
        in = vi < nvec;
        const int64_t vc = in ? vi : 0;
        typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));
        const u32x4g raw = ((const __attribute__((address_space(1))) u32x4g *)vals)[vc];
        __builtin_memcpy(&v, &raw, 16);
        const int64_t b = vb.none ? 0 : vb.bit0 + vc * VPT;
        const __attribute__((address_space(1))) uint32_t *wp =
            (const __attribute__((address_space(1))) uint32_t *)vb.base + (b >> 5);
        w0 = wp[0];
        w1 = wp[1];
        sh = (uint32_t)(b & 31);
    }
    __device__ __forceinline__ uint32_t bits(const VBits &vb) const {
        constexpr uint32_t full = VPT >= 32 ? 0xFFFFFFFFu : ((1u << VPT) - 1u);
        const uint32_t x = vb.none ? full : (__builtin_amdgcn_alignbit(w1, w0, sh) & full);
        return in ? x : 0u;
    }
    // bits() without a branch on vb.none (a branch between a load and its use
    // made the compiler wait vmcnt(0) there, draining the prefetched next
    // tile; pass 1 -- in pass 2 the extra live words spilled)
    __device__ __forceinline__ uint32_t bits_nb(const VBits &vb) const {
        constexpr uint32_t full = VPT >= 32 ? 0xFFFFFFFFu : ((1u << VPT) - 1u);
        const uint32_t x = (__builtin_amdgcn_alignbit(w1, w0, sh) | (vb.none ? 0xFFFFFFFFu : 0u)) & full;
        return in ? x : 0u;
    }
};

__device__ __forceinline__ bool valid_bit(const uint8_t *bm, int64_t bitoff, int64_t idx) {
    if (bm == nullptr) return true;
    const int64_t b = bitoff + idx;
    return (bm[b >> 3] >> (b & 7)) & 1;
}

// ---- compensated summation (TwoSum) -----------------------------------------
__device__ __forceinline__ void two_sum_acc(double &s, double &c, double x) {
    const double t = s + x;
    const double bp = t - s;
    c += (s - (t - bp)) + (x - bp);
    s = t;
}
__device__ __forceinline__ void dd_add(double &ah, double &al, double bh, double bl) {
    double s = ah + bh;
    double bp = s - ah;
    double e = (ah - (s - bp)) + (bh - bp);
    e += al + bl;
    ah = s + e;
    al = e - (ah - s);
}

// ---- wave reductions (64 lanes, DPP/shuffle via __shfl_xor) ------------------
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ __forceinline__ void wave_sum_dd(double &h, double &l) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        double oh = __shfl_xor(h, o, WAVE), ol = __shfl_xor(l, o, WAVE);
        dd_add(h, l, oh, ol);
    }
}
__device__ __forceinline__ double wave_min_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, WAVE));
    return v;
}
__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, WAVE));
    return v;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { int64_t w = __shfl_xor(v, o, WAVE); v = w < v ? w : v; }
    return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { int64_t w = __shfl_xor(v, o, WAVE); v = w > v ? w : v; }
    return v;
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
    return (int64_t)wave_sum_u64((uint64_t)v);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (WAVE - 1); }

// Wave-uniform copies of lane values (lane 0's / the first active lane's).
// __builtin_amdgcn_readfirstlane returns int: widened straight to 64 bits it
// sign-extends, so a word >= 2^31 turned a rebuilt 64-bit pointer into garbage
// (the round-6 illegal accesses of the block-layout dedup and of pass 1's
// candidate slots).  Every use goes through these helpers
// (tests/test_sources_cpu.py checks that).
__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    return ((uint64_t)uniform_u32((uint32_t)(v >> 32)) << 32) | (uint64_t)uniform_u32((uint32_t)v);
}
template <typename P> __device__ __forceinline__ P *uniform_ptr(P *p) { return (P *)uniform_u64((uint64_t)p); }
// Workgroup barrier for LDS hand-offs only.  __syncthreads() carries a
// workgroup release/acquire fence, which drains vmcnt: every global load still
// in flight (a prefetched next tile) would be waited for at the barrier.  This
// waits for this wave's LDS operations only, so prefetches keep flying.  Use it
// only where the barrier orders LDS accesses, never global memory.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// number of set bits of `mask` below this lane
__device__ __forceinline__ int lane_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// 64-bit mixer: fold, one odd multiply, fold -- a bijection, so a record (the
// mix of a fixed-width key) is equal to another exactly when the keys are.
// Round 5: splitmix64's finalizer (two 64-bit multiplies, i.e. eight
// quarter-rate 32-bit multiplies per key) cost 1.9 of 17.0 ms in the pass-2 +
// level-1 count of six 1e9-row f64 columns (profiles/r05q_*); this form
// spreads structured keys (sequences, strides, small integers as doubles) over
// the level-1 / level-2 buckets and table slots at least as evenly, and random
// keys the same (tools/mixer_quality.py).
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 32;
    x *= 0xD6E8FEB86659FD93ull;
    x ^= x >> 32;
    return x;
}
// its inverse: a fixed key from its record
__host__ __device__ __forceinline__ uint64_t inv_mix64(uint64_t x) {
    x ^= x >> 32;
    x *= 0xCFEE444D8B59A89Bull;
    x ^= x >> 32;
    return x;
}

// Spark comparisons on doubles with NaN ordered above every number (A.8)
__device__ __forceinline__ bool spark_lt(double x, double t) {
    return (t != t) ? (x == x) : (x == x && x < t);
}
__device__ __forceinline__ bool spark_gt(double x, double t) {
    return (t != t) ? false : (x != x || x > t);
}
__device__ __forceinline__ bool spark_ge(double x, double t) { return !spark_lt(x, t); }

}  // namespace sdp
