// sdp_heavy.h -- heavy-key LDS tables and the fixed-width grouping key, shared by
// the partitioning kernels (sdp_part.hip) and the fused pass-2 + level-1 count
// kernel (sdp_numeric.hip).  Keys seen >= HEAVY_MIN times in the pre-pass
// sample are counted in an LDS table and never become partition records, so
// skewed columns (describe.py:251's hot groups) cannot pile into one bucket.
#pragma once
#include <type_traits>
#include "sdp_common.h"

namespace sdp {

constexpr int MAXB = 1024;              // buckets per level (b <= 10)
constexpr int HEAVY_MAX = SDP_HEAVY_MAX;
// the byte records kernel (one workgroup per CU, 110 KB of LDS) holds more:
// on a zipf(1.1) string column over 1e8 labels the top 1024 keys cover ~62 %
// of the rows against ~54 % for the top 256, and every heavy row is one
// 24-byte record fewer through both scatters and the de-duplication
constexpr int HEAVY_MAX_REC = SDP_HEAVY_MAX_REC;
// open-addressing slots: load <= 1/4 at 256 keys, <= 1/2 at 1024
template <int MAXK>
constexpr int heavy_slots() { return MAXK <= 256 ? 1024 : 2 * MAXK; }
constexpr int HEAVY_SLOTS = heavy_slots<HEAVY_MAX>();
constexpr int HEAVY_FILTER = 16384;     // filter bits: most non-heavy rows need one LDS read
constexpr int SHORT_MAX = 16;

// ---- heavy keys ---------------------------------------------------------------
struct HeavyArg {
    const uint64_t *h;      // [n] hashes (fixed: h = mix64(key))
    const uint64_t *k0;     // bytes only
    const uint64_t *k1;
    const uint64_t *meta;
    int32_t n;
};
// (byte keys also keep each heavy key's first 16 bytes and length)
template <bool BYTES, int MAXK = HEAVY_MAX>
struct HeavyLdsT {
    static constexpr int MAX = MAXK;
    static constexpr int SLOTS = heavy_slots<MAXK>();
    uint64_t h[SLOTS];
    uint32_t filter[HEAVY_FILTER / 32];
    int16_t idx[SLOTS];
    uint32_t cnt[MAXK];
    uint64_t k0[BYTES ? MAXK : 1];
    uint64_t k1[BYTES ? MAXK : 1];
    uint32_t len[BYTES ? MAXK : 1];
};
// filter bit of a hash: bits 20..33 (the slot uses the low bits, buckets the top)
__device__ __forceinline__ uint32_t heavy_filter_bit(uint64_t h) { return (uint32_t)(h >> 20) & (HEAVY_FILTER - 1); }
template <bool BYTES, int MAXK>
__device__ __forceinline__ bool heavy_maybe(const HeavyLdsT<BYTES, MAXK> &s, uint64_t h) {
    const uint32_t fb = heavy_filter_bit(h);
    return (s.filter[fb >> 5] >> (fb & 31)) & 1u;
}
template <bool BYTES, int MAXK>
__device__ void heavy_build(HeavyLdsT<BYTES, MAXK> &s, const HeavyArg &a) {
    constexpr int SLOTS = HeavyLdsT<BYTES, MAXK>::SLOTS;
    for (int i = threadIdx.x; i < SLOTS; i += blockDim.x) s.h[i] = EMPTY64;
    for (int i = threadIdx.x; i < MAXK; i += blockDim.x) s.cnt[i] = 0;
    for (int i = threadIdx.x; i < HEAVY_FILTER / 32; i += blockDim.x) s.filter[i] = 0;
    lds_barrier();
    for (int i = threadIdx.x; i < a.n; i += blockDim.x) {
        const uint64_t h = a.h[i];
        const uint32_t fb = heavy_filter_bit(h);
        atomicOr(&s.filter[fb >> 5], 1u << (fb & 31));
        uint32_t pos = (uint32_t)h & (SLOTS - 1);
        while (true) {
            const uint64_t old = atomicCAS((unsigned long long *)&s.h[pos], (unsigned long long)EMPTY64,
                                           (unsigned long long)h);
            if (old == EMPTY64) { s.idx[pos] = (int16_t)i; break; }
            pos = (pos + 1) & (SLOTS - 1);
        }
        if constexpr (BYTES) {
            s.k0[i] = a.k0[i];
            s.k1[i] = a.k1[i];
            s.len[i] = (uint32_t)(a.meta[i] >> 40);
        }
    }
    lds_barrier();
}
// index of the heavy key equal to this row, or -1
__device__ __forceinline__ int heavy_find_u64(const HeavyLdsT<false> &s, int n, uint64_t h) {
    if (n == 0 || h == EMPTY64 || !heavy_maybe(s, h)) return -1;
    uint32_t pos = (uint32_t)h & (HEAVY_SLOTS - 1);
    while (true) {
        const uint64_t v = s.h[pos];
        if (v == h) return s.idx[pos];
        if (v == EMPTY64) return -1;
        pos = (pos + 1) & (HEAVY_SLOTS - 1);
    }
}
template <int MAXK>
__device__ __forceinline__ int heavy_find_bytes(const HeavyLdsT<true, MAXK> &s, int n, uint64_t h, uint64_t k0,
                                                uint64_t k1, uint32_t len) {
    constexpr int SLOTS = HeavyLdsT<true, MAXK>::SLOTS;
    if (n == 0 || len > SHORT_MAX || h == EMPTY64 || !heavy_maybe(s, h)) return -1;
    uint32_t pos = (uint32_t)h & (SLOTS - 1);
    while (true) {
        const uint64_t v = s.h[pos];
        if (v == EMPTY64) return -1;
        if (v == h) {
            const int i = s.idx[pos];
            if (s.k0[i] == k0 && s.k1[i] == k1 && s.len[i] == len) return i;
        }
        pos = (pos + 1) & (SLOTS - 1);
    }
}
// one device atomic per workgroup (not per wave) for a block total
__device__ void block_add_u64(uint64_t v, uint64_t *dst) {
    __shared__ uint64_t s_part[1024 / WAVE];
    lds_barrier();                      // a previous call's reads of s_part are done
    v = wave_sum_u64(v);
    if (lane_id() == 0) s_part[threadIdx.x / WAVE] = v;
    lds_barrier();
    if (threadIdx.x == 0) {
        uint64_t tot = 0;
        for (int w = 0; w < (int)(blockDim.x / WAVE); ++w) tot += s_part[w];
        if (tot) atomicAdd((unsigned long long *)dst, (unsigned long long)tot);
    }
}
// Byte heavy keys of the records kernel (round 5): a slot holds the key's
// hash, first 16 bytes, length and index, so one probe is one pair of 16-byte
// LDS reads instead of the chain hash -> index -> key bytes, and the rows of a
// lane are probed together (filter words, then first probes, each a batch of
// independent reads; further probes only in a wave that needs one).  With the
// chained form the heavy lookup took 3.9 of 11.6 ms of the records kernel on
// a 1e8-label column (profiles/r05ai_*: the kernel without it, writing every
// row as a record, ran 7.7 ms).
struct HeavySlot {
    uint64_t h, k0, k1;
    uint32_t len;
    int32_t idx;
};
template <int MAXK>
struct HeavyRecT {
    static constexpr int SLOTS = heavy_slots<MAXK>();
    HeavySlot slot[SLOTS];
    uint32_t filter[HEAVY_FILTER / 32];
    uint32_t cnt[MAXK];
};
template <int MAXK>
__device__ void heavy_rec_build(HeavyRecT<MAXK> &s, const HeavyArg &a) {
    constexpr int SLOTS = HeavyRecT<MAXK>::SLOTS;
    for (int i = threadIdx.x; i < SLOTS; i += blockDim.x) s.slot[i].h = EMPTY64;
    for (int i = threadIdx.x; i < MAXK; i += blockDim.x) s.cnt[i] = 0;
    for (int i = threadIdx.x; i < HEAVY_FILTER / 32; i += blockDim.x) s.filter[i] = 0;
    lds_barrier();
    for (int i = threadIdx.x; i < a.n; i += blockDim.x) {
        const uint64_t h = a.h[i];
        const uint32_t fb = heavy_filter_bit(h);
        atomicOr(&s.filter[fb >> 5], 1u << (fb & 31));
        uint32_t pos = (uint32_t)h & (SLOTS - 1);
        while (true) {
            const uint64_t old = atomicCAS((unsigned long long *)&s.slot[pos].h, (unsigned long long)EMPTY64,
                                           (unsigned long long)h);
            if (old == EMPTY64) break;
            pos = (pos + 1) & (SLOTS - 1);
        }
        s.slot[pos].k0 = a.k0[i];
        s.slot[pos].k1 = a.k1[i];
        s.slot[pos].len = (uint32_t)(a.meta[i] >> 40);
        s.slot[pos].idx = i;
    }
    lds_barrier();
}
// heavy index of each of a lane's RPT rows (bit q of vmask: row q valid), or -1
template <int MAXK, int RPT>
__device__ __forceinline__ void heavy_rec_find(const HeavyRecT<MAXK> &s, int n, const uint64_t (&h)[RPT],
                                               const uint64_t (&k0)[RPT], const uint64_t (&k1)[RPT],
                                               const uint64_t (&meta)[RPT], uint32_t vmask, int (&hv)[RPT]) {
    constexpr int SLOTS = HeavyRecT<MAXK>::SLOTS;
#pragma unroll
    for (int q = 0; q < RPT; ++q) hv[q] = -1;
    if (n == 0) return;                                // (uniform)
    uint32_t maybe = 0;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const uint32_t fb = heavy_filter_bit(h[q]);
        const uint32_t fw = s.filter[fb >> 5];
        const bool c = ((vmask >> q) & 1u) && (uint32_t)(meta[q] >> 40) <= (uint32_t)SHORT_MAX && h[q] != EMPTY64;
        maybe |= (uint32_t)(c && ((fw >> (fb & 31)) & 1u)) << q;
    }
    uint32_t more = 0;
    uint32_t pos[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        pos[q] = (uint32_t)h[q] & (SLOTS - 1);
        const HeavySlot sl = s.slot[pos[q]];           // every lane reads (no branch); masked below
        const bool m = (maybe >> q) & 1u;
        const bool eq = sl.h == h[q] && sl.k0 == k0[q] && sl.k1 == k1[q] && sl.len == (uint32_t)(meta[q] >> 40);
        if (m && eq) hv[q] = sl.idx;
        more |= (uint32_t)(m && !eq && sl.h != EMPTY64) << q;
    }
    while (__ballot(more != 0)) {                      // rare: further probes
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            if ((more >> q) & 1u) {
                pos[q] = (pos[q] + 1) & (SLOTS - 1);
                const HeavySlot sl = s.slot[pos[q]];
                if (sl.h == h[q] && sl.k0 == k0[q] && sl.k1 == k1[q] && sl.len == (uint32_t)(meta[q] >> 40)) {
                    hv[q] = sl.idx;
                    more &= ~(1u << q);
                } else if (sl.h == EMPTY64) {
                    more &= ~(1u << q);
                }
            }
        }
    }
}
template <int MAXK>
__device__ void heavy_rec_flush(HeavyRecT<MAXK> &s, int n, uint64_t *counts) {
    lds_barrier();
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (s.cnt[i]) atomicAdd((unsigned long long *)&counts[i], (unsigned long long)s.cnt[i]);
}
template <bool BYTES, int MAXK>
__device__ void heavy_flush(HeavyLdsT<BYTES, MAXK> &s, int n, uint64_t *counts) {
    lds_barrier();
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        if (s.cnt[i]) atomicAdd((unsigned long long *)&counts[i], (unsigned long long)s.cnt[i]);
}

// ---- 32-bit key spaces (sdp_distinct32; its level-1 count rides pass 2) -------
// float32: the order-preserving 32-bit key (NaN one value, -0.0 == 0.0);
// integral columns with imax - imin < 2^32: v - lo.  h = mix32(key) is a
// bijection of [0, 2^32); its top D32_B1 bits pick the level-1 bucket.
constexpr int D32_B1 = 6;
constexpr int D32_NB1 = 1 << D32_B1;
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}
template <typename T>
__device__ __forceinline__ uint32_t key32_rel(T v, int64_t lo) {
    if constexpr (std::is_same<T, float>::value) return v != v ? 0xFFC00000u : Key32<float>::key(v);
    else if constexpr (std::is_same<T, double>::value) return 0u;             // (never a 32-bit key space)
    else return (uint32_t)(uint64_t)((int64_t)v - lo);
}

// ---- grouping key of a fixed-width element (order-preserving u64) ----------
template <typename T> __device__ __forceinline__ uint64_t key_of(T v);
template <> __device__ __forceinline__ uint64_t key_of<double>(double v) { return f64_key(v); }
template <> __device__ __forceinline__ uint64_t key_of<float>(float v) { return f64_key((double)v); }
template <> __device__ __forceinline__ uint64_t key_of<int64_t>(int64_t v) { return i64_key(v); }
template <> __device__ __forceinline__ uint64_t key_of<int32_t>(int32_t v) { return i64_key(v); }
template <> __device__ __forceinline__ uint64_t key_of<int16_t>(int16_t v) { return i64_key(v); }
template <> __device__ __forceinline__ uint64_t key_of<int8_t>(int8_t v) { return i64_key(v); }
template <> __device__ __forceinline__ uint64_t key_of<uint64_t>(uint64_t v) { return v; }
template <> __device__ __forceinline__ uint64_t key_of<uint32_t>(uint32_t v) { return v; }
template <> __device__ __forceinline__ uint64_t key_of<uint16_t>(uint16_t v) { return v; }
template <> __device__ __forceinline__ uint64_t key_of<uint8_t>(uint8_t v) { return v; }

}  // namespace sdp
