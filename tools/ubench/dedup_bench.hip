// Microbenchmark: final-bucket dedup variants on synthetic hash-partitioned
// records (all keys distinct, ~3.6 K records per bucket, 2^18 buckets).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 dedup_bench.hip -o dedup_bench -L../../spark-df-profiling_amd/spark_df_profiling/lib -lsdp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../../include/sdp.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 31; return x;
}
constexpr uint64_t EMPTY = ~0ull;

__global__ void gen(uint64_t *rec, const uint64_t *starts, int64_t nb, int bits) {
    int64_t f = blockIdx.x;
    if (f >= nb) return;
    for (int64_t r = starts[f] + threadIdx.x; r < starts[f + 1]; r += blockDim.x)
        rec[r] = ((uint64_t)f << (64 - bits)) | (mix64((uint64_t)r * 2654435761ull + 17) >> bits);
}

__global__ void sum_kernel(const uint64_t *rec, int64_t n, uint64_t *out) {
    uint64_t s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s ^= rec[i];
    if (s == 0x123) out[0] = s;
}

// V4: LDS counting partition of the bucket into 512 sub-buckets by low hash
// bits, then each thread counts distinct keys of its sub-bucket (O(k^2)).
constexpr int VT = 512;
constexpr int VCAP = 8192;
constexpr int VB = 8;            // records per thread per batch (<= VCAP/VT = 16)
__global__ void __launch_bounds__(VT) dedup_sub(const uint64_t *in, const uint64_t *starts, int64_t nb, uint64_t *out) {
    __shared__ uint64_t keys[VCAP];
    __shared__ uint32_t cnt[VT];
    __shared__ uint32_t off[VT];
    __shared__ uint32_t wsum[VT / 64];
    const int t = threadIdx.x;
    uint64_t total = 0;
    for (int64_t f = blockIdx.x; f < nb; f += gridDim.x) {
        const int64_t lo = starts[f], hi = starts[f + 1];
        const int m = (int)(hi - lo);
        cnt[t] = 0;
        uint64_t h[16];
        uint32_t rk[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int i = q * VT + t;
            h[q] = i < m ? in[lo + i] : EMPTY;
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (q * VT + t < m) rk[q] = atomicAdd(&cnt[(uint32_t)h[q] & (VT - 1)], 1u);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // exclusive scan of cnt (one entry per thread)
        uint32_t v = cnt[t], x = v;
        const int lane = t & 63;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) { uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
        if (lane == 63) wsum[t / 64] = x;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint32_t wb = 0;
        for (int k = 0; k < t / 64; ++k) wb += wsum[k];
        off[t] = wb + x - v;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (q * VT + t < m) keys[off[(uint32_t)h[q] & (VT - 1)] + rk[q]] = h[q];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const uint32_t b0 = off[t], k = cnt[t];
        uint32_t fresh = 0;
        for (uint32_t i = 0; i < k; ++i) {
            const uint64_t a = keys[b0 + i];
            bool dup = false;
            for (uint32_t j = 0; j < i; ++j) dup |= keys[b0 + j] == a;
            fresh += !dup;
        }
        total += fresh;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    if ((t & 63) == 0 && total) atomicAdd((unsigned long long *)out, (unsigned long long)total);
}

// V7: 4 sub-buckets per thread (2048 per bucket, ~1.8 keys each); PF: the next
// bucket's records are loaded while this one is processed.
constexpr int NS = 2048;
template <bool PF>
__global__ void __launch_bounds__(VT) dedup_sub4(const uint64_t *in, const uint64_t *starts, int64_t nb, uint64_t *out) {
    __shared__ uint64_t keys[VCAP];
    __shared__ uint32_t cnt[NS];
    __shared__ uint32_t off[NS];
    __shared__ uint32_t wsum[VT / 64];
    const int t = threadIdx.x;
    uint64_t total = 0;
    constexpr int Q = 8;
    uint64_t h[Q], hn[Q];
    int64_t f = blockIdx.x;
    int64_t lo = 0, hi = 0;
    if (f < nb) {
        lo = starts[f]; hi = starts[f + 1];
#pragma unroll
        for (int q = 0; q < Q; ++q) { const int64_t i = lo + q * VT + t; h[q] = i < hi ? in[i] : EMPTY; }
    }
    for (; f < nb; f += gridDim.x) {
        const int m = (int)(hi - lo);
        const int64_t fn = f + gridDim.x;
        int64_t lo_n = 0, hi_n = 0;
        if (PF && fn < nb) {
            lo_n = starts[fn]; hi_n = starts[fn + 1];
#pragma unroll
            for (int q = 0; q < Q; ++q) { const int64_t i = lo_n + q * VT + t; hn[q] = i < hi_n ? in[i] : EMPTY; }
        }
#pragma unroll
        for (int k = 0; k < NS / VT; ++k) cnt[k * VT + t] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint32_t rk[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (q * VT + t < m) rk[q] = atomicAdd(&cnt[(uint32_t)h[q] & (NS - 1)], 1u);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // exclusive scan of cnt: thread t owns entries 4t..4t+3
        uint32_t c4[4], sum = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) { c4[k] = cnt[4 * t + k]; sum += c4[k]; }
        uint32_t x = sum;
        const int lane = t & 63;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) { uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
        if (lane == 63) wsum[t / 64] = x;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint32_t run = x - sum;
        for (int k = 0; k < t / 64; ++k) run += wsum[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) { off[4 * t + k] = run; run += c4[k]; }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (q * VT + t < m) keys[off[(uint32_t)h[q] & (NS - 1)] + rk[q]] = h[q];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint32_t fresh = 0;
        const uint32_t base = off[4 * t];
        uint32_t kk[4];
        kk[0] = c4[0]; kk[1] = c4[1]; kk[2] = c4[2]; kk[3] = c4[3];
        uint32_t b = base;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            for (uint32_t i = 0; i < kk[s4]; ++i) {
                const uint64_t a = keys[b + i];
                bool dup = false;
                for (uint32_t j = 0; j < i; ++j) dup |= keys[b + j] == a;
                fresh += !dup;
            }
            b += kk[s4];
        }
        total += fresh;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (PF) {
            lo = lo_n; hi = hi_n;
#pragma unroll
            for (int q = 0; q < Q; ++q) h[q] = hn[q];
        } else if (fn < nb) {
            lo = starts[fn]; hi = starts[fn + 1];
#pragma unroll
            for (int q = 0; q < Q; ++q) { const int64_t i = lo + q * VT + t; h[q] = i < hi ? in[i] : EMPTY; }
        }
    }
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    if ((t & 63) == 0 && total) atomicAdd((unsigned long long *)out, (unsigned long long)total);
}

// V9: counting sort of the bucket into 4096 sub-buckets (low 12 bits; ~0.9
// keys each) in LDS, then each thread compares keys only inside its 8
// contiguous sub-buckets.  64 KB of LDS -> 2 workgroups per CU.
constexpr int NS9 = 4096;
constexpr int CAP9 = 6144;
template <int T9>
__global__ void __launch_bounds__(T9) dedup_v9(const uint64_t *in, const uint64_t *starts, int64_t nb, uint64_t *out,
                                            uint64_t *skipped) {
    constexpr int PER = NS9 / T9;            // sub-buckets per thread
    constexpr int Q = CAP9 / T9;             // records per thread
    __shared__ uint64_t keys[CAP9];
    __shared__ __attribute__((aligned(16))) uint32_t cnt[NS9];
    __shared__ uint32_t wsum[T9 / 64];
    const int t = threadIdx.x;
    uint64_t total = 0, skip = 0;
    for (int64_t f = blockIdx.x; f < nb; f += gridDim.x) {
        const int64_t lo = starts[f], hi = starts[f + 1];
        const int m = (int)(hi - lo);
        if (m > CAP9) { if (t == 0) ++skip; continue; }
        uint64_t h[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) { const int i = q * T9 + t; h[q] = i < m ? in[lo + i] : EMPTY; }
#pragma unroll
        for (int k = 0; k < PER; ++k) cnt[t * PER + k] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint32_t rk[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (q * T9 + t < m) rk[q] = atomicAdd(&cnt[(uint32_t)h[q] & (NS9 - 1)], 1u);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint32_t c[PER], sum = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) { c[k] = cnt[t * PER + k]; sum += c[k]; }
        uint32_t x = sum;
        const int lane = t & 63;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) { uint32_t y = __shfl_up(x, o, 64); if (lane >= o) x += y; }
        if (lane == 63) wsum[t / 64] = x;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint32_t run = x - sum;
        for (int k = 0; k < t / 64; ++k) run += wsum[k];
        const uint32_t my0 = run;
#pragma unroll
        for (int k = 0; k < PER; ++k) { const uint32_t v = c[k]; cnt[t * PER + k] = run; run += v; }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (q * T9 + t < m) keys[cnt[(uint32_t)h[q] & (NS9 - 1)] + rk[q]] = h[q];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint32_t fresh = 0, b = my0;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const uint32_t e = b + c[k];
            for (uint32_t i = b; i < e; ++i) {
                const uint64_t a = keys[i];
                bool dup = false;
                for (uint32_t j = b; j < i; ++j) dup |= keys[j] == a;
                fresh += !dup;
            }
            b = e;
        }
        total += fresh;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    if ((t & 63) == 0 && total) atomicAdd((unsigned long long *)out, (unsigned long long)total);
    if (t == 0 && skip) atomicAdd((unsigned long long *)skipped, (unsigned long long)skip);
}

// V10: one WAVE per bucket (~480 keys), wave-private 1024-slot LDS hash table,
// lane-local probe queues, no workgroup barriers.  4 waves per workgroup.
constexpr int W10 = 4;
constexpr int SL10 = 1024;
constexpr int Q10 = 12;          // <= 768 keys per bucket
__global__ void __launch_bounds__(64 * W10) dedup_v10(const uint64_t *in, const uint64_t *starts, int64_t nb,
                                                     uint64_t *out, uint64_t *skipped) {
    __shared__ uint64_t tab[W10][SL10];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t *T = tab[w];
    uint64_t total = 0, skip = 0;
    for (int64_t f = (int64_t)blockIdx.x * W10 + w; f < nb; f += (int64_t)gridDim.x * W10) {
        const int64_t lo = starts[f], hi = starts[f + 1];
        const int m = (int)(hi - lo);
        if (m > Q10 * 64) { ++skip; continue; }
        uint64_t h[Q10];
#pragma unroll
        for (int q = 0; q < Q10; ++q) { const int i = q * 64 + lane; h[q] = i < m ? in[lo + i] : EMPTY; }
#pragma unroll
        for (int k = 0; k < SL10 / 64; ++k) T[k * 64 + lane] = EMPTY;
        __builtin_amdgcn_wave_barrier();
        int left = m > lane ? (m - lane + 63) / 64 : 0;
        uint64_t x = 0;
        uint32_t pos = 0;
        bool have = false;
        uint32_t fresh = 0;
        while (true) {
            if (!have) {
                if (left == 0) break;
                x = h[0];
#pragma unroll
                for (int k = 0; k < Q10 - 1; ++k) h[k] = h[k + 1];
                --left;
                pos = (uint32_t)x & (SL10 - 1);
                have = true;
            }
            uint64_t cur = T[pos];
            if (cur == EMPTY) {
                cur = atomicCAS((unsigned long long *)&T[pos], (unsigned long long)EMPTY, (unsigned long long)x);
                if (cur == EMPTY) ++fresh;
            }
            if (cur == EMPTY || cur == x) { have = false; continue; }
            pos = (pos + 1) & (SL10 - 1);
        }
        total += fresh;
        __builtin_amdgcn_wave_barrier();
    }
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    if (lane == 0 && total) atomicAdd((unsigned long long *)out, (unsigned long long)total);
    if (lane == 0 && skip) atomicAdd((unsigned long long *)skipped, (unsigned long long)skip);
}

// V11 (= V10 with CAS-only probes): one WAVE per bucket (~480 keys), wave-private 1024-slot LDS hash table,
// lane-local probe queues, no workgroup barriers.  4 waves per workgroup.
__global__ void __launch_bounds__(64 * W10) dedup_v11(const uint64_t *in, const uint64_t *starts, int64_t nb,
                                                     uint64_t *out, uint64_t *skipped) {
    __shared__ uint64_t tab[W10][SL10];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t *T = tab[w];
    uint64_t total = 0, skip = 0;
    for (int64_t f = (int64_t)blockIdx.x * W10 + w; f < nb; f += (int64_t)gridDim.x * W10) {
        const int64_t lo = starts[f], hi = starts[f + 1];
        const int m = (int)(hi - lo);
        if (m > Q10 * 64) { ++skip; continue; }
        uint64_t h[Q10];
#pragma unroll
        for (int q = 0; q < Q10; ++q) { const int i = q * 64 + lane; h[q] = i < m ? in[lo + i] : EMPTY; }
#pragma unroll
        for (int k = 0; k < SL10 / 64; ++k) T[k * 64 + lane] = EMPTY;
        __builtin_amdgcn_wave_barrier();
        int left = m > lane ? (m - lane + 63) / 64 : 0;
        uint64_t x = 0;
        uint32_t pos = 0;
        bool have = false;
        uint32_t fresh = 0;
        while (true) {
            if (!have) {
                if (left == 0) break;
                x = h[0];
#pragma unroll
                for (int k = 0; k < Q10 - 1; ++k) h[k] = h[k + 1];
                --left;
                pos = (uint32_t)x & (SL10 - 1);
                have = true;
            }
            const uint64_t cur = atomicCAS((unsigned long long *)&T[pos], (unsigned long long)EMPTY, (unsigned long long)x);
            if (cur == EMPTY) ++fresh;
            if (cur == EMPTY || cur == x) { have = false; continue; }
            pos = (pos + 1) & (SL10 - 1);
        }
        total += fresh;
        __builtin_amdgcn_wave_barrier();
    }
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    if (lane == 0 && total) atomicAdd((unsigned long long *)out, (unsigned long long)total);
    if (lane == 0 && skip) atomicAdd((unsigned long long *)skipped, (unsigned long long)skip);
}

// V12: V11 generalised: W waves per workgroup, SL-slot wave-private tables
template <int W, int SL, int Q>
__global__ void __launch_bounds__(64 * W) dedup_v12(const uint64_t *in, const uint64_t *starts, int64_t nb,
                                                   uint64_t *out, uint64_t *skipped) {
    __shared__ uint64_t tab[W][SL];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t *T = tab[w];
    uint64_t total = 0, skip = 0;
    for (int64_t f = (int64_t)blockIdx.x * W + w; f < nb; f += (int64_t)gridDim.x * W) {
        const int64_t lo = starts[f], hi = starts[f + 1];
        const int m = (int)(hi - lo);
        if (m > Q * 64) { ++skip; continue; }
        uint64_t h[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) { const int i = q * 64 + lane; h[q] = i < m ? in[lo + i] : EMPTY; }
#pragma unroll
        for (int k = 0; k < SL / 64; ++k) T[k * 64 + lane] = EMPTY;
        __builtin_amdgcn_wave_barrier();
        int left = m > lane ? (m - lane + 63) / 64 : 0;
        uint64_t x = 0;
        uint32_t pos = 0;
        bool have = false;
        uint32_t fresh = 0;
        while (true) {
            if (!have) {
                if (left == 0) break;
                x = h[0];
#pragma unroll
                for (int k = 0; k < Q - 1; ++k) h[k] = h[k + 1];
                --left;
                pos = (uint32_t)x & (SL - 1);
                have = true;
            }
            const uint64_t cur = atomicCAS((unsigned long long *)&T[pos], (unsigned long long)EMPTY, (unsigned long long)x);
            if (cur == EMPTY) ++fresh;
            if (cur == EMPTY || cur == x) { have = false; continue; }
            pos = (pos + 1) & (SL - 1);
        }
        total += fresh;
        __builtin_amdgcn_wave_barrier();
    }
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    if (lane == 0 && total) atomicAdd((unsigned long long *)out, (unsigned long long)total);
    if (lane == 0 && skip) atomicAdd((unsigned long long *)skipped, (unsigned long long)skip);
}

// V13: V12 cfg1 + feature flags (RF read-first, PR probe limit, SP special, BL batch loop)
template <bool RF, bool PR, bool SP, bool BL>
__global__ void __launch_bounds__(256) dedup_v13(const uint64_t *in, const uint64_t *starts, int64_t nb,
                                                 uint64_t *out, uint64_t *skipped) {
    constexpr int W = 4, SL = 2048, Q = 20;
    __shared__ uint64_t tab[W][SL];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t *T = tab[w];
    uint64_t total = 0, skip = 0, special = 0;
    bool full = false;
    for (int64_t f = (int64_t)blockIdx.x * W + w; f < nb; f += (int64_t)gridDim.x * W) {
        const int64_t lo = starts[f], hi = starts[f + 1];
        if (!BL && hi - lo > Q * 64) { ++skip; continue; }
        if (lo == hi) continue;
#pragma unroll
        for (int k = 0; k < SL / 64; ++k) T[k * 64 + lane] = EMPTY;
        __builtin_amdgcn_wave_barrier();
        uint32_t fresh = 0;
        for (int64_t rb = lo; rb < hi; rb += Q * 64) {
            uint64_t h[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) { const int64_t r = rb + q * 64 + lane; h[q] = r < hi ? in[r] : EMPTY; }
            const int64_t rem = hi - rb - lane;
            int left = rem <= 0 ? 0 : (int)min((int64_t)Q, (rem + 63) / 64);
            uint64_t x = 0;
            uint32_t pos = 0;
            int probes = 0;
            bool have = false;
            while (true) {
                if (!have) {
                    if (left == 0) break;
                    x = h[0];
#pragma unroll
                    for (int k = 0; k < Q - 1; ++k) h[k] = h[k + 1];
                    --left;
                    if (SP && x == EMPTY) { ++special; continue; }
                    pos = (uint32_t)x & (SL - 1);
                    probes = 0;
                    have = true;
                }
                uint64_t cur;
                if (RF) {
                    cur = T[pos];
                    if (cur == EMPTY) {
                        cur = atomicCAS((unsigned long long *)&T[pos], (unsigned long long)EMPTY, (unsigned long long)x);
                        if (cur == EMPTY) ++fresh;
                    }
                } else {
                    cur = atomicCAS((unsigned long long *)&T[pos], (unsigned long long)EMPTY, (unsigned long long)x);
                    if (cur == EMPTY) ++fresh;
                }
                if (cur == EMPTY || cur == x) { have = false; continue; }
                pos = (pos + 1) & (SL - 1);
                if (PR && ++probes >= SL / 2) { full = true; have = false; }
            }
            if (!BL) break;
        }
        total += fresh;
        __builtin_amdgcn_wave_barrier();
    }
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    if (lane == 0 && total) atomicAdd((unsigned long long *)out, (unsigned long long)total);
    if (lane == 0 && (skip + special + full)) atomicAdd((unsigned long long *)skipped, (unsigned long long)(skip + special + full));
}

int main() {
    const int bits = 18;
    const int64_t nb = 1 << bits;
    std::vector<uint64_t> st(nb + 1);
    st[0] = 0;
    for (int64_t f = 0; f < nb; ++f) st[f + 1] = st[f] + 3400 + (int64_t)((f * 7919) % 400);
    const int64_t n = st[nb];
    printf("records %lld buckets %lld\n", (long long)n, (long long)nb);
    uint64_t *rec, *starts, *out, *stats;
    uint32_t *ng;
    CK(hipMalloc(&rec, n * 8));
    CK(hipMalloc(&starts, (nb + 1) * 8));
    CK(hipMalloc(&out, 8 * 128));
    CK(hipMalloc(&stats, 8 * 128));
    CK(hipMalloc(&ng, 4 * nb));
    CK(hipMemcpy(starts, st.data(), (nb + 1) * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(gen, dim3(nb), dim3(256), 0, 0, rec, starts, nb, bits);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, n * 8 / (ms * 1e-3) / 1e9);
    };
    timeit("read-only baseline", [&] { hipLaunchKernelGGL(sum_kernel, dim3(2048), dim3(512), 0, 0, rec, n, out); });
    sdp_records r{rec, nullptr, nullptr};
    timeit("libsdp part_dedup (u64)", [&] {
        hipMemset(stats, 0, 8 * 128);
        sdp_part_dedup(&r, 0, nullptr, starts, nb, 0, nullptr, nullptr, ng, stats, 0);
    });
    std::vector<uint64_t> hs(68);
    CK(hipMemcpy(hs.data(), stats, 68 * 8, hipMemcpyDeviceToHost));
    uint64_t g = 0;
    for (int i = 4; i < 68; ++i) g += hs[i];
    printf("  groups %llu (expect %lld) full=%llu\n", (unsigned long long)g, (long long)n, (unsigned long long)hs[3]);
    for (int grid : {512, 1024, 2048}) {
        char nm[64];
        snprintf(nm, sizeof nm, "sub-bucket V4 grid %d", grid);
        timeit(nm, [&] {
            hipMemset(out, 0, 8);
            hipLaunchKernelGGL(dedup_sub, dim3(grid), dim3(VT), 0, 0, rec, starts, nb, out);
        });
        uint64_t o;
        CK(hipMemcpy(&o, out, 8, hipMemcpyDeviceToHost));
        printf("  groups %llu\n", (unsigned long long)o);
    }
    for (int pf = 0; pf < 2; ++pf) {
        timeit(pf ? "sub4 V7 prefetch grid 1024" : "sub4 V7 grid 1024", [&] {
            hipMemset(out, 0, 8);
            if (pf) hipLaunchKernelGGL(dedup_sub4<true>, dim3(1024), dim3(VT), 0, 0, rec, starts, nb, out);
            else hipLaunchKernelGGL(dedup_sub4<false>, dim3(1024), dim3(VT), 0, 0, rec, starts, nb, out);
        });
        uint64_t o;
        CK(hipMemcpy(&o, out, 8, hipMemcpyDeviceToHost));
        printf("  groups %llu\n", (unsigned long long)o);
    }
    for (int T : {512, 1024}) {
        for (int grid : {512, 1024}) {
            char nm[64];
            snprintf(nm, sizeof nm, "V9 T%d grid %d", T, grid);
            timeit(nm, [&] {
                hipMemset(out, 0, 16);
                if (T == 512) hipLaunchKernelGGL(dedup_v9<512>, dim3(grid), dim3(512), 0, 0, rec, starts, nb, out, out + 1);
                else hipLaunchKernelGGL(dedup_v9<1024>, dim3(grid), dim3(1024), 0, 0, rec, starts, nb, out, out + 1);
            });
            uint64_t o[2];
            CK(hipMemcpy(o, out, 16, hipMemcpyDeviceToHost));
            printf("  groups %llu skipped %llu\n", (unsigned long long)o[0], (unsigned long long)o[1]);
        }
    }
    {
        // small buckets for V10: 2^21 buckets of ~450 records
        const int b2 = 21;
        const int64_t nb2 = 1 << b2;
        std::vector<uint64_t> st2(nb2 + 1);
        st2[0] = 0;
        for (int64_t f = 0; f < nb2; ++f) st2[f + 1] = st2[f] + 400 + (int64_t)((f * 7919) % 100);
        const int64_t n2 = st2[nb2];
        uint64_t *starts2;
        CK(hipMalloc(&starts2, (nb2 + 1) * 8));
        CK(hipMemcpy(starts2, st2.data(), (nb2 + 1) * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(gen, dim3(nb2), dim3(256), 0, 0, rec, starts2, nb2, b2);
        CK(hipDeviceSynchronize());
        printf("small buckets: records %lld buckets %lld\n", (long long)n2, (long long)nb2);
        for (int grid : {1024, 4096}) {
            char nm[64];
            for (int v = 10; v <= 11; ++v) {
            snprintf(nm, sizeof nm, "V%d wave/bucket grid %d", v, grid);
            timeit(nm, [&] {
                hipMemset(out, 0, 16);
                if (v == 10) hipLaunchKernelGGL(dedup_v10, dim3(grid), dim3(64 * W10), 0, 0, rec, starts2, nb2, out, out + 1);
                else hipLaunchKernelGGL(dedup_v11, dim3(grid), dim3(64 * W10), 0, 0, rec, starts2, nb2, out, out + 1);
            });
            uint64_t o[2];
            CK(hipMemcpy(o, out, 16, hipMemcpyDeviceToHost));
            printf("  groups %llu (expect %lld) skipped %llu\n", (unsigned long long)o[0], (long long)n2, (unsigned long long)o[1]);
            }
        }
    }
    {
        const int b3 = 20;
        const int64_t nb3 = 1 << b3;
        std::vector<uint64_t> st3(nb3 + 1);
        st3[0] = 0;
        for (int64_t f = 0; f < nb3; ++f) st3[f + 1] = st3[f] + 850 + (int64_t)((f * 7919) % 100);
        const int64_t n3 = st3[nb3];
        uint64_t *starts3;
        CK(hipMalloc(&starts3, (nb3 + 1) * 8));
        CK(hipMemcpy(starts3, st3.data(), (nb3 + 1) * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(gen, dim3(nb3), dim3(256), 0, 0, rec, starts3, nb3, b3);
        CK(hipDeviceSynchronize());
        printf("mid buckets: records %lld buckets %lld\n", (long long)n3, (long long)nb3);
        timeit("libsdp part_dedup mid", [&] {
            hipMemset(stats, 0, 8 * 128);
            sdp_part_dedup(&r, 0, nullptr, starts3, nb3, 0, nullptr, nullptr, ng, stats, 0);
        });
        {
            std::vector<uint64_t> hs3(68);
            CK(hipMemcpy(hs3.data(), stats, 68 * 8, hipMemcpyDeviceToHost));
            uint64_t g3 = 0;
            for (int i = 4; i < 68; ++i) g3 += hs3[i];
            printf("  groups %llu (expect %lld) full=%llu\n", (unsigned long long)g3, (long long)n3, (unsigned long long)hs3[3]);
        }
        auto run13 = [&](const char *nm, auto kern) {
            timeit(nm, [&] {
                hipMemset(out, 0, 16);
                hipLaunchKernelGGL(kern, dim3(4096), dim3(256), 0, 0, rec, starts3, nb3, out, out + 1);
            });
            uint64_t o[2];
            CK(hipMemcpy(o, out, 16, hipMemcpyDeviceToHost));
            printf("  groups %llu skipped %llu\n", (unsigned long long)o[0], (unsigned long long)o[1]);
        };
        run13("V13 base", dedup_v13<false, false, false, false>);
        run13("V13 RF", dedup_v13<true, false, false, false>);
        run13("V13 PR", dedup_v13<false, true, false, false>);
        run13("V13 SP", dedup_v13<false, false, true, false>);
        run13("V13 BL", dedup_v13<false, false, false, true>);
        run13("V13 all", dedup_v13<true, true, true, true>);
        for (int cfg = 0; cfg < 3; ++cfg) {
            for (int grid : {1024, 4096}) {
                char nm[64];
                snprintf(nm, sizeof nm, "V12 cfg%d grid %d", cfg, grid);
                timeit(nm, [&] {
                    hipMemset(out, 0, 16);
                    if (cfg == 0) hipLaunchKernelGGL((dedup_v12<2, 2048, 20>), dim3(grid), dim3(128), 0, 0, rec, starts3, nb3, out, out + 1);
                    else if (cfg == 1) hipLaunchKernelGGL((dedup_v12<4, 2048, 20>), dim3(grid), dim3(256), 0, 0, rec, starts3, nb3, out, out + 1);
                    else hipLaunchKernelGGL((dedup_v12<1, 2048, 20>), dim3(grid), dim3(64), 0, 0, rec, starts3, nb3, out, out + 1);
                });
                uint64_t o[2];
                CK(hipMemcpy(o, out, 16, hipMemcpyDeviceToHost));
                printf("  groups %llu (expect %lld) skipped %llu\n", (unsigned long long)o[0], (long long)n3, (unsigned long long)o[1]);
            }
        }
    }
    return 0;
}
