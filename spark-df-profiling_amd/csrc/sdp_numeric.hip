// sdp_numeric.hip -- numeric column path of describe() on gfx950.
//
// Replaces the per-column Spark job chain of describe_numeric_1d
// (/root/reference/spark_df_profiling/describe.py:192-229) and the common block
// of describe_1d (:143-151):
//   sample + plan  -> value windows around each requested quantile
//   pass 1         -> count / min / max / sum / shifted power sums / zeros and
//                     the window statistics + candidates (one HBM read)
//   radix select   -> exact order statistics inside a window (small arrays)
//   pass 2         -> mad, CASE-WHEN histogram, outlier counts (one HBM read)
// All block partials are merged by a single-block kernel in block order, so
// every result is deterministic for a given grid.
#include <type_traits>
#include "sdp_heavy.h"
#include "sdp_internal.h"

namespace sdp {

constexpr int P1_BLOCK = 256;
constexpr int P1_UNROLL = 2;          // 16-B vectors per thread per tile (x2: the next tile is prefetched)
constexpr int P1_MAX_GRID = 1024;     // 4 blocks per CU on 256 CUs
#ifndef P1_STAGES
#define P1_STAGES 3                   // tiles of pass 1's whole-tile ring (2 in flight)
#endif
#ifndef P1_EXCL_FAST
#define P1_EXCL_FAST 1                // exclusive windows on the whole-tile ring too (2-pair ring; 3.12 -> 3.05 ms per i64 column, profiles/r06p_ab.log)
#endif
#ifndef P1_U32
#define P1_U32 2                      // 16-byte vectors per thread per tile, 4-byte types
#endif
constexpr int SORT_MAX = 16384;       // one-workgroup LDS bitonic sort (128 KiB)

#define SDP_DISPATCH_NUMERIC(DT, ...)                                             \
    switch (DT) {                                                                 \
    case SDP_I8: { using T = int8_t; __VA_ARGS__; } break;                        \
    case SDP_I16: { using T = int16_t; __VA_ARGS__; } break;                      \
    case SDP_I32: { using T = int32_t; __VA_ARGS__; } break;                      \
    case SDP_I64: { using T = int64_t; __VA_ARGS__; } break;                      \
    case SDP_U8: { using T = uint8_t; __VA_ARGS__; } break;                       \
    case SDP_U16: { using T = uint16_t; __VA_ARGS__; } break;                     \
    case SDP_U32: { using T = uint32_t; __VA_ARGS__; } break;                     \
    case SDP_F32: { using T = float; __VA_ARGS__; } break;                        \
    case SDP_F64: { using T = double; __VA_ARGS__; } break;                       \
    default: return set_error(SDP_EINVAL, "unsupported numeric dtype %d", (int)(DT)); \
    }

static int elem_size(int dt) {
    switch (dt) {
    case SDP_I8: case SDP_U8: return 1;
    case SDP_I16: case SDP_U16: return 2;
    case SDP_I32: case SDP_U32: case SDP_F32: return 4;
    case SDP_I64: case SDP_U64: case SDP_F64: return 8;
    default: return 0;
    }
}

static int check_col(const sdp_column *c, const char *who) {
    if (c == nullptr) return set_error(SDP_EINVAL, "%s: null column", who);
    if (c->length < 0) return set_error(SDP_EINVAL, "%s: negative length", who);
    if (c->length > 0 && c->d_values == nullptr) return set_error(SDP_EINVAL, "%s: null values", who);
    if (!aligned16(c->d_values)) return set_error(SDP_EALIGN, "%s: values not 16-byte aligned", who);
    if (elem_size(c->dtype) == 0 || c->dtype == SDP_U64)
        return set_error(SDP_EINVAL, "%s: dtype %d is not a numeric column", who, c->dtype);
    return SDP_OK;
}

static int p1_grid(int64_t n, int dt) {
    const int vpt = 16 / elem_size(dt);
    const int64_t nvec = n / vpt;
    int64_t tiles = (nvec + (int64_t)P1_BLOCK * P1_UNROLL - 1) / ((int64_t)P1_BLOCK * P1_UNROLL);
    if (tiles < 1) tiles = 1;
    return (int)(tiles < P1_MAX_GRID ? tiles : P1_MAX_GRID);
}

// ============================================================================
// sampling and window planning
// ============================================================================

template <typename T>
__global__ void sample_keys_kernel(sdp_column col, int32_t ns, uint64_t *out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ns) return;
    const int64_t n = col.length;
    const int64_t i = (int64_t)(((double)j + 0.5) * (double)n / (double)ns);
    uint64_t k = EMPTY64;
    if (i < n && valid_bit(col.d_validity, col.validity_bit_offset, i)) {
        const T x = ((const T *)col.d_values)[i];
        const double xd = Elem<T>::d(x);
        if (xd == xd) k = Elem<T>::key(x);
    }
    out[j] = k;
}

// every column's sample in one launch (blockIdx.y = column; the dtype is read
// per column, so the tables may mix dtypes): column c's keys at out + c * ns
template <typename T>
__device__ __forceinline__ uint64_t sample_key_at(const sdp_column &col, int64_t i) {
    const T x = ((const T *)col.d_values)[i];
    const double xd = Elem<T>::d(x);
    return xd == xd ? Elem<T>::key(x) : EMPTY64;
}
__global__ void sample_keys_batch_kernel(const sdp_column *cols, int32_t ns, uint64_t *out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ns) return;
    const sdp_column col = cols[blockIdx.y];
    const int64_t n = col.length;
    const int64_t i = (int64_t)(((double)j + 0.5) * (double)n / (double)ns);
    uint64_t k = EMPTY64;
    if (i < n && valid_bit(col.d_validity, col.validity_bit_offset, i)) {
        switch (col.dtype) {
        case SDP_I8: k = sample_key_at<int8_t>(col, i); break;
        case SDP_I16: k = sample_key_at<int16_t>(col, i); break;
        case SDP_I32: k = sample_key_at<int32_t>(col, i); break;
        case SDP_I64: k = sample_key_at<int64_t>(col, i); break;
        case SDP_U8: k = sample_key_at<uint8_t>(col, i); break;
        case SDP_U16: k = sample_key_at<uint16_t>(col, i); break;
        case SDP_U32: k = sample_key_at<uint32_t>(col, i); break;
        case SDP_F32: k = sample_key_at<float>(col, i); break;
        case SDP_F64: k = sample_key_at<double>(col, i); break;
        default: break;
        }
    }
    out[(int64_t)blockIdx.y * ns + j] = k;
}

// LDS bitonic sort of `n` keys (n <= SORT_MAX); pads with EMPTY64.
__device__ void block_sort_keys(uint64_t *s, int n) {
    int P = 2;
    while (P < n) P <<= 1;
    for (int i = n + threadIdx.x; i < P; i += blockDim.x) s[i] = EMPTY64;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = s[i], b = s[ixj];
                    const bool asc = (i & k) == 0;
                    if ((a > b) == asc) { s[i] = b; s[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
}

// one workgroup per column: column b's sample at sample + b * ns, plan at plan + b
__global__ void __launch_bounds__(1024) quantile_plan_kernel(uint64_t *sample, int32_t ns,
                                                             const double *probs, int32_t np,
                                                             int32_t is_float, const int32_t *is_float_v,
                                                             sdp_qplan *plan) {
    __shared__ uint64_t s[SORT_MAX];
    sample += (int64_t)blockIdx.x * ns;
    plan += blockIdx.x;
    if (is_float_v) is_float = is_float_v[blockIdx.x];
    for (int i = threadIdx.x; i < ns; i += blockDim.x) s[i] = sample[i];
    __syncthreads();
    block_sort_keys(s, ns);
    for (int i = threadIdx.x; i < ns; i += blockDim.x) sample[i] = s[i];
    if (threadIdx.x != 0) return;
    int m = 0;
    {   // valid sample keys sort before the EMPTY64 markers
        int lo = 0, hi = ns;
        while (lo < hi) { int mid = (lo + hi) >> 1; if (s[mid] != EMPTY64) lo = mid + 1; else hi = mid; }
        m = lo;
    }
    sdp_qplan p;
    for (int w = 0; w < SDP_MAX_WINDOWS; ++w) { p.lo[w] = 0; p.hi[w] = EMPTY64; p.in_sample[w] = 0; }
    p.n_sample = m;
    p.excl_mask = 0;
    p._pad = 0;
    if (m == 0) {
        p.n_windows = np > 0 ? 1 : 0;
        p.shift = 0.0;
        *plan = p;
        return;
    }
    const uint64_t med = s[(m - 1) / 2];
    p.shift = is_float ? key_f64(med) : (double)key_i64(med);
    int nw = 0;
    // a bound key seen twice in the sample may be frequent: that window keeps
    // exclusive bounds (its bound copies are counted, not collected)
    auto dup = [&](int i) { return (i > 0 && s[i - 1] == s[i]) || (i + 1 < m && s[i + 1] == s[i]); };
    for (int t = 0; t < np && t < SDP_MAX_WINDOWS; ++t) {
        const double q = probs[t];
        const double r = q * (double)(m - 1);
        const int d = (int)ceil(4.0 * sqrt((double)m * q * (1.0 - q))) + 2;
        int il = (int)floor(r) - d, ih = (int)ceil(r) + d;
        if (il < 0) il = 0;
        if (ih > m - 1) ih = m - 1;
        const uint64_t lo = (il == 0) ? 0ull : s[il];
        const uint64_t hi = (ih == m - 1) ? EMPTY64 : s[ih];
        const bool ex = lo == 0ull || (il > 0 && dup(il)) || (ih < m - 1 && dup(ih));
        if (nw > 0 && lo <= p.hi[nw - 1]) {
            if (hi > p.hi[nw - 1]) p.hi[nw - 1] = hi;
            if (ex) p.excl_mask |= 1 << (nw - 1);
        } else {
            p.lo[nw] = lo;
            p.hi[nw] = hi;
            if (ex) p.excl_mask |= 1 << nw;
            ++nw;
        }
    }
    for (int w = 0; w < nw; ++w) {
        // #(s < hi) - #(s <= lo) by binary search on the sorted sample
        int a = 0, b = m;
        while (a < b) { int mid = (a + b) >> 1; if (s[mid] < p.hi[w]) a = mid + 1; else b = mid; }
        const int below_hi = a;
        a = 0; b = m;
        while (a < b) { int mid = (a + b) >> 1; if (s[mid] <= p.lo[w]) a = mid + 1; else b = mid; }
        p.in_sample[w] = below_hi > a ? below_hi - a : 0;
    }
    p.n_windows = nw;
    *plan = p;
}

// Window refinement from a second, larger sample S2 (one workgroup per column).
// The S1 windows are +-(4 sigma + 2) sample ranks of the previous sample; S2's
// keys are counted per window, the windows whose S2 keys fit the LDS sort
// together (in window order) are chosen, their keys sorted, and around each
// probability in a chosen window a window of +-(4 sigma2 + 2) S2 ranks is taken
// inside it, so windows shrink by sqrt(n2 / n1) at the same miss probability.
// A probability in an unchosen window (a heavy value's window holding a large
// share of S2) keeps that S1 window.  S2 keys below each window place the
// ranks.  If a rank lands outside every S1 window the S1 plan stands (windows
// are a performance device: a miss falls back exactly).
__global__ void __launch_bounds__(1024) quantile_refine_kernel(const uint64_t *samples2, int32_t ns2,
                                                               const double *probs, int32_t np, sdp_qplan *plans) {
    __shared__ uint64_t s[SORT_MAX];
    __shared__ uint32_t s_cnt, s_valid, s_chosen;
    __shared__ uint32_t s_below[SDP_MAX_WINDOWS], s_in[SDP_MAX_WINDOWS];
    const uint64_t *sample2 = samples2 + (int64_t)blockIdx.x * ns2;
    sdp_qplan *plan = plans + blockIdx.x;
    const int nw = plan->n_windows;
    if (nw == 0 || plan->n_sample < 64 || ns2 <= plan->n_sample) return;     // (uniform per block)
    uint64_t lo[SDP_MAX_WINDOWS], hi[SDP_MAX_WINDOWS];
#pragma unroll
    for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
        lo[w] = w < nw ? plan->lo[w] : EMPTY64;
        hi[w] = w < nw ? plan->hi[w] : EMPTY64;
    }
    if (threadIdx.x == 0) { s_cnt = 0; s_valid = 0; }
    if (threadIdx.x < SDP_MAX_WINDOWS) { s_below[threadIdx.x] = 0; s_in[threadIdx.x] = 0; }
    __syncthreads();
    uint32_t valid = 0, below[SDP_MAX_WINDOWS], inw[SDP_MAX_WINDOWS];
#pragma unroll
    for (int w = 0; w < SDP_MAX_WINDOWS; ++w) below[w] = inw[w] = 0;
    for (int i = threadIdx.x; i < ns2; i += blockDim.x) {        // pass 1: counts
        const uint64_t k = sample2[i];
        if (k == EMPTY64) continue;                  // null / NaN rows of the sample
        ++valid;
#pragma unroll
        for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
            if (w >= nw) break;
            below[w] += k < lo[w];
            inw[w] += k >= lo[w] && k <= hi[w];
        }
    }
    // block sums of the per-thread counters (fixed-order wave sums, then LDS atomics of 16 partials)
    const uint32_t vs = (uint32_t)wave_sum_u64(valid);
    if (lane_id() == 0) atomicAdd(&s_valid, vs);
#pragma unroll
    for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
        const uint32_t b = (uint32_t)wave_sum_u64(below[w]), c = (uint32_t)wave_sum_u64(inw[w]);
        if (lane_id() == 0 && w < nw) { atomicAdd(&s_below[w], b); atomicAdd(&s_in[w], c); }
    }
    __syncthreads();
    if (threadIdx.x == 0) {                          // windows whose keys fit the sort, in order
        uint32_t acc = 0, ch = 0;
        for (int w = 0; w < nw; ++w)
            if (acc + s_in[w] <= (uint32_t)SORT_MAX) { acc += s_in[w]; ch |= 1u << w; }
        s_chosen = ch;
    }
    __syncthreads();
    const uint32_t chosen = s_chosen;
    if (chosen == 0) return;                         // the S1 plan stands
    for (int i = threadIdx.x; i < ns2; i += blockDim.x) {        // pass 2: keys of the chosen windows
        const uint64_t k = sample2[i];
        if (k == EMPTY64) continue;
        bool in = false;
#pragma unroll
        for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
            if (w >= nw) break;
            in = in || (((chosen >> w) & 1u) && k >= lo[w] && k <= hi[w]);
        }
        if (in) {
            const uint32_t pos = atomicAdd(&s_cnt, 1u);
            if (pos < SORT_MAX) s[pos] = k;
        }
    }
    __syncthreads();
    const uint32_t cnt = s_cnt;
    if (cnt > SORT_MAX || cnt == 0) return;        // the S1 plan stands
    block_sort_keys(s, (int)cnt);                  // windows are disjoint: window w's keys form one run
    if (threadIdx.x != 0) return;
    const uint32_t m2 = s_valid;
    sdp_qplan p = *plan;
    uint32_t seg0[SDP_MAX_WINDOWS];
    uint32_t acc = 0;
    for (int w = 0; w < nw; ++w) { seg0[w] = acc; if ((chosen >> w) & 1u) acc += s_in[w]; }
    uint64_t nlo[SDP_MAX_WINDOWS], nhi[SDP_MAX_WINDOWS];
    int nn = 0, nex = 0;
    for (int t = 0; t < np && t < SDP_MAX_WINDOWS; ++t) {
        const double q = probs[t];
        const double r = q * (double)(m2 - 1);
        int w = -1;
        for (int v = 0; v < nw; ++v)
            if ((double)s_below[v] <= floor(r) && ceil(r) < (double)(s_below[v] + s_in[v])) { w = v; break; }
        if (w < 0) return;                         // a rank outside the S1 windows: keep the S1 plan
        const bool s1ex = ((p.excl_mask >> w) & 1) != 0;
        uint64_t l, h;
        bool ex;
        if ((chosen >> w) & 1u) {
            const int d = (int)ceil(4.0 * sqrt((double)m2 * q * (1.0 - q))) + 2;
            const int cw = (int)s_in[w];
            const int il = (int)floor(r) - d - (int)s_below[w], ih = (int)ceil(r) + d - (int)s_below[w];
            l = il <= 0 ? p.lo[w] : s[seg0[w] + il];
            h = ih >= cw - 1 ? p.hi[w] : s[seg0[w] + ih];
            // exclusive bounds: an S1 bound kept from an exclusive S1 window, lo == 0,
            // or a bound key repeated among the S2 keys of its window
            const int a0 = (int)seg0[w], a1 = a0 + cw;
            auto dup2 = [&](int i) { return (i > a0 && s[i - 1] == s[i]) || (i + 1 < a1 && s[i + 1] == s[i]); };
            ex = l == 0ull || (il <= 0 ? s1ex : dup2(a0 + il)) || (ih >= cw - 1 ? s1ex : dup2(a0 + ih));
        } else {                                   // kept as it was
            l = p.lo[w];
            h = p.hi[w];
            ex = s1ex;
        }
        if (nn > 0 && l <= nhi[nn - 1]) {
            if (h > nhi[nn - 1]) nhi[nn - 1] = h;
            if (ex) nex |= 1 << (nn - 1);
        } else {
            nlo[nn] = l;
            nhi[nn] = h;
            if (ex) nex |= 1 << nn;
            ++nn;
        }
    }
    for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
        p.lo[w] = w < nn ? nlo[w] : 0;
        p.hi[w] = w < nn ? nhi[w] : EMPTY64;
        p.in_sample[w] = 0;
    }
    for (int w = 0; w < nn; ++w) {
        // S2 keys strictly inside (lo, hi): binary search on the sorted keys of
        // the chosen windows, plus the (inclusive, so over-) counts of the
        // unchosen S1 windows it overlaps -- the slot sizing reads this
        int a = 0, b = (int)cnt;
        while (a < b) { int mid = (a + b) >> 1; if (s[mid] < p.hi[w]) a = mid + 1; else b = mid; }
        const int below_hi = a;
        a = 0; b = (int)cnt;
        while (a < b) { int mid = (a + b) >> 1; if (s[mid] <= p.lo[w]) a = mid + 1; else b = mid; }
        uint32_t in_s = below_hi > a ? (uint32_t)(below_hi - a) : 0u;
        for (int v = 0; v < nw; ++v)
            if (!((chosen >> v) & 1u) && lo[v] <= p.hi[w] && hi[v] >= p.lo[w]) in_s += s_in[v];
        p.in_sample[w] = (int32_t)in_s;
    }
    p.n_windows = nn;
    p.n_sample = (int32_t)m2;
    p.excl_mask = nex;
    *plan = p;
}

// ============================================================================
// pass 1
// ============================================================================

// Per-block partial: plain arrays so the epilogue reduces field-wise without
// runtime-indexed register arrays (which hipcc would place in scratch).
constexpr int W_ = SDP_MAX_WINDOWS;
constexpr int NU = 4 + 4 * W_;   // count, n_valid, n_nan, n_zero, gt[W], eqlo[W], eqhi[W], in[W]
struct P1Partial {
    uint64_t u[NU];
    int64_t i[3];                // isum, imin, imax
    double d[8];                 // s1h, s1l, s2, s3h, s3l, s4, dmin, dmax
    uint32_t overflow, _pad;
};

struct P1Thread {
    uint32_t count, n_valid, n_zero;
    uint32_t ncalls;                  // p1_elem calls (wave-uniform): skipped = ncalls - count
    int64_t isum, imin, imax;
    double dmin, dmax;
    double s1, s1c, s2, s3, s3c, s4;
    double t1, t3;                    // plain sums of d and d^3 over the current tile
    uint32_t gt[SDP_MAX_WINDOWS], eqlo[SDP_MAX_WINDOWS], eqhi[SDP_MAX_WINDOWS];
    uint32_t wcur[SDP_MAX_WINDOWS];   // wave-uniform candidate cursors (wave-private slots)
};

constexpr int P1_WPB = 4;            // waves per pass-1 block (P1_BLOCK / WAVE)

struct P1Ctx {
    uint64_t lo[SDP_MAX_WINDOWS], hi[SDP_MAX_WINDOWS];
    uint32_t lo32[SDP_MAX_WINDOWS], hi32[SDP_MAX_WINDOWS];   // 4-byte types, inclusive windows
    uint64_t *seg[SDP_MAX_WINDOWS];   // this wave's candidate slot range of window w
    int nw;
    double K;
    int64_t cap;
};

// One element; every lane of the wave calls this in lockstep (ballots inside).
// Window counts use the key with skipped elements (null, NaN, padding) mapped
// to key 0: no skipped element is above a bound or strictly inside a window,
// and the ones counted as equal to a bound of 0 are taken off in the block
// epilogue (ncalls - count skipped elements), as are eqhi counts of windows
// with lo == hi -- so each window costs two compare-and-carry counts, one
// equality count and the inside test, with no per-element validity masking.
// Per element only `count` is kept among the element counters: n_valid is
// added per vector from its validity bits (p1_valid), NaNs are n_valid -
// count and skipped elements ncalls - count (round 6: 64 -> ~40 VALU per f64
// element).  The key of a kept element is built inside the `ok` branch from
// a value with -0.0 turned into +0.0 by adding +0.0 (IEEE round-to-nearest;
// denormals are preserved in these kernels), so it needs no zero test.
// A candidate store through the global address space: a flat store (the
// slot pointers come from a task table, so they are generic) is unordered
// against the loads on vmcnt, and one in flight made the compiler wait
// vmcnt(0) -- draining the prefetched tiles -- before every use of a tile.
__device__ __forceinline__ void gstore(uint64_t *p, uint32_t i, uint64_t v) {
    ((__attribute__((address_space(1))) uint64_t *)p)[i] = v;
}
template <typename T, bool WIN, bool INCL = false, bool K32 = false>
__device__ __forceinline__ void p1_elem(P1Thread &st, const P1Ctx &cx, T x, bool valid) {
    const double xd = Elem<T>::d(x);
    bool ok = valid;
    if constexpr (Elem<T>::is_float) ok = valid && !(xd != xd);
    uint64_t key = 0ull;
    uint32_t k32 = 0u;
    if (ok) {
        st.count += 1;
        if (Elem<T>::is_float) {
            st.dmin = dmin_nn(st.dmin, xd);       // xd is not NaN here
            st.dmax = dmax_nn(st.dmax, xd);
        } else {
            const int64_t xi = Elem<T>::i(x);
            st.imin = xi < st.imin ? xi : st.imin;
            st.imax = xi > st.imax ? xi : st.imax;
            st.isum = (int64_t)((uint64_t)st.isum + (uint64_t)xi);
        }
        st.n_zero += (xd == 0.0);
        // d and d^3 are summed plainly over the thread's tile (<= 16 terms) and
        // folded into the compensated totals once per tile (p1_fold): the sum
        // errs by <= ~3 eps * sum|d| instead of costing two TwoSums per element
        // (a branch-free form of this block with selects measured 1.8x slower)
        const double d = xd - cx.K;
        const double d2 = d * d;
        st.t1 += d;
        st.s2 += d2;
        st.t3 = fma(d2, d, st.t3);
        st.s4 = fma(d2, d2, st.s4);
        if constexpr (WIN && INCL) {
            if constexpr (K32) k32 = Key32<T>::key_nn(x);
            else key = Elem<T>::key_nn(x);
        }
    }
    if (!WIN) return;                   // no quantile windows (date/timestamp min/max)
    // (exclusive windows: the key after the branch -- built inside it, it
    // stayed live beside the moments and spilled the window counters)
    if constexpr (!INCL) key = ok ? Elem<T>::key(x) : 0ull;
    if constexpr (INCL && K32) {
        // 4-byte types: the same inclusive test on 32-bit keys against bounds
        // mapped into the 32-bit key space (pass1_body; every lo32 > 0, so the
        // skipped elements' key 0 is below every window); a candidate is
        // stored as its 32-bit key (widened after the sweep)
#pragma unroll
        for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
            const uint32_t lo = cx.lo32[w], hi = cx.hi32[w];
            const bool lt = k32 < lo, le = k32 <= hi;
            st.gt[w] += (uint32_t)lt;
            const uint64_t m = __builtin_amdgcn_ballot_w64(le) & ~__builtin_amdgcn_ballot_w64(lt);
            if (m) {
                const uint32_t c = st.wcur[w];
                const uint32_t pos = c + (uint32_t)lane_rank(m);
                if (le && !lt && (int64_t)pos < cx.cap) gstore(cx.seg[w], pos, (uint64_t)k32);
                st.wcur[w] = c + (uint32_t)__popcll(m);
            }
        }
        return;
    }
    if constexpr (INCL) {
        // Inclusive windows (every bound key rare in the sample, lo > 0): one
        // count #(key < lo) -- held in gt[] and turned into #(key > hi) in the
        // epilogue -- and candidates lo <= key <= hi, from the same two
        // compares (the inside mask is ballot(le) & ~ballot(lt): three VALU per
        // window).  Skipped elements (key 0) are below every lo; unused
        // windows have lo > hi (never inside).
#pragma unroll
        for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
            const uint64_t lo = cx.lo[w], hi = cx.hi[w];
            const bool lt = key < lo, le = key <= hi;
            st.gt[w] += (uint32_t)lt;
            const uint64_t m = __builtin_amdgcn_ballot_w64(le) & ~__builtin_amdgcn_ballot_w64(lt);
            if (m) {
                const uint32_t c = st.wcur[w];
                const uint32_t pos = c + (uint32_t)lane_rank(m);
                if (le && !lt && (int64_t)pos < cx.cap) gstore(cx.seg[w], pos, key);
                st.wcur[w] = c + (uint32_t)__popcll(m);
            }
        }
        return;
    }
    // Every window slot is evaluated: unused ones have lo = hi = UINT64_MAX
    // (nothing inside, nothing above; their counts are never read), which
    // keeps the loop free of per-window branches.
#pragma unroll
    for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
        const uint64_t lo = cx.lo[w], hi = cx.hi[w];
        st.gt[w] += (uint32_t)(key > hi);
        st.eqlo[w] += (uint32_t)(key == lo);
        st.eqhi[w] += (uint32_t)(key == hi);
        const bool gt = key > lo, lt = key < hi;
        const bool in = gt & lt;
        const uint64_t m = __builtin_amdgcn_ballot_w64(gt) & __builtin_amdgcn_ballot_w64(lt);
        if (m) {   // wave-uniform; no atomics: this wave owns its slot range
            const uint32_t c = st.wcur[w];
            const uint32_t pos = c + (uint32_t)lane_rank(m);
            if (in && (int64_t)pos < cx.cap) gstore(cx.seg[w], pos, key);
            st.wcur[w] = c + (uint32_t)__popcll(m);
        }
    }
}

__device__ __forceinline__ void p1_fold(P1Thread &st) {
    two_sum_acc(st.s1, st.s1c, st.t1);
    two_sum_acc(st.s3, st.s3c, st.t3);
    st.t1 = st.t3 = 0.0;
}

// The sweep of pass 1 over block bx's tiles (+ the tail), accumulating into st.
// K32: 4-byte types with inclusive windows test 32-bit keys (cx.lo32/hi32).
template <typename T, bool WIN, bool INCL, bool K32>
__device__ __forceinline__ void pass1_sweep(P1Thread &st, const P1Ctx &cx, const sdp_column &col, int64_t cap,
                                            const int G, const int bx) {
    constexpr int VPT = Vec16<T>::N;
    const int64_t n = col.length;
    const int64_t nvec = n / VPT;
    const Vec16<T> *vals = (const Vec16<T> *)col.d_values;
    // 8-byte types: 2 vectors per tile; narrower ones 1 (4-16 elements already)
    constexpr int U = sizeof(T) >= 8 ? P1_UNROLL : sizeof(T) == 4 ? P1_U32 : 1;
    const int64_t tile_vecs = (int64_t)P1_BLOCK * U;
    const int64_t ntiles = (nvec + tile_vecs - 1) / tile_vecs;
    // ping-pong tiles: tile i + 1 is loading while tile i is worked on
    const VBits vbm = vbits_init(col.d_validity, col.validity_bit_offset, col.d_values);
    VecIn<T> ta[U], tb[U];
    auto load = [&](VecIn<T> (&x)[U], int64_t tile) {
#pragma unroll
        for (int u = 0; u < U; ++u) x[u].load(vals, vbm, tile * tile_vecs + (int64_t)u * P1_BLOCK + threadIdx.x, nvec);
    };
    auto work = [&](const VecIn<T> (&x)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t vbits = x[u].bits_nb(vbm);
            st.n_valid += (uint32_t)__popc(vbits);
            st.ncalls += VPT;
#pragma unroll
            for (int e = 0; e < VPT; ++e) p1_elem<T, WIN, INCL, K32>(st, cx, x[u].v.v[e], (vbits >> e) & 1u);
        }
        p1_fold(st);
    };
    // Whole tiles of a column without a bitmap or with a bitmap starting on a
    // 32-bit word (the common case, workgroup-uniform test): loads from a
    // tile base in scalar registers plus a per-lane constant, no clamping, and
    // ONE validity dword per vector, whose word and shift are per-lane
    // constants (a tile covers a multiple of 32 rows).  The general path below
    // (clamped vectors, two validity dwords and an alignbit per vector) takes
    // the last, partial tile and unaligned bitmaps.
    // (exclusive windows: a two-tile ring -- their counters leave no room for
    // a third; with the slot pointers in VGPRs this loop spilled them, 5.9 ->
    // 9.4 ms for C3's int64 columns, profiles/r06e_kernel_stats.csv)
    const bool fast = (INCL || P1_EXCL_FAST) && (vbm.none || (vbm.bit0 & 31) == 0);
    const int64_t nfull = fast ? nvec / tile_vecs : 0;
    int64_t tile = bx;
    if constexpr (INCL || P1_EXCL_FAST) if (tile < nfull) {
        typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));
        typedef const __attribute__((address_space(1))) u32x4g gvec;
        typedef const __attribute__((address_space(1))) uint32_t gword;
        const int t = threadIdx.x;
        const uint32_t lsh = (uint32_t)(t * VPT) & 31u;                      // this lane's first bit in its word
        const int64_t w0 = vbm.bit0 >> 5;
        const uint32_t wnone = vbm.none ? 0xFFFFFFFFu : 0u;
        struct FIn {
            Vec16<T> v[U];
            uint32_t w[U];
        };
        auto loadf = [&](FIn &x, int64_t tl) {
            const int64_t vb = tl * tile_vecs;                                // wave-uniform
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u32x4g raw = ((gvec *)(vals + vb + (int64_t)u * P1_BLOCK))[t];
                __builtin_memcpy(&x.v[u], &raw, 16);
                // (loaded either way -- without a bitmap from the values, which
                // are longer -- and OR-ed with all ones: a load under a branch
                // made the compiler drain the ring with vmcnt(0))
                x.w[u] = ((gword *)vbm.base + w0 + (((vb + (int64_t)u * P1_BLOCK) * VPT) >> 5))[(t * VPT) >> 5] | wnone;
            }
        };
        auto workf = [&](const FIn &x) {
            constexpr uint32_t full = VPT >= 32 ? 0xFFFFFFFFu : ((1u << VPT) - 1u);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t vbits = (x.w[u] >> lsh) & full;
                st.n_valid += (uint32_t)__popc(vbits);
                st.ncalls += VPT;
#pragma unroll
                for (int e = 0; e < VPT; ++e) p1_elem<T, WIN, INCL, K32>(st, cx, x.v[u].v[e], (vbits >> e) & 1u);
            }
            p1_fold(st);
        };
        // a ring of P1_STAGES tiles: P1_STAGES - 1 in flight while one is
        // worked on (ping-pong kept ~32 KB per CU in flight, latency-bound;
        // an HBM miss wants ~72 KB, MI355X_MICROARCH.md)
        constexpr int S = INCL ? P1_STAGES : 2;       // (the exclusive-window counters leave no room for a third tile)
        FIn r[S];
        const int64_t last = nfull - 1;
        auto clampt = [&](int64_t x) { return x <= last ? x : last; };   // past the last whole tile: re-read it
#pragma unroll
        for (int k = 0; k < S - 1; ++k) loadf(r[k], clampt(tile + (int64_t)k * G));
        bool go = true;
        while (go) {
#pragma unroll
            for (int k = 0; k < S; ++k) {
                if (go) {
                    loadf(r[(k + S - 1) % S], clampt(tile + (int64_t)(S - 1) * G));
                    workf(r[k]);
                    tile += G;
                    go = tile < nfull;
                }
            }
        }
    }
    // the general path: every tile (fast == false) or the partial last one
    tile = fast ? (nfull < ntiles && bx == (int)(nfull % G) ? nfull : ntiles) : bx;
    if (tile < ntiles) {
        load(ta, tile);
        while (true) {
            load(tb, tile + G);         // past the last tile: clamped, zero bits, never worked on
            work(ta);
            tile += G;
            if (tile >= ntiles) break;
            load(ta, tile + G);
            work(tb);
            tile += G;
            if (tile >= ntiles) break;
        }
    }
    // tail elements (n % VPT) by the first wave of block 0
    if (bx == 0 && threadIdx.x < WAVE) {
        const int64_t i = nvec * VPT + threadIdx.x;
        const bool inb = i < n;
        T x = inb ? ((const T *)col.d_values)[i] : (T)0;
        const bool valid = inb && valid_bit(col.d_validity, col.validity_bit_offset, i);
        st.n_valid += valid;
        st.ncalls += 1;
        p1_elem<T, WIN, INCL, K32>(st, cx, x, valid);
        p1_fold(st);
    }
    if constexpr (INCL && K32) {
        // widen this wave's 32-bit candidate keys in place (its own stores,
        // complete after the vmcnt wait; its slots are read by no other wave)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
            if (w >= cx.nw) break;
            const int64_t nc = (int64_t)st.wcur[w] < cap ? (int64_t)st.wcur[w] : cap;
            uint64_t *seg = cx.seg[w];
            for (int64_t i = lane_id(); i < nc; i += WAVE) seg[i] = Key32<T>::widen_valid((uint32_t)seg[i]);
        }
    }
}

// pass 1 of one column by block bx of a G-block grid (the batched launch runs
// several columns' grids side by side, blockIdx.y = column)
template <typename T, bool WIN, bool INCL>
__device__ __forceinline__ void pass1_body(const sdp_column &col, const sdp_qplan *plan, P1Partial *partials,
                                           uint64_t *cand, uint32_t *cand_counts, int64_t cap, const int G,
                                           const int bx) {
    P1Ctx cx;
    cx.nw = plan->n_windows;
#pragma unroll
    for (int w = 0; w < SDP_MAX_WINDOWS; ++w) {
        cx.lo[w] = w < cx.nw ? plan->lo[w] : EMPTY64;
        cx.hi[w] = w < cx.nw ? plan->hi[w] : (INCL ? EMPTY64 - 1 : EMPTY64);
        const int64_t seg = ((int64_t)w * G + bx) * P1_WPB + (threadIdx.x / WAVE);
        // (wave-uniform: held in scalar registers -- as lane values these ten
        // VGPRs spilled the exclusive-window kernels, whose reloads then put a
        // full vmcnt(0) drain into every element)
        cx.seg[w] = uniform_ptr(cand + seg * cap);
    }
    cx.K = plan->shift;
    cx.cap = cap;
    bool use32 = false;
    if constexpr (INCL && Key32<T>::ok) {
        // 32-bit bounds: lane j < W computes lo32[j], lane W + j hi32[j] (a
        // 32-step search each), read back as wave-uniform values; unused windows
        // have lo32 > hi32 (nothing inside).  The 32-bit test is exact only when
        // every used lo has a preimage above key 0 (the key skipped elements
        // take; lo32 == 0 happens for a window starting at INT32_MIN or 0u) and
        // below 2^32; otherwise the column takes the 64-bit test.
        const int ln = lane_id();
        const int w = ln % SDP_MAX_WINDOWS;
        uint32_t v = 0;
        bool bad = false;
        if (ln < 2 * SDP_MAX_WINDOWS) {
            if (w < cx.nw) {
                if (ln < SDP_MAX_WINDOWS) {
                    const uint64_t l = key32_lower<T>(plan->lo[w]);
                    bad = l == 0 || l > 0xFFFFFFFFull;
                    v = (uint32_t)l;
                } else {
                    // 2^32 (no preimage of hi + 1): every 32-bit key is <= hi
                    v = (uint32_t)(key32_lower<T>(plan->hi[w] + 1) - 1);
                }
            } else {
                v = ln < SDP_MAX_WINDOWS ? 0xFFFFFFFFu : 0xFFFFFFFEu;
            }
        }
#pragma unroll
        for (int j = 0; j < SDP_MAX_WINDOWS; ++j) {
            cx.lo32[j] = __builtin_amdgcn_readlane(v, j);
            cx.hi32[j] = __builtin_amdgcn_readlane(v, SDP_MAX_WINDOWS + j);
        }
        use32 = __builtin_amdgcn_ballot_w64(bad) == 0;
    }

    P1Thread st;
    st.count = st.n_valid = st.n_zero = st.ncalls = 0;
    st.isum = 0;
    st.imin = INT64_MAX;
    st.imax = INT64_MIN;
    st.dmin = __builtin_inf();
    st.dmax = -__builtin_inf();
    st.s1 = st.s1c = st.s2 = st.s3 = st.s3c = st.s4 = 0.0;
    st.t1 = st.t3 = 0.0;
#pragma unroll
    for (int w = 0; w < SDP_MAX_WINDOWS; ++w) st.gt[w] = st.eqlo[w] = st.eqhi[w] = st.wcur[w] = 0;

    if constexpr (INCL && Key32<T>::ok) {
        if (use32) pass1_sweep<T, WIN, INCL, true>(st, cx, col, cap, G, bx);
        else pass1_sweep<T, WIN, INCL, false>(st, cx, col, cap, G, bx);
    } else {
        pass1_sweep<T, WIN, INCL, false>(st, cx, col, cap, G, bx);
    }
    // ---- block reduction: waves, then LDS, fixed order ----------------------
    __shared__ uint64_t s_u[P1_BLOCK / WAVE][NU];
    __shared__ int64_t s_i[P1_BLOCK / WAVE][3];
    __shared__ double s_d[P1_BLOCK / WAVE][8];
    const int wid = threadIdx.x / WAVE, lane = lane_id();
    {
        double h = st.s1, l = st.s1c;
        wave_sum_dd(h, l);
        double h3 = st.s3, l3 = st.s3c;
        wave_sum_dd(h3, l3);
        const double s2 = wave_sum_f64(st.s2), s4 = wave_sum_f64(st.s4);
        const double dmn = wave_min_f64(st.dmin), dmx = wave_max_f64(st.dmax);
        const int64_t isum = wave_sum_i64(st.isum), imn = wave_min_i64(st.imin), imx = wave_max_i64(st.imax);
        const uint64_t c0 = wave_sum_u64(st.count), c1 = wave_sum_u64(st.n_valid);
        const uint64_t c2 = Elem<T>::is_float ? c1 - c0 : 0ull, c3 = wave_sum_u64(st.n_zero);
        if (lane == 0) {
            s_d[wid][0] = h; s_d[wid][1] = l; s_d[wid][2] = s2; s_d[wid][3] = h3;
            s_d[wid][4] = l3; s_d[wid][5] = s4; s_d[wid][6] = dmn; s_d[wid][7] = dmx;
            s_i[wid][0] = isum; s_i[wid][1] = imn; s_i[wid][2] = imx;
            s_u[wid][0] = c0; s_u[wid][1] = c1; s_u[wid][2] = c2; s_u[wid][3] = c3;
        }
        const uint64_t skip = wave_sum_u64(st.ncalls) - c0;
#pragma unroll
        for (int w = 0; w < W_; ++w) {
            uint64_t g = wave_sum_u64(st.gt[w]);
            uint64_t e1 = wave_sum_u64(st.eqlo[w]);
            uint64_t e2 = wave_sum_u64(st.eqhi[w]);
            if (INCL) {                                     // g = #(key < lo), skipped elements included
                g = c0 - (g - skip) - st.wcur[w];           // -> #(key > hi)
                e1 = e2 = 0;
            } else {
                if (cx.lo[w] == 0) e1 -= skip;              // skipped elements carry key 0
                if (cx.hi[w] == 0) e2 -= skip;
                if (cx.hi[w] == cx.lo[w]) e2 = 0;           // one bound: counted as eqlo only
            }
            if (lane == 0) {
                s_u[wid][4 + w] = g; s_u[wid][4 + W_ + w] = e1; s_u[wid][4 + 2 * W_ + w] = e2;
                s_u[wid][4 + 3 * W_ + w] = st.wcur[w];
                if (w < cx.nw)
                    cand_counts[((int64_t)w * G + bx) * P1_WPB + wid] =
                        (int64_t)st.wcur[w] < cap ? st.wcur[w] : (uint32_t)cap;
            }
        }
    }
    __syncthreads();
    P1Partial *out = partials + bx;
    const int t = threadIdx.x;
    constexpr int NW = P1_BLOCK / WAVE;
    if (t < NU) {
        uint64_t a = 0;
        for (int w = 0; w < NW; ++w) a += s_u[w][t];
        out->u[t] = a;
    } else if (t == 64) {
        int64_t a = s_i[0][0], mn = s_i[0][1], mx = s_i[0][2];
        for (int w = 1; w < NW; ++w) {
            a = (int64_t)((uint64_t)a + (uint64_t)s_i[w][0]);
            mn = s_i[w][1] < mn ? s_i[w][1] : mn;
            mx = s_i[w][2] > mx ? s_i[w][2] : mx;
        }
        out->i[0] = a; out->i[1] = mn; out->i[2] = mx;
    } else if (t == 65 || t == 66) {
        const int o = (t == 65) ? 0 : 3;   // (s1h,s1l) or (s3h,s3l)
        double h = s_d[0][o], l = s_d[0][o + 1];
        for (int w = 1; w < NW; ++w) dd_add(h, l, s_d[w][o], s_d[w][o + 1]);
        out->d[o] = h; out->d[o + 1] = l;
    } else if (t == 67) {
        double a = 0.0, b = 0.0, mn = s_d[0][6], mx = s_d[0][7];
        for (int w = 0; w < NW; ++w) { a += s_d[w][2]; b += s_d[w][5]; }
        for (int w = 1; w < NW; ++w) { mn = fmin(mn, s_d[w][6]); mx = fmax(mx, s_d[w][7]); }
        out->d[2] = a; out->d[5] = b; out->d[6] = mn; out->d[7] = mx;
    } else if (t == 68) {
        uint32_t ovf = 0;
        for (int w = 0; w < cx.nw; ++w)
            for (int v = 0; v < NW; ++v)
                if ((int64_t)s_u[v][4 + 3 * W_ + w] > cap) ovf |= 1u << w;
        out->overflow = ovf;
        out->_pad = 0;
    }
}

template <typename T, bool WIN, bool INCL = false>
__global__ void __launch_bounds__(P1_BLOCK, 4) pass1_kernel(sdp_column col, const sdp_qplan *plan,
                                                         P1Partial *partials, uint64_t *cand,
                                                         uint32_t *cand_counts, int64_t cap) {
    pass1_body<T, WIN, INCL>(col, plan, partials, cand, cand_counts, cap, (int)gridDim.x, (int)blockIdx.x);
}
// several columns of one dtype and window mode in one launch: blockIdx.y = task
template <typename T, bool WIN, bool INCL = false>
__global__ void __launch_bounds__(P1_BLOCK, 4) pass1_batch_kernel(const sdp_pass1_task *tasks) {
    const sdp_pass1_task &tk = tasks[blockIdx.y];
    if ((int)blockIdx.x >= tk.grid) return;
    pass1_body<T, WIN, INCL>(tk.col, tk.d_plan, (P1Partial *)tk.d_work, tk.d_cand, tk.d_cand_counts,
                             tk.slot_capacity, tk.grid, (int)blockIdx.x);
}

// Deterministic merge of the block partials: every field is reduced by the
// whole workgroup (strided partial sums, then a fixed-order tree in LDS).
constexpr int MERGE_T = 256;

__device__ __forceinline__ void block_reduce_dd(double &h, double &l, double *sh, double *sl) {
    sh[threadIdx.x] = h; sl[threadIdx.x] = l;
    __syncthreads();
    for (int o = MERGE_T / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) dd_add(sh[threadIdx.x], sl[threadIdx.x], sh[threadIdx.x + o], sl[threadIdx.x + o]);
        __syncthreads();
    }
    h = sh[0]; l = sl[0];
    __syncthreads();
}

template <typename V, typename Op>
__device__ __forceinline__ V block_reduce(V v, V *sm, Op op) {
    sm[threadIdx.x] = v;
    __syncthreads();
    for (int o = MERGE_T / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) sm[threadIdx.x] = op(sm[threadIdx.x], sm[threadIdx.x + o]);
        __syncthreads();
    }
    v = sm[0];
    __syncthreads();
    return v;
}

__device__ __forceinline__ void pass1_merge_body(const P1Partial *partials, int grid, const sdp_qplan *plan,
                                                 sdp_pass1_result *out);
__global__ void __launch_bounds__(MERGE_T) pass1_merge_kernel(const P1Partial *partials, int grid,
                                                              const sdp_qplan *plan, sdp_pass1_result *out) {
    pass1_merge_body(partials, grid, plan, out);
}
__global__ void __launch_bounds__(MERGE_T) pass1_merge_batch_kernel(const sdp_pass1_task *tasks) {
    const sdp_pass1_task &tk = tasks[blockIdx.x];
    pass1_merge_body((const P1Partial *)tk.d_work, tk.grid, tk.d_plan, tk.d_result);
}
__device__ __forceinline__ void pass1_merge_body(const P1Partial *partials, int grid, const sdp_qplan *plan,
                                                 sdp_pass1_result *out) {
    __shared__ double sh[MERGE_T], sl[MERGE_T];
    __shared__ uint64_t su[MERGE_T];
    __shared__ int64_t si[MERGE_T];
    const int t = threadIdx.x;
    auto addu = [](uint64_t a, uint64_t b) { return a + b; };
    for (int f = 0; f < NU; ++f) {
        uint64_t a = 0;
        for (int b = t; b < grid; b += MERGE_T) a += partials[b].u[f];
        a = block_reduce(a, su, addu);
        if (t == 0) {
            uint64_t *dst;
            if (f < 4) dst = (&out->count) + f;
            else if (f < 4 + W_) dst = out->w_gt + (f - 4);
            else if (f < 4 + 2 * W_) dst = out->w_eq_lo + (f - 4 - W_);
            else if (f < 4 + 3 * W_) dst = out->w_eq_hi + (f - 4 - 2 * W_);
            else dst = out->w_in + (f - 4 - 3 * W_);
            *dst = a;
        }
    }
    {
        int64_t a = 0, mn = INT64_MAX, mx = INT64_MIN;
        for (int b = t; b < grid; b += MERGE_T) {
            a = (int64_t)((uint64_t)a + (uint64_t)partials[b].i[0]);
            mn = partials[b].i[1] < mn ? partials[b].i[1] : mn;
            mx = partials[b].i[2] > mx ? partials[b].i[2] : mx;
        }
        a = block_reduce(a, si, [](int64_t x, int64_t y) { return (int64_t)((uint64_t)x + (uint64_t)y); });
        mn = block_reduce(mn, si, [](int64_t x, int64_t y) { return x < y ? x : y; });
        mx = block_reduce(mx, si, [](int64_t x, int64_t y) { return x > y ? x : y; });
        if (t == 0) { out->isum = a; out->imin = mn; out->imax = mx; }
    }
    for (int o = 0; o <= 3; o += 3) {
        double h = 0.0, l = 0.0;
        for (int b = t; b < grid; b += MERGE_T) dd_add(h, l, partials[b].d[o], partials[b].d[o + 1]);
        block_reduce_dd(h, l, sh, sl);
        if (t == 0) {
            if (o == 0) { out->s1_hi = h; out->s1_lo = l; } else { out->s3_hi = h; out->s3_lo = l; }
        }
    }
    {
        double a = 0.0, c = 0.0, mn = __builtin_inf(), mx = -__builtin_inf();
        uint64_t ovf = 0;
        for (int b = t; b < grid; b += MERGE_T) {
            a += partials[b].d[2]; c += partials[b].d[5];
            mn = fmin(mn, partials[b].d[6]); mx = fmax(mx, partials[b].d[7]);
            ovf |= partials[b].overflow;
        }
        auto addd = [](double x, double y) { return x + y; };
        a = block_reduce(a, sh, addd);
        c = block_reduce(c, sh, addd);
        mn = block_reduce(mn, sh, [](double x, double y) { return fmin(x, y); });
        mx = block_reduce(mx, sh, [](double x, double y) { return fmax(x, y); });
        ovf = block_reduce(ovf, su, [](uint64_t x, uint64_t y) { return x | y; });
        if (t == 0) {
            out->s2 = a; out->s4 = c; out->dmin = mn; out->dmax = mx;
            out->w_overflow = (uint32_t)ovf;
            out->_pad = 0;
            out->shift = plan->shift;
        }
    }
}

// ============================================================================
// candidate compaction and radix select
// ============================================================================

// counts[nseg] per-segment counts -> dense copy, in two kernels: a single
// workgroup scans the counts into exclusive offsets (chunks of 1024, carried
// sequentially), then one workgroup per segment copies it.
__global__ void __launch_bounds__(1024) scan_counts_kernel(const uint32_t *counts, int nseg, uint64_t *offs,
                                                           uint64_t *total) {
    __shared__ uint64_t s[1024];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < nseg; base += 1024) {
        const int i = base + threadIdx.x;
        const uint64_t v = i < nseg ? counts[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {     // Hillis-Steele inclusive scan
            const uint64_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < nseg) offs[i] = carry + s[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += s[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ void copy_segments_kernel(const uint64_t *cand, const uint32_t *counts, const uint64_t *offs,
                                     int nseg, int64_t cap, uint64_t *out) {
    for (int b = blockIdx.x; b < nseg; b += gridDim.x) {
        const uint32_t c = counts[b];
        const uint64_t base = offs[b];
        const uint64_t *src = cand + (int64_t)b * cap;
        for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) out[base + i] = src[i];
    }
}

__global__ void radix_hist_kernel(const uint64_t *keys, const uint64_t *n_ptr, uint64_t prefix,
                                  int shift, uint64_t *hist) {
    __shared__ uint32_t h[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t n = *n_ptr;
    const int top = shift + 11;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        const bool match = top >= 64 ? true : ((k >> top) == prefix);
        if (match) atomicAdd(&h[(k >> shift) & 2047u], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += blockDim.x)
        if (h[i]) atomicAdd((unsigned long long *)&hist[i], (unsigned long long)h[i]);
}

// Block-staged compaction: matches gather in an LDS buffer and leave with one
// global atomic per flush (not one per wave per iteration).
constexpr int STAGE = 4096;

struct Stager {
    uint64_t *buf;      // LDS [STAGE]
    uint32_t *cnt;      // LDS
    uint64_t *gbase;    // LDS
};

// every thread calls with its candidate (keep) -- all threads of the block
__device__ __forceinline__ void stage_push(Stager &sg, bool keep, uint64_t v, uint64_t *out,
                                           unsigned long long *out_n, bool last) {
    const uint64_t m = __ballot(keep);
    if (m) {
        uint32_t base = 0;
        const int leader = __ffsll((long long)m) - 1;
        if (lane_id() == leader) base = atomicAdd(sg.cnt, (uint32_t)__popcll(m));
        base = __shfl(base, leader, WAVE);
        if (keep) sg.buf[base + lane_rank(m)] = v;
    }
    // (the barriers order LDS only: the flushed stores and the caller's next
    // loads stay in flight)
    lds_barrier();
    const uint32_t c = *sg.cnt;
    if (c > STAGE - blockDim.x || (last && c > 0)) {
        if (threadIdx.x == 0) *sg.gbase = atomicAdd(out_n, (unsigned long long)c);
        lds_barrier();
        const uint64_t b = *sg.gbase;
        for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) out[b + i] = sg.buf[i];
        lds_barrier();
        if (threadIdx.x == 0) *sg.cnt = 0;
    }
    lds_barrier();
}

__global__ void radix_filter_kernel(const uint64_t *keys, const uint64_t *n_ptr, uint64_t prefix,
                                    int shift, uint64_t *out, uint64_t *out_n) {
    __shared__ uint64_t s_buf[STAGE];
    __shared__ uint32_t s_cnt;
    __shared__ uint64_t s_gbase;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    Stager sg{s_buf, &s_cnt, &s_gbase};
    const uint64_t n = *n_ptr;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t iters = (n + stride - 1) / stride;
    for (uint64_t it = 0; it < iters; ++it) {
        const uint64_t i = it * stride + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        uint64_t k = 0;
        bool keep = false;
        if (i < n) {
            k = keys[i];
            keep = shift >= 64 ? true : ((k >> shift) == prefix);
        }
        stage_push(sg, keep, k, out, (unsigned long long *)out_n, it + 1 == iters);
    }
}

// ---- device-driven k-th key (single rank) ----------------------------------------
// The digit of every radix round is chosen on the GPU (radix_decide_kernel) from
// a state the next round's kernels read, so a whole select -- up to six 11-bit
// rounds -- is queued without a host round trip; the host reads the results of
// all quantiles of a column at once.
struct SelState {
    uint64_t prefix;     // digits fixed so far (bits above shift + 11)
    int64_t k;           // rank among the keys that match prefix
    int32_t shift;       // bit position of the digit of the current round
    int32_t done;
    uint64_t result;
    int32_t width;       // batched selects: bits of the current digit (<= 11)
    int32_t _pad;
};

// d_k (nullable): the rank is read from device memory (a rank computed on the
// device from a device-side count, sdp_quantiles) instead of `k`
__global__ void select_init_kernel(SelState *st, uint64_t prefix, int64_t k, int shift, uint64_t *hist,
                                   const int64_t *d_k) {
    if (threadIdx.x == 0) {
        st->prefix = prefix;
        st->k = d_k ? *d_k : k;
        st->shift = shift;
        st->done = 0;
        st->result = EMPTY64;
    }
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) hist[i] = 0;
}

__global__ void radix_hist_st_kernel(const uint64_t *keys, const uint64_t *n_ptr, const SelState *st,
                                     uint64_t *hist) {
    if (st->done) return;
    __shared__ uint32_t h[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t n = *n_ptr, prefix = st->prefix;
    const int shift = st->shift, top = shift + 11;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // four independent loads in flight per thread before the LDS atomics
    constexpr int R = 4;
    for (; i + (R - 1) * stride < n; i += R * stride) {
        uint64_t k[R];
#pragma unroll
        for (int r = 0; r < R; ++r) k[r] = keys[i + r * stride];
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (top >= 64 || (k[r] >> top) == prefix) atomicAdd(&h[(k[r] >> shift) & 2047u], 1u);
    }
    for (; i < n; i += stride) {
        const uint64_t k = keys[i];
        if (top >= 64 || (k >> top) == prefix) atomicAdd(&h[(k >> shift) & 2047u], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += blockDim.x)
        if (h[i]) atomicAdd((unsigned long long *)&hist[i], (unsigned long long)h[i]);
}

// one workgroup of 1024 threads: digit j with cum[j-1] <= k < cum[j]; the
// histogram and the next round's output counter are cleared for the next round
__global__ void __launch_bounds__(1024) radix_decide_kernel(uint64_t *hist, SelState *st, uint64_t *next_n,
                                                            uint64_t *result) {
    if (st->done) return;
    __shared__ uint64_t s[1024];
    __shared__ int s_j;
    __shared__ uint64_t s_before;
    const int t = threadIdx.x;
    const uint64_t a = hist[2 * t], b = hist[2 * t + 1];
    s[t] = a + b;
    if (t == 0) { s_j = -1; s_before = 0; }
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {        // inclusive scan of the pair sums
        const uint64_t v = t >= o ? s[t - o] : 0;
        __syncthreads();
        s[t] += v;
        __syncthreads();
    }
    const uint64_t k = (uint64_t)st->k;
    const uint64_t excl = s[t] - a - b;
    if (excl <= k && k < s[t]) {
        s_j = k < excl + a ? 2 * t : 2 * t + 1;
        s_before = k < excl + a ? excl : excl + a;
    }
    __syncthreads();
    hist[2 * t] = 0;
    hist[2 * t + 1] = 0;
    if (t == 0) {
        if (s_j < 0) {                          // k beyond the keys: no such rank
            st->done = 1;
            st->result = EMPTY64;
            if (result) *result = EMPTY64;
        } else {
            st->k = (int64_t)(k - s_before);
            st->prefix = (st->shift + 11 >= 64 ? 0ull : (st->prefix << 11)) | (uint64_t)s_j;
            if (st->shift == 0) {
                st->done = 1;
                st->result = st->prefix;
                if (result) *result = st->prefix;
            } else {
                st->shift -= 11;
            }
        }
        if (next_n) *next_n = 0;
    }
}

__global__ void radix_filter_st_kernel(const uint64_t *keys, const uint64_t *n_ptr, const SelState *st,
                                       uint64_t *out, uint64_t *out_n) {
    if (st->done) return;
    __shared__ uint64_t s_buf[STAGE];
    __shared__ uint32_t s_cnt;
    __shared__ uint64_t s_gbase;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    Stager sg{s_buf, &s_cnt, &s_gbase};
    const uint64_t n = *n_ptr, prefix = st->prefix;
    const int top = st->shift + 11;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t iters = (n + stride - 1) / stride;
    for (uint64_t it = 0; it < iters; ++it) {
        const uint64_t i = it * stride + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        uint64_t k = 0;
        bool keep = false;
        if (i < n) {
            k = keys[i];
            keep = top >= 64 ? true : ((k >> top) == prefix);
        }
        stage_push(sg, keep, k, out, (unsigned long long *)out_n, it + 1 == iters);
    }
}

// filter of one round fused with the next round's digit histogram: the keys
// that survive (prefix match after radix_decide_kernel moved the state on)
// are compacted AND counted by their next digit, so a round costs one pass over
// its candidates and two launches (decide, filter+hist) instead of three.
__global__ void radix_filter_hist_st_kernel(const uint64_t *keys, const uint64_t *n_ptr, const SelState *st,
                                            uint64_t *out, uint64_t *out_n, uint64_t *hist) {
    if (st->done) return;
    __shared__ uint64_t s_buf[STAGE];
    __shared__ uint32_t s_cnt;
    __shared__ uint64_t s_gbase;
    __shared__ uint32_t h[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) h[i] = 0;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    Stager sg{s_buf, &s_cnt, &s_gbase};
    const uint64_t n = *n_ptr, prefix = st->prefix;
    const int shift = st->shift, top = shift + 11;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t iters = (n + stride - 1) / stride;
    for (uint64_t it = 0; it < iters; ++it) {
        const uint64_t i = it * stride + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        uint64_t k = 0;
        bool keep = false;
        if (i < n) {
            k = keys[i];
            keep = top >= 64 ? true : ((k >> top) == prefix);
            if (keep) atomicAdd(&h[(k >> shift) & 2047u], 1u);
        }
        stage_push(sg, keep, k, out, (unsigned long long *)out_n, it + 1 == iters);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += blockDim.x)
        if (h[i]) atomicAdd((unsigned long long *)&hist[i], (unsigned long long)h[i]);
}

__global__ void __launch_bounds__(1024) sort_small_kernel(uint64_t *keys, const uint64_t *n_ptr) {
    __shared__ uint64_t s[SORT_MAX];
    const int n = (int)min((uint64_t)SORT_MAX, *n_ptr);
    for (int i = threadIdx.x; i < n; i += blockDim.x) s[i] = keys[i];
    __syncthreads();
    block_sort_keys(s, n);
    for (int i = threadIdx.x; i < n; i += blockDim.x) keys[i] = s[i];
}

// n_sets independent sorts of n_each keys each (one workgroup per set)
__global__ void __launch_bounds__(1024) sort_small_batch_kernel(uint64_t *keys, int32_t n_each) {
    __shared__ uint64_t s[SORT_MAX];
    keys += (int64_t)blockIdx.x * n_each;
    for (int i = threadIdx.x; i < n_each; i += blockDim.x) s[i] = keys[i];
    __syncthreads();
    block_sort_keys(s, n_each);
    for (int i = threadIdx.x; i < n_each; i += blockDim.x) keys[i] = s[i];
}

// keys of the na.drop rows with lo <= key <= hi (the whole column: 0, UINT64_MAX)
template <typename T>
__global__ void column_keys_kernel(sdp_column col, uint64_t lo, uint64_t hi, uint64_t *out, uint64_t *out_n) {
    __shared__ uint64_t s_buf[STAGE];
    __shared__ uint32_t s_cnt;
    __shared__ uint64_t s_gbase;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    Stager sg{s_buf, &s_cnt, &s_gbase};
    const int64_t n = col.length;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t iters = (n + stride - 1) / stride;
    for (int64_t it = 0; it < iters; ++it) {
        const int64_t i = it * stride + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        bool keep = false;
        uint64_t k = 0;
        if (i < n && valid_bit(col.d_validity, col.validity_bit_offset, i)) {
            const T x = ((const T *)col.d_values)[i];
            const double xd = Elem<T>::d(x);
            k = Elem<T>::key(x);
            keep = xd == xd && k >= lo && k <= hi;
        }
        stage_push(sg, keep, k, out, (unsigned long long *)out_n, it + 1 == iters);
    }
}

// ---- countDistinct of a sorted column -------------------------------------------
// A column whose na.drop keys are non-decreasing in row order (ids, timestamps,
// pre-sorted data) has distinct = 1 + #(key changes between consecutive valid
// rows) -- one streaming read instead of the partitioning pipeline.  Each
// element compares its key with the previous valid row's (a walk back over
// nulls, normally one cached load); any decrease sets the violation flag and
// the caller takes the grouping path.  out: [0] distinct (the first valid row
// counts 1), [1] violation, [2] first valid row, [3] last valid row (indices,
// turned into keys by sorted_distinct_final_kernel).
constexpr int SD_T = 256;
constexpr int SD_WALK = 256;            // rows walked back over nulls at most

template <typename T>
__device__ __forceinline__ bool sd_fetch(const sdp_column &c, int64_t i, uint64_t &k) {
    if (!valid_bit(c.d_validity, c.validity_bit_offset, i)) return false;
    const T x = ((const T *)c.d_values)[i];
    k = Elem<T>::key(x);                // NaN: one canonical key; -0.0 == +0.0
    return true;
}

// Each lane takes SD_V consecutive rows (whole 16-byte vectors and one read of
// their validity bits), counts the key changes inside them, and learns the
// key before its first valid row from the lane to its left (__shfl_up: that
// lane holds the rows just before); lane 0 of a wave, or a lane whose left
// neighbour saw only nulls, walks back row by row (rare: one lookup per 64
// lanes, or SD_V nulls in a row).  The element-at-a-time form it replaced
// waited on every row's validity byte and value: 3.3 ms per 1e9-row int64
// column, 2.4 TB/s.
constexpr int SD_V = 8;                 // rows per lane per step
template <typename T>
__global__ void __launch_bounds__(SD_T) sorted_distinct_kernel(sdp_column col, uint64_t *out) {
    constexpr int VPT = Vec16<T>::N;
    constexpr int SV = SD_V > VPT ? SD_V : VPT;        // rows per lane (1-byte types: 16)
    constexpr int NV = SV / VPT;
    const int64_t n = col.length;
    const int64_t ngroups = (n + SV - 1) / SV;
    const int64_t stride = (int64_t)gridDim.x * SD_T;
    const int lane = lane_id();
    uint64_t d = 0;
    bool viol = false;
    int64_t first = INT64_MAX, last = -1;
    for (int64_t gb = (int64_t)blockIdx.x * SD_T; gb < ngroups; gb += stride) {
        const int64_t gi = gb + threadIdx.x;           // (the wave's lanes take consecutive groups)
        const int64_t i0 = gi * SV;
        uint64_t k[SV];
        uint32_t vm = 0;
        if (gi < ngroups && i0 + SV <= n) {
            const Vec16<T> *vp = (const Vec16<T> *)col.d_values + i0 / VPT;
#pragma unroll
            for (int u = 0; u < NV; ++u) {
                const Vec16<T> v = vp[u];
#pragma unroll
                for (int e = 0; e < VPT; ++e) k[u * VPT + e] = Elem<T>::key(v.v[e]);
            }
            vm = valid_bits(col.d_validity, col.validity_bit_offset, i0, SV);
        } else {
#pragma unroll
            for (int e = 0; e < SV; ++e) {
                k[e] = 0;
                const int64_t i = i0 + e;
                if (gi < ngroups && i < n && sd_fetch<T>(col, i, k[e])) vm |= 1u << e;
            }
        }
        // changes inside the lane's rows (its first valid row counted as new)
        uint64_t prev = 0, fk = 0;
        bool have = false;
        uint32_t dl = 0;
#pragma unroll
        for (int e = 0; e < SV; ++e) {
            if ((vm >> e) & 1u) {
                dl += (!have || k[e] != prev);
                viol |= have && k[e] < prev;
                if (!have) fk = k[e];
                prev = k[e];
                have = true;
            }
        }
        if (vm) {
            first = min(first, i0 + (int64_t)__builtin_ctz(vm));
            last = max(last, i0 + 31 - (int64_t)__builtin_clz(vm));
        }
        // the key before this lane's first valid row: the left lane's last one
        const uint64_t lk = __shfl_up(prev, 1, WAVE);
        const bool lh = __shfl_up(have ? 1 : 0, 1, WAVE) != 0;
        if (vm) {
            uint64_t pk = lk;
            bool ph = lane > 0 && lh;
            if (!ph) {                                  // walk back over nulls
                int64_t j = i0 - 1;
                for (int w = 0; j >= 0 && w < SD_WALK; --j, ++w)
                    if (sd_fetch<T>(col, j, pk)) { ph = true; break; }
                if (!ph && j >= 0) viol = true;         // (a null run too long to walk)
            }
            if (ph) {
                dl -= (fk == pk);
                viol |= fk < pk;
            }
        }
        d += dl;
    }
    // one set of atomics per workgroup (per wave, 4 x 32 K same-address atomics
    // cost ~1 ms per launch whatever the column length)
    __shared__ uint64_t s_d[SD_T / WAVE];
    __shared__ int64_t s_f[SD_T / WAVE], s_l[SD_T / WAVE];
    __shared__ int s_v[SD_T / WAVE];
    const int wid = threadIdx.x / WAVE;
    d = wave_sum_u64(d);
    const bool any_viol = __any(viol);
    const int64_t fmin = wave_min_i64(first), lmax = wave_max_i64(last);
    if (lane == 0) { s_d[wid] = d; s_v[wid] = any_viol ? 1 : 0; s_f[wid] = fmin; s_l[wid] = lmax; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t bd = 0;
        int bv = 0;
        int64_t bf = INT64_MAX, bl = -1;
        for (int w = 0; w < SD_T / WAVE; ++w) {
            bd += s_d[w];
            bv |= s_v[w];
            bf = min(bf, s_f[w]);
            bl = max(bl, s_l[w]);
        }
        if (bd) atomicAdd((unsigned long long *)&out[0], (unsigned long long)bd);
        if (bv) atomicOr((unsigned long long *)&out[1], 1ull);
        if (bf != INT64_MAX) atomicMin((long long *)&out[2], (long long)bf);
        if (bl >= 0) atomicMax((long long *)&out[3], (long long)bl);
    }
}
__global__ void sorted_distinct_init_kernel(uint64_t *out) {
    out[0] = 0; out[1] = 0; out[2] = (uint64_t)INT64_MAX; out[3] = (uint64_t)(int64_t)-1;
}
template <typename T>
__global__ void sorted_distinct_final_kernel(sdp_column col, uint64_t *out) {
    const int64_t f = (int64_t)out[2], l = (int64_t)out[3];
    uint64_t k = EMPTY64;
    out[2] = (l >= 0 && sd_fetch<T>(col, f, k)) ? k : EMPTY64;
    k = EMPTY64;
    out[3] = (l >= 0 && sd_fetch<T>(col, l, k)) ? k : EMPTY64;
}

// ============================================================================
// pass 2: mad + histogram + outliers
// ============================================================================

constexpr int P2_BLOCK = 256;
constexpr int P2_UNROLL = 4;

constexpr int P2_SMALL_BINS = 16;
struct P2Ctx {
    double mean, hi_t, lo_t, e0, inv_w;
    const double *edges;      // LDS copy
    double ev[P2_SMALL_BINS]; // the edges again, wave-uniform (SGPRs), for the cumulative path
    int bins;
    bool monotone;
};

// bin per the CASE-WHEN chain (describe.py:46, :20-35); -1 = no branch matched
__device__ __forceinline__ int case_bin(const P2Ctx &c, double x) {
    const int b = c.bins;
    if (c.monotone) {
        if (!(x >= c.e0)) return -1;
        double f = (x - c.e0) * c.inv_w;
        int j = (f >= (double)(b - 1)) ? b - 1 : (f > 0.0 ? (int)f : 0);
        while (j + 1 < b && x >= c.edges[j + 1]) ++j;
        while (j > 0 && x < c.edges[j]) --j;
        return j;
    }
    for (int i = 0; i < b; ++i) {
        const bool cond = (i < b - 1) ? (spark_ge(x, c.edges[i]) && spark_lt(x, c.edges[i + 1]))
                                      : spark_ge(x, c.edges[i]);
        if (cond) return i;
    }
    return -1;
}


struct P2Thread {
    double mad;
    uint32_t high, low, unbinned, okc;
    uint32_t bc[P2_SMALL_BINS];       // wave-uniform bin counts (SGPRs) for bins <= 16
};

// SMALL: <= 16 bins counted per wave with ballots.  MONO (finite non-decreasing
// edges): bc[j] counts x >= e_j, one compare against a wave-uniform edge per
// bin and no bin search; the CASE-WHEN bins are differences of these
// cumulative counts (bin j = [e_j, e_j+1), last bin x >= e_b-1, x < e_0 unbinned),
// formed once per wave in the epilogue.
template <typename T, bool SMALL, bool MONO, int NB>
__device__ __forceinline__ void p2_elem(P2Thread &st, const P2Ctx &c, uint32_t *lds_hist, T x,
                                        bool valid) {
    const double xd = Elem<T>::d(x);
    const bool isnan_ = Elem<T>::is_float && (xd != xd);
    const bool ok = valid && !isnan_;
    if (valid) {
        st.high += spark_gt(xd, c.hi_t);
        st.low += spark_lt(xd, c.lo_t);
    }
    if (SMALL && MONO) {
        st.okc += ok;
        if (ok) st.mad += fabs(xd - c.mean);
        // per-lane counts (compare + add-with-carry each; summed over the wave
        // in the epilogue): wave ballots of every element of a tile ran out of
        // SGPRs.  A skipped element compares as -inf; unused edges are +inf
        // and their counts are never read.
        const double xv = ok ? xd : -__builtin_inf();
#pragma unroll
        for (int j = 0; j < NB; ++j) st.bc[j] += (uint32_t)(xv >= c.ev[j]);
        return;
    }
    int bin = -1;
    if (ok) {
        st.mad += fabs(xd - c.mean);
        bin = case_bin(c, xd);
        st.unbinned += (bin < 0);
    }
    if (SMALL) {
        // one compare + ballot per bin; counts stay wave-uniform (scalar unit)
#pragma unroll
        for (int j = 0; j < P2_SMALL_BINS; ++j)
            if (j < c.bins) st.bc[j] += (uint32_t)__popcll(__ballot(bin == j));
    } else {
        if (bin >= 0) atomicAdd(&lds_hist[bin], 1u);
    }
}

template <typename T, bool SMALL, bool MONO, int NB = P2_SMALL_BINS>
__global__ void __launch_bounds__(P2_BLOCK, 4) pass2_kernel(sdp_column col, double mean, const double *edges,
                                                         int bins, int monotone, double hi_t, double lo_t,
                                                         double *part_mad, uint64_t *part_cnt) {
    constexpr int VPT = Vec16<T>::N;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double *s_edges = (double *)smem;
    uint32_t *s_hist = (uint32_t *)(smem + sizeof(double) * bins);
    for (int i = threadIdx.x; i < bins; i += blockDim.x) { s_edges[i] = edges[i]; s_hist[i] = 0; }
    __syncthreads();
    P2Ctx c;
    c.mean = mean; c.hi_t = hi_t; c.lo_t = lo_t; c.edges = s_edges; c.bins = bins;
    c.monotone = monotone != 0;
    c.e0 = s_edges[0];
#pragma unroll
    for (int j = 0; j < P2_SMALL_BINS; ++j) c.ev[j] = j < bins ? edges[j] : __builtin_inf();   // uniform loads
    {
        const double w = (bins > 1) ? (s_edges[bins - 1] - s_edges[0]) / (double)(bins - 1) : 0.0;
        c.inv_w = (w > 0.0) ? 1.0 / w : 0.0;
    }
    P2Thread st;
    st.mad = 0.0; st.high = st.low = st.unbinned = st.okc = 0;
#pragma unroll
    for (int j = 0; j < P2_SMALL_BINS; ++j) st.bc[j] = 0;

    const int64_t n = col.length;
    const int64_t nvec = n / VPT;
    const Vec16<T> *vals = (const Vec16<T> *)col.d_values;
    // (wider tiles of the narrower types run out of registers)
    constexpr int U = sizeof(T) >= 8 ? P2_UNROLL : (std::is_same<T, float>::value ? P2_UNROLL / 2 : 1);
    const int64_t tile_vecs = (int64_t)P2_BLOCK * U;
    const int64_t ntiles = (nvec + tile_vecs - 1) / tile_vecs;
    (void)vals;
    const VBits vbm = vbits_init(col.d_validity, col.validity_bit_offset, col.d_values);
    VecIn<T> ta[U], tb[U];
    auto load = [&](VecIn<T> (&x)[U], int64_t tile) {
#pragma unroll
        for (int u = 0; u < U; ++u) x[u].load(vals, vbm, tile * tile_vecs + (int64_t)u * P2_BLOCK + threadIdx.x, nvec);
    };
    auto work = [&](const VecIn<T> (&x)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t vbits = x[u].bits(vbm);
#pragma unroll
            for (int e = 0; e < VPT; ++e) p2_elem<T, SMALL, MONO, NB>(st, c, s_hist, x[u].v.v[e], (vbits >> e) & 1u);
        }
    };
    int64_t tile = blockIdx.x;
    if (tile < ntiles) {
        load(ta, tile);
        while (true) {
            load(tb, tile + gridDim.x);         // next tile in flight (clamped past the end)
            work(ta);
            tile += gridDim.x;
            if (tile >= ntiles) break;
            load(ta, tile + gridDim.x);
            work(tb);
            tile += gridDim.x;
            if (tile >= ntiles) break;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < WAVE) {
        const int64_t i = nvec * VPT + threadIdx.x;
        const bool inb = i < n;
        T x = inb ? ((const T *)col.d_values)[i] : (T)0;
        const bool valid = inb && valid_bit(col.d_validity, col.validity_bit_offset, i);
        p2_elem<T, SMALL, MONO, NB>(st, c, s_hist, x, valid);
    }
    // ---- block reduction (fixed order) ----
    __shared__ double s_mad[P2_BLOCK / WAVE];
    __shared__ uint64_t s_u[P2_BLOCK / WAVE][3];
    const int wid = threadIdx.x / WAVE, lane = lane_id();
    const double mad = wave_sum_f64(st.mad);
    const uint64_t hi = wave_sum_u64(st.high), lo = wave_sum_u64(st.low);
    uint64_t ub = wave_sum_u64(st.unbinned);
    if (SMALL && MONO) {                // per-lane cumulative counts -> CASE-WHEN bins of the wave
#pragma unroll
        for (int j = 0; j < P2_SMALL_BINS; ++j) st.bc[j] = j < NB ? (uint32_t)wave_sum_u64(st.bc[j]) : 0u;
        ub = wave_sum_u64(st.okc) - st.bc[0];
#pragma unroll
        for (int j = 0; j < P2_SMALL_BINS - 1; ++j)
            if (j + 1 < bins) st.bc[j] -= st.bc[j + 1];
    }
    if (lane == 0) { s_mad[wid] = mad; s_u[wid][0] = hi; s_u[wid][1] = lo; s_u[wid][2] = ub; }
    if (SMALL && lane == 0) {
#pragma unroll
        for (int j = 0; j < P2_SMALL_BINS; ++j)
            if (j < bins && st.bc[j]) atomicAdd(&s_hist[j], st.bc[j]);
    }
    __syncthreads();
    const int stride = 3 + bins;
    if (threadIdx.x == 0) {
        double m = 0.0;
        uint64_t a = 0, b = 0, u = 0;
        for (int w = 0; w < P2_BLOCK / WAVE; ++w) { m += s_mad[w]; a += s_u[w][0]; b += s_u[w][1]; u += s_u[w][2]; }
        part_mad[blockIdx.x] = m;
        part_cnt[(int64_t)blockIdx.x * stride + 0] = a;
        part_cnt[(int64_t)blockIdx.x * stride + 1] = b;
        part_cnt[(int64_t)blockIdx.x * stride + 2] = u;
    }
    for (int i = threadIdx.x; i < bins; i += blockDim.x)
        part_cnt[(int64_t)blockIdx.x * stride + 3 + i] = s_hist[i];
}

// ---- pass 2 fused with the level-1 partition count --------------------------
// For a NUM column whose countDistinct (describe.py:143) takes the partitioning
// path, pass 2 also does the level-1 count of sdp_part_rows (phase 0) on the
// same read: block g streams rows [g * rpb, min(n, (g + 1) * rpb)) -- the row
// ranges of the partition scatter, so its per-block bucket histogram is the
// count kernel's -- doing pass 2's per-element work and, for every valid row,
// hashing the grouping key and counting it into the heavy-key table or the LDS
// bucket histogram.  One column read instead of two.
struct P2CountLds {
    HeavyLdsT<false> heavy;
    uint32_t hist[MAXB];
};

// block g of a G-block grid (the batched launch runs several columns' grids
// side by side, blockIdx.y = column)
template <typename T, bool SMALL, bool MONO, int NB>
__device__ __forceinline__ void pass2_count_body(const sdp_column &col, double mean, const double *edges, int bins,
                                                 int monotone, double hi_t, double lo_t, double *part_mad,
                                                 uint64_t *part_cnt, const HeavyArg &heavy, int b1,
                                                 int64_t rows_per_block, uint32_t *hist, uint64_t *heavy_counts,
                                                 uint64_t *stats, const int G, const int g, int64_t lo32 = 0) {
    constexpr int VPT = Vec16<T>::N;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ P2CountLds cl;
    double *s_edges = (double *)smem;
    uint32_t *s_hist = (uint32_t *)(smem + sizeof(double) * bins);
    const int t = threadIdx.x;
    // b1 < 0: the level-1 count of sdp_distinct32 (32-bit key spaces) instead
    const bool d32 = b1 < 0;
    const int nb = d32 ? D32_NB1 : 1 << b1;
    const int shift = d32 ? 0 : 64 - b1;
    for (int i = t; i < bins; i += blockDim.x) { s_edges[i] = edges[i]; s_hist[i] = 0; }
    for (int b = t; b < nb; b += P2_BLOCK) cl.hist[b] = 0;
    heavy_build<false>(cl.heavy, heavy);               // (ends with a barrier)
    P2Ctx c;
    c.mean = mean; c.hi_t = hi_t; c.lo_t = lo_t; c.edges = s_edges; c.bins = bins;
    c.monotone = monotone != 0;
    c.e0 = s_edges[0];
#pragma unroll
    for (int j = 0; j < P2_SMALL_BINS; ++j) c.ev[j] = j < bins ? edges[j] : __builtin_inf();
    {
        const double w = (bins > 1) ? (s_edges[bins - 1] - s_edges[0]) / (double)(bins - 1) : 0.0;
        c.inv_w = (w > 0.0) ? 1.0 / w : 0.0;
    }
    P2Thread st;
    st.mad = 0.0; st.high = st.low = st.unbinned = st.okc = 0;
#pragma unroll
    for (int j = 0; j < P2_SMALL_BINS; ++j) st.bc[j] = 0;
    uint64_t rows = 0, special = 0;
    const bool any_heavy = heavy.n > 0;
    auto count = [&](T x, bool valid) {
        if (!valid) return;
        ++rows;
        if constexpr (!std::is_same<T, double>::value) {
            if (d32) {
                atomicAdd(&cl.hist[mix32(key32_rel<T>(x, lo32)) >> (32 - D32_B1)], 1u);
                return;
            }
        } else {
            if (d32) return;        // no 32-bit key space for doubles (sdp.h: b1 = -1 is F32 / integral only)
        }
        const uint64_t h = mix64(key_of<T>(x));
        const int hv = any_heavy ? heavy_find_u64(cl.heavy, heavy.n, h) : -1;
        if (hv >= 0) atomicAdd(&cl.heavy.cnt[hv], 1u);
        else if (h == EMPTY64) ++special;              // the key whose hash is the empty marker
        else atomicAdd(&cl.hist[b1 ? (int)(h >> shift) : 0], 1u);
    };

    const int64_t n = col.length;
    const int64_t r0 = (int64_t)g * rows_per_block;    // a multiple of 16 K rows: whole vectors
    const int64_t r1 = min(n, r0 + rows_per_block);
    const int64_t v0 = r0 / VPT, v1 = r1 / VPT;        // whole vectors of this block's rows
    const Vec16<T> *vals = (const Vec16<T> *)col.d_values;
    // (doubles: two vectors per tile -- at four the fp64 moments, the hash and
    // the bin search spill 18 VGPRs: 18.1 -> 17.1 ms for six 1e9-row columns;
    // int64 measured flat, profiles/r04p2c_pass2_count_unroll_ab.log)
    constexpr int U = std::is_same<T, double>::value ? 2
                      : sizeof(T) >= 8 ? P2_UNROLL : (std::is_same<T, float>::value ? P2_UNROLL / 2 : 1);
    constexpr int64_t TV = (int64_t)P2_BLOCK * U;
    // ping-pong tiles of this block's whole vectors [v0, v1)
    const VBits vbm = vbits_init(col.d_validity, col.validity_bit_offset, col.d_values);
    VecIn<T> ta[U], tb[U];
    auto load = [&](VecIn<T> (&x)[U], int64_t vb) {
#pragma unroll
        for (int u = 0; u < U; ++u) x[u].load(vals, vbm, vb + (int64_t)u * P2_BLOCK + t, v1);
    };
    auto work = [&](const VecIn<T> (&x)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t vbits = x[u].bits(vbm);
#pragma unroll
            for (int e = 0; e < VPT; ++e) {
                const bool valid = (vbits >> e) & 1u;
                p2_elem<T, SMALL, MONO, NB>(st, c, s_hist, x[u].v.v[e], valid);
                count(x[u].v.v[e], valid);
            }
        }
    };
    int64_t vb = v0;
    if (vb < v1) {
        load(ta, vb);
        while (true) {
            load(tb, vb + TV);
            work(ta);
            vb += TV;
            if (vb >= v1) break;
            load(ta, vb + TV);
            work(tb);
            vb += TV;
            if (vb >= v1) break;
        }
    }
    if (r1 == n && t < WAVE) {                         // the column's last n % VPT rows (last block)
        const int64_t i = v1 * VPT + t;
        const bool inb = i < n;
        T x = inb ? ((const T *)col.d_values)[i] : (T)0;
        const bool valid = inb && valid_bit(col.d_validity, col.validity_bit_offset, i);
        p2_elem<T, SMALL, MONO, NB>(st, c, s_hist, x, valid);
        count(x, valid);
    }
    // ---- pass-2 block partial (as pass2_kernel) ----
    __shared__ double s_mad[P2_BLOCK / WAVE];
    __shared__ uint64_t s_u[P2_BLOCK / WAVE][3];
    const int wid = t / WAVE, lane = lane_id();
    const double mad = wave_sum_f64(st.mad);
    const uint64_t hi = wave_sum_u64(st.high), lo = wave_sum_u64(st.low);
    uint64_t ub = wave_sum_u64(st.unbinned);
    if (SMALL && MONO) {
#pragma unroll
        for (int j = 0; j < P2_SMALL_BINS; ++j) st.bc[j] = j < NB ? (uint32_t)wave_sum_u64(st.bc[j]) : 0u;
        ub = wave_sum_u64(st.okc) - st.bc[0];
#pragma unroll
        for (int j = 0; j < P2_SMALL_BINS - 1; ++j)
            if (j + 1 < bins) st.bc[j] -= st.bc[j + 1];
    }
    if (lane == 0) { s_mad[wid] = mad; s_u[wid][0] = hi; s_u[wid][1] = lo; s_u[wid][2] = ub; }
    if (SMALL && lane == 0) {
#pragma unroll
        for (int j = 0; j < P2_SMALL_BINS; ++j)
            if (j < bins && st.bc[j]) atomicAdd(&s_hist[j], st.bc[j]);
    }
    __syncthreads();
    const int stride = 3 + bins;
    if (t == 0) {
        double m = 0.0;
        uint64_t a = 0, b = 0, u = 0;
        for (int w = 0; w < P2_BLOCK / WAVE; ++w) { m += s_mad[w]; a += s_u[w][0]; b += s_u[w][1]; u += s_u[w][2]; }
        part_mad[g] = m;
        part_cnt[(int64_t)g * stride + 0] = a;
        part_cnt[(int64_t)g * stride + 1] = b;
        part_cnt[(int64_t)g * stride + 2] = u;
    }
    for (int i = t; i < bins; i += blockDim.x) part_cnt[(int64_t)g * stride + 3 + i] = s_hist[i];
    // ---- level-1 count outputs (as part_count_rows_u64_kernel) ----
    for (int b = t; b < nb; b += P2_BLOCK) hist[(int64_t)b * G + g] = cl.hist[b];
    if (d32) {                                         // sdp_distinct32's out[1]: non-null rows
        block_add_u64(rows, &stats[1]);
        return;
    }
    heavy_flush(cl.heavy, heavy.n, heavy_counts);
    block_add_u64(rows, &stats[0]);
    block_add_u64(special, &stats[1]);
}
template <typename T, bool SMALL, bool MONO, int NB = P2_SMALL_BINS>
__global__ void __launch_bounds__(P2_BLOCK, 4) pass2_count_kernel(sdp_column col, double mean, const double *edges,
                                                               int bins, int monotone, double hi_t, double lo_t,
                                                               double *part_mad, uint64_t *part_cnt, HeavyArg heavy,
                                                               int b1, int64_t rows_per_block, uint32_t *hist,
                                                               uint64_t *heavy_counts, uint64_t *stats) {
    pass2_count_body<T, SMALL, MONO, NB>(col, mean, edges, bins, monotone, hi_t, lo_t, part_mad, part_cnt, heavy, b1,
                                         rows_per_block, hist, heavy_counts, stats, (int)gridDim.x, (int)blockIdx.x);
}
template <typename T, bool SMALL, bool MONO, int NB = P2_SMALL_BINS>
__global__ void __launch_bounds__(P2_BLOCK, 4) pass2_count_batch_kernel(const sdp_pass2_task *tasks) {
    const sdp_pass2_task &tk = tasks[blockIdx.y];
    if ((int)blockIdx.x >= tk.grid) return;
    const HeavyArg hv{tk.heavy.d_h, nullptr, nullptr, nullptr, tk.heavy.n};
    double *pm = (double *)tk.d_work;
    uint64_t *pc = (uint64_t *)((char *)tk.d_work + (int64_t)tk.grid * sizeof(double));
    pass2_count_body<T, SMALL, MONO, NB>(tk.col, tk.mean, tk.d_edges, tk.bins, tk.edges_monotone, tk.hi_t, tk.lo_t,
                                         pm, pc, hv, tk.b1, tk.rows_per_block, tk.d_part_hist, tk.d_heavy_counts,
                                         tk.d_stats, tk.grid, (int)blockIdx.x, tk.key32_lo);
}

__device__ __forceinline__ void pass2_merge_body(const double *part_mad, const uint64_t *part_cnt, int grid,
                                                 int bins, sdp_pass2_result *out, uint64_t *hist);
__global__ void __launch_bounds__(MERGE_T) pass2_merge_kernel(const double *part_mad, const uint64_t *part_cnt,
                                                              int grid, int bins, sdp_pass2_result *out,
                                                              uint64_t *hist) {
    pass2_merge_body(part_mad, part_cnt, grid, bins, out, hist);
}
__global__ void __launch_bounds__(MERGE_T) pass2_merge_batch_kernel(const sdp_pass2_task *tasks) {
    const sdp_pass2_task &tk = tasks[blockIdx.x];
    pass2_merge_body((const double *)tk.d_work,
                     (const uint64_t *)((const char *)tk.d_work + (int64_t)tk.grid * sizeof(double)), tk.grid,
                     tk.bins, tk.d_result, tk.d_hist);
}
__device__ __forceinline__ void pass2_merge_body(const double *part_mad, const uint64_t *part_cnt, int grid,
                                                 int bins, sdp_pass2_result *out, uint64_t *hist) {
    __shared__ double sh[MERGE_T];
    __shared__ uint64_t su[MERGE_T];
    const int stride = 3 + bins;
    const int t = threadIdx.x;
    auto addu = [](uint64_t a, uint64_t b) { return a + b; };
    for (int f = 0; f < 3 + bins; ++f) {
        uint64_t a = 0;
        for (int b = t; b < grid; b += MERGE_T) a += part_cnt[(int64_t)b * stride + f];
        a = block_reduce(a, su, addu);
        if (t == 0) {
            if (f == 0) out->n_high = a;
            else if (f == 1) out->n_low = a;
            else if (f == 2) out->n_unbinned = a;
            else hist[f - 3] = a;
        }
    }
    double m = 0.0;
    for (int b = t; b < grid; b += MERGE_T) m += part_mad[b];
    m = block_reduce(m, sh, [](double x, double y) { return x + y; });
    if (t == 0) out->abs_dev_sum = m;
}

static int p2_grid(int64_t n, int dt) {
    const int vpt = 16 / elem_size(dt);
    const int64_t nvec = n / vpt;
    int64_t tiles = (nvec + (int64_t)P2_BLOCK * P2_UNROLL - 1) / ((int64_t)P2_BLOCK * P2_UNROLL);
    if (tiles < 1) tiles = 1;
    return (int)(tiles < 2048 ? tiles : 2048);
}

}  // namespace sdp

using namespace sdp;

// ============================================================================
// C ABI
// ============================================================================

extern "C" int32_t sdp_pass1_grid(int64_t length, int32_t dtype) {
    if (elem_size(dtype) == 0) return 0;
    return p1_grid(length, dtype);
}

extern "C" int64_t sdp_pass1_workspace_bytes(int64_t length, int32_t dtype) {
    if (elem_size(dtype) == 0) return -1;
    return (int64_t)p1_grid(length, dtype) * (int64_t)sizeof(P1Partial);
}

extern "C" int64_t sdp_pass2_workspace_bytes(int64_t length, int32_t dtype, int32_t bins) {
    if (elem_size(dtype) == 0 || bins < 1) return -1;
    const int64_t g = p2_grid(length, dtype);
    return g * (int64_t)sizeof(double) + g * (int64_t)(3 + bins) * (int64_t)sizeof(uint64_t);
}

extern "C" int sdp_sample_keys(const sdp_column *col, int32_t n_sample, uint64_t *d_sample, void *stream) {
    int rc = check_col(col, "sdp_sample_keys");
    if (rc) return rc;
    if (n_sample < 1 || n_sample > (1 << 22)) return set_error(SDP_EINVAL, "sdp_sample_keys: n_sample %d", n_sample);
    hipStream_t s = (hipStream_t)stream;
    const int blocks = (n_sample + 255) / 256;
    SDP_DISPATCH_NUMERIC(col->dtype,
        hipLaunchKernelGGL(sample_keys_kernel<T>, dim3(blocks), dim3(256), 0, s, *col, n_sample, d_sample));
    return check_launch("sample_keys_kernel");
}

extern "C" int sdp_sample_keys_batch(const sdp_column *d_cols, int32_t n_cols, int32_t n_sample, uint64_t *d_sample,
                                     void *stream) {
    if (d_cols == nullptr || n_cols < 1 || n_cols > 65535 || n_sample < 1 || n_sample > (1 << 22))
        return set_error(SDP_EINVAL, "sdp_sample_keys_batch: n_cols %d n_sample %d", n_cols, n_sample);
    hipLaunchKernelGGL(sample_keys_batch_kernel, dim3((n_sample + 255) / 256, n_cols), dim3(256), 0,
                       (hipStream_t)stream, d_cols, n_sample, d_sample);
    return check_launch("sample_keys_batch_kernel");
}

extern "C" int sdp_quantile_plan(uint64_t *d_sample, int32_t n_sample, const double *d_probs, int32_t n_probs,
                                 int32_t is_float, sdp_qplan *d_plan, void *stream) {
    if (n_sample < 1 || n_sample > SORT_MAX) return set_error(SDP_EINVAL, "sdp_quantile_plan: n_sample %d", n_sample);
    if (n_probs < 0 || n_probs > SDP_MAX_WINDOWS) return set_error(SDP_EINVAL, "sdp_quantile_plan: n_probs %d", n_probs);
    hipLaunchKernelGGL(quantile_plan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_sample, n_sample,
                       d_probs, n_probs, is_float, (const int32_t *)nullptr, d_plan);
    return check_launch("quantile_plan_kernel");
}

extern "C" int sdp_quantile_refine_batch(const uint64_t *d_samples2, int32_t n_sample2, int32_t n_cols,
                                         const double *d_probs, int32_t n_probs, sdp_qplan *d_plans, void *stream) {
    if (n_sample2 < 1 || n_cols < 1 || n_probs < 0 || n_probs > SDP_MAX_WINDOWS)
        return set_error(SDP_EINVAL, "sdp_quantile_refine_batch: n_sample2 %d n_cols %d", n_sample2, n_cols);
    hipLaunchKernelGGL(quantile_refine_kernel, dim3(n_cols), dim3(1024), 0, (hipStream_t)stream, d_samples2,
                       n_sample2, d_probs, n_probs, d_plans);
    return check_launch("quantile_refine_kernel");
}
extern "C" int sdp_quantile_plan_batch(uint64_t *d_samples, int32_t n_sample, int32_t n_cols, const double *d_probs,
                                       int32_t n_probs, const int32_t *d_is_float, sdp_qplan *d_plans,
                                       void *stream) {
    if (n_sample < 1 || n_sample > SORT_MAX) return set_error(SDP_EINVAL, "sdp_quantile_plan_batch: n_sample %d", n_sample);
    if (n_probs < 0 || n_probs > SDP_MAX_WINDOWS) return set_error(SDP_EINVAL, "sdp_quantile_plan_batch: n_probs %d", n_probs);
    if (n_cols < 1 || d_is_float == nullptr) return set_error(SDP_EINVAL, "sdp_quantile_plan_batch: n_cols %d", n_cols);
    hipLaunchKernelGGL(quantile_plan_kernel, dim3(n_cols), dim3(1024), 0, (hipStream_t)stream, d_samples, n_sample,
                       d_probs, n_probs, 0, d_is_float, d_plans);
    return check_launch("quantile_plan_kernel");
}

extern "C" int sdp_pass1(const sdp_column *col, const sdp_qplan *d_plan, void *d_work, int64_t work_bytes,
                         uint64_t *d_cand, uint32_t *d_cand_counts, int64_t slot_capacity, int32_t flags,
                         sdp_pass1_result *d_result, void *stream) {
    int rc = check_col(col, "sdp_pass1");
    if (rc) return rc;
    const int grid = p1_grid(col->length, col->dtype);
    if (work_bytes < (int64_t)grid * (int64_t)sizeof(P1Partial))
        return set_error(SDP_ECAP, "sdp_pass1: workspace %lld < %lld", (long long)work_bytes,
                         (long long)grid * (long long)sizeof(P1Partial));
    if (slot_capacity < 0 || slot_capacity > 0xFFFFFFFFll) return set_error(SDP_EINVAL, "sdp_pass1: slot_capacity");
    hipStream_t s = (hipStream_t)stream;
    P1Partial *parts = (P1Partial *)d_work;
    if (slot_capacity > 0 && (flags & SDP_PASS1_INCLUSIVE)) {
        SDP_DISPATCH_NUMERIC(col->dtype,
            hipLaunchKernelGGL((pass1_kernel<T, true, true>), dim3(grid), dim3(P1_BLOCK), 0, s, *col, d_plan, parts,
                               d_cand, d_cand_counts, slot_capacity));
    } else if (slot_capacity > 0) {
        SDP_DISPATCH_NUMERIC(col->dtype,
            hipLaunchKernelGGL((pass1_kernel<T, true>), dim3(grid), dim3(P1_BLOCK), 0, s, *col, d_plan, parts, d_cand,
                               d_cand_counts, slot_capacity));
    } else {            // no windows: moments / min / max only
        SDP_DISPATCH_NUMERIC(col->dtype,
            hipLaunchKernelGGL((pass1_kernel<T, false>), dim3(grid), dim3(P1_BLOCK), 0, s, *col, d_plan, parts,
                               d_cand, d_cand_counts, slot_capacity));
    }
    rc = check_launch("pass1_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(pass1_merge_kernel, dim3(1), dim3(MERGE_T), 0, s, parts, grid, d_plan, d_result);
    return check_launch("pass1_merge_kernel");
}

extern "C" int sdp_pass1_batch(const sdp_pass1_task *d_tasks, int32_t ntasks, int32_t dtype, int32_t windowed,
                               int32_t flags, int32_t max_grid, void *stream) {
    if (d_tasks == nullptr || ntasks < 1 || ntasks > 65535 || max_grid < 1 || max_grid > P1_MAX_GRID)
        return set_error(SDP_EINVAL, "sdp_pass1_batch: args");
    if (elem_size(dtype) <= 0 || dtype == SDP_BOOL) return set_error(SDP_EINVAL, "sdp_pass1_batch: dtype %d", dtype);
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(max_grid, ntasks);
    if (windowed && (flags & SDP_PASS1_INCLUSIVE)) {
        SDP_DISPATCH_NUMERIC(dtype,
            hipLaunchKernelGGL((pass1_batch_kernel<T, true, true>), grid, dim3(P1_BLOCK), 0, s, d_tasks));
    } else if (windowed) {
        SDP_DISPATCH_NUMERIC(dtype,
            hipLaunchKernelGGL((pass1_batch_kernel<T, true>), grid, dim3(P1_BLOCK), 0, s, d_tasks));
    } else {
        SDP_DISPATCH_NUMERIC(dtype,
            hipLaunchKernelGGL((pass1_batch_kernel<T, false>), grid, dim3(P1_BLOCK), 0, s, d_tasks));
    }
    int rc = check_launch("pass1_batch_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(pass1_merge_batch_kernel, dim3(ntasks), dim3(MERGE_T), 0, s, d_tasks);
    return check_launch("pass1_merge_batch_kernel");
}

extern "C" int sdp_compact_candidates(const uint64_t *d_cand, const uint32_t *d_cand_counts, int32_t nseg,
                                      int64_t slot_capacity, uint64_t *d_offsets_work, uint64_t *d_out,
                                      uint64_t *d_out_count, void *stream) {
    if (nseg < 1 || d_offsets_work == nullptr) return set_error(SDP_EINVAL, "sdp_compact_candidates: nseg %d", nseg);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(scan_counts_kernel, dim3(1), dim3(1024), 0, s, d_cand_counts, nseg, d_offsets_work,
                       d_out_count);
    int rc = check_launch("scan_counts_kernel");
    if (rc) return rc;
    const int grid = nseg < 65536 ? nseg : 65536;
    hipLaunchKernelGGL(copy_segments_kernel, dim3(grid), dim3(256), 0, s, d_cand, d_cand_counts, d_offsets_work,
                       nseg, slot_capacity, d_out);
    return check_launch("copy_segments_kernel");
}

extern "C" int sdp_radix_hist(const uint64_t *d_keys, const uint64_t *d_n, uint64_t prefix, int32_t shift,
                              uint64_t *d_hist, void *stream) {
    if (shift < 0 || shift > 63) return set_error(SDP_EINVAL, "sdp_radix_hist: shift %d", shift);
    hipLaunchKernelGGL(radix_hist_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, d_keys, d_n, prefix, shift,
                       d_hist);
    return check_launch("radix_hist_kernel");
}

extern "C" int sdp_radix_filter(const uint64_t *d_keys, const uint64_t *d_n, uint64_t prefix, int32_t shift,
                                uint64_t *d_out, uint64_t *d_out_n, void *stream) {
    if (shift < 0 || shift > 64) return set_error(SDP_EINVAL, "sdp_radix_filter: shift %d", shift);
    hipLaunchKernelGGL(radix_filter_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, d_keys, d_n, prefix,
                       shift, d_out, d_out_n);
    return check_launch("radix_filter_kernel");
}

static int64_t sel_align(int64_t x) { return (x + 255) / 256 * 256; }

extern "C" int64_t sdp_select_kth_workspace_bytes(int64_t n_cap) {
    if (n_cap < 0) return -1;
    return sel_align(sizeof(SelState)) + sel_align(2048 * 8) + 2 * sel_align(8) + 2 * sel_align(8 * (n_cap > 0 ? n_cap : 1));
}

struct SelWork {
    SelState *st;
    uint64_t *hist;
    uint64_t *cnt[2];
    uint64_t *buf[2];
};
static SelWork sel_layout(void *d_work, int64_t n_cap) {
    char *w = (char *)d_work;
    SelWork L;
    L.st = (SelState *)w;
    w += sel_align(sizeof(SelState));
    L.hist = (uint64_t *)w;
    w += sel_align(2048 * 8);
    L.cnt[0] = (uint64_t *)w;
    L.cnt[1] = (uint64_t *)(w + sel_align(8));
    w += 2 * sel_align(8);
    L.buf[0] = (uint64_t *)w;
    L.buf[1] = (uint64_t *)(w + sel_align(8 * (n_cap > 0 ? n_cap : 1)));
    return L;
}
static int sel_shift0(uint64_t lo_key, uint64_t hi_key) {
    const uint64_t x = lo_key ^ hi_key;
    return x ? ((63 - __builtin_clzll(x)) / 11) * 11 : 0;
}

extern "C" int sdp_select_kth(const uint64_t *d_keys, const uint64_t *d_n, int64_t n_cap, int64_t k,
                              uint64_t lo_key, uint64_t hi_key, void *d_work, int64_t work_bytes,
                              uint64_t *d_result, void *stream) {
    return select_kth_dev(d_keys, d_n, n_cap, k, nullptr, lo_key, hi_key, d_work, work_bytes, d_result, stream);
}

int select_kth_dev(const uint64_t *d_keys, const uint64_t *d_n, int64_t n_cap, int64_t k, const int64_t *d_k,
                   uint64_t lo_key, uint64_t hi_key, void *d_work, int64_t work_bytes, uint64_t *d_result,
                   void *stream) {
    if (n_cap < 0 || k < 0 || d_result == nullptr) return set_error(SDP_EINVAL, "sdp_select_kth: args");
    if (work_bytes < sdp_select_kth_workspace_bytes(n_cap)) return set_error(SDP_ECAP, "sdp_select_kth: workspace");
    const SelWork L = sel_layout(d_work, n_cap);
    const int shift0 = sel_shift0(lo_key, hi_key);
    const uint64_t prefix0 = shift0 + 11 < 64 ? (lo_key >> (shift0 + 11)) : 0ull;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(select_init_kernel, dim3(1), dim3(256), 0, s, L.st, prefix0, k, shift0, L.hist,
                       (const int64_t *)d_k);
    int rc = check_launch("select_init_kernel");
    if (rc) return rc;
    const uint64_t *cur = d_keys, *cur_n = d_n;
    hipLaunchKernelGGL(radix_hist_st_kernel, dim3(512), dim3(256), 0, s, cur, cur_n, L.st, L.hist);
    for (int shift = shift0, r = 0;; shift -= 11, ++r) {
        hipLaunchKernelGGL(radix_decide_kernel, dim3(1), dim3(1024), 0, s, L.hist, L.st,
                           shift ? L.cnt[r & 1] : nullptr, d_result);
        if ((rc = check_launch("radix_decide_kernel"))) return rc;
        if (shift == 0) break;
        hipLaunchKernelGGL(radix_filter_hist_st_kernel, dim3(512), dim3(256), 0, s, cur, cur_n, L.st, L.buf[r & 1],
                           L.cnt[r & 1], L.hist);
        if ((rc = check_launch("radix_filter_hist_st_kernel"))) return rc;
        cur = L.buf[r & 1];
        cur_n = L.cnt[r & 1];
    }
    return 0;
}

// ---- the same select, one round per call (row-sharded tables) ----------------------
// Every rank runs the same rounds on its own keys; between sdp_select_hist and
// sdp_select_step the caller all-reduces d_hist on the same stream (RCCL is
// stream-ordered), so the digit each rank's decide kernel picks is the global
// one and no round needs a host round trip.
extern "C" int sdp_select_rounds(uint64_t lo_key, uint64_t hi_key) { return sel_shift0(lo_key, hi_key) / 11 + 1; }

extern "C" int sdp_select_init(int64_t k, uint64_t lo_key, uint64_t hi_key, void *d_work, int64_t work_bytes,
                               int64_t n_cap, uint64_t *d_hist, void *stream) {
    if (n_cap < 0 || k < 0 || d_hist == nullptr) return set_error(SDP_EINVAL, "sdp_select_init: args");
    if (work_bytes < sdp_select_kth_workspace_bytes(n_cap)) return set_error(SDP_ECAP, "sdp_select_init: workspace");
    const SelWork L = sel_layout(d_work, n_cap);
    const int shift0 = sel_shift0(lo_key, hi_key);
    const uint64_t prefix0 = shift0 + 11 < 64 ? (lo_key >> (shift0 + 11)) : 0ull;
    hipLaunchKernelGGL(select_init_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, L.st, prefix0, k, shift0,
                       d_hist, (const int64_t *)nullptr);
    return check_launch("select_init_kernel");
}

static int sel_round_io(const uint64_t *d_keys, const uint64_t *d_n, const SelWork &L, int round,
                        const uint64_t *&cur, const uint64_t *&cur_n) {
    if (round < 0 || round > 5) return set_error(SDP_EINVAL, "sdp_select: round %d", round);
    cur = round == 0 ? d_keys : L.buf[(round - 1) & 1];
    cur_n = round == 0 ? d_n : L.cnt[(round - 1) & 1];
    return 0;
}

extern "C" int sdp_select_hist(const uint64_t *d_keys, const uint64_t *d_n, int64_t n_cap, int32_t round,
                               void *d_work, int64_t work_bytes, uint64_t *d_hist, void *stream) {
    if (work_bytes < sdp_select_kth_workspace_bytes(n_cap)) return set_error(SDP_ECAP, "sdp_select_hist: workspace");
    const SelWork L = sel_layout(d_work, n_cap);
    const uint64_t *cur, *cur_n;
    int rc = sel_round_io(d_keys, d_n, L, round, cur, cur_n);
    if (rc) return rc;
    hipLaunchKernelGGL(radix_hist_st_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, cur, cur_n, L.st, d_hist);
    return check_launch("radix_hist_st_kernel");
}

extern "C" int sdp_select_step(const uint64_t *d_keys, const uint64_t *d_n, int64_t n_cap, int32_t round,
                               int32_t last, void *d_work, int64_t work_bytes, uint64_t *d_hist, uint64_t *d_result,
                               void *stream) {
    if (d_result == nullptr || d_hist == nullptr) return set_error(SDP_EINVAL, "sdp_select_step: args");
    if (work_bytes < sdp_select_kth_workspace_bytes(n_cap)) return set_error(SDP_ECAP, "sdp_select_step: workspace");
    const SelWork L = sel_layout(d_work, n_cap);
    const uint64_t *cur, *cur_n;
    int rc = sel_round_io(d_keys, d_n, L, round, cur, cur_n);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(radix_decide_kernel, dim3(1), dim3(1024), 0, s, d_hist, L.st, last ? nullptr : L.cnt[round & 1],
                       d_result);
    if ((rc = check_launch("radix_decide_kernel"))) return rc;
    if (last) return 0;
    // survivors compacted and counted by the next digit: d_hist then holds the
    // local histogram of round + 1 (the caller all-reduces it before the next step)
    hipLaunchKernelGGL(radix_filter_hist_st_kernel, dim3(512), dim3(256), 0, s, cur, cur_n, L.st, L.buf[round & 1],
                       L.cnt[round & 1], d_hist);
    return check_launch("radix_filter_hist_st_kernel");
}

// ---- batched selects: every order statistic of every column of a table -------------
// One launch per stage for all Q tasks (blockIdx.y = task), so the selects of a
// whole table cost ~2 launches per radix round instead of ~2 per round per
// select (512 columns x 5 quantiles = 2560 selects in C5).  Task i keeps the
// workspace layout of sdp_select_kth in tasks[i].d_work and its round-r digit
// histogram at d_hist + 2048 i (the array a sharded caller all-reduces).
static __device__ __forceinline__ SelState *task_state(const sdp_select_task &t) { return (SelState *)t.d_work; }
static __device__ __forceinline__ int64_t sel_align_d(int64_t x) { return (x + 255) / 256 * 256; }
static __device__ __forceinline__ void task_io(const sdp_select_task &t, int round, const uint64_t *&cur,
                                               const uint64_t *&cur_n, uint64_t *&out, uint64_t *&out_n) {
    char *w = (char *)t.d_work + sel_align_d(sizeof(SelState)) + sel_align_d(2048 * 8);
    uint64_t *cnt0 = (uint64_t *)w, *cnt1 = (uint64_t *)(w + sel_align_d(8));
    w += 2 * sel_align_d(8);
    uint64_t *buf0 = (uint64_t *)w;
    uint64_t *buf1 = (uint64_t *)(w + sel_align_d(8 * (t.n_cap > 0 ? t.n_cap : 1)));
    cur = round == 0 ? t.d_keys : ((round - 1) & 1 ? buf1 : buf0);
    cur_n = round == 0 ? t.d_n : ((round - 1) & 1 ? cnt1 : cnt0);
    out = (round & 1) ? buf1 : buf0;
    out_n = (round & 1) ? cnt1 : cnt0;
}

__global__ void select_init_batch_kernel(const sdp_select_task *tasks, uint64_t *hist) {
    const sdp_select_task t = tasks[blockIdx.x];
    SelState *st = task_state(t);
    if (threadIdx.x == 0) {
        // the first digit is the 11 highest bits in which the window's keys can
        // differ (msb - 10 .. msb), later digits 11 bits each, the last one
        // what is left (same number of rounds as 11-bit digits aligned at
        // multiples of 11: 1 + msb / 11).  Aligned digits left a window whose
        // keys differ in bits 44-45 (f32 quantile windows) 4 of 2048 buckets
        // in round 0, so up to half the candidates survived into round 1.
        const uint64_t x = t.lo_key ^ t.hi_key;
        const int msb = x ? 63 - __clzll((long long)x) : 0;
        const int shift0 = msb >= 11 ? msb - 10 : 0;
        st->prefix = shift0 + 11 < 64 ? (t.lo_key >> (shift0 + 11)) : 0ull;
        st->k = t.k;
        st->shift = shift0;
        st->width = 11;
        st->done = 0;
        st->result = EMPTY64;
    }
    uint64_t *h = hist + (int64_t)blockIdx.x * 2048;
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) h[i] = 0;
}

__global__ void radix_hist_batch_kernel(const sdp_select_task *tasks, int round, uint64_t *hist) {
    const sdp_select_task t = tasks[blockIdx.y];
    const SelState *st = task_state(t);
    if (st->done) return;
    const uint64_t *keys, *n_ptr;
    uint64_t *o, *on;
    task_io(t, round, keys, n_ptr, o, on);
    __shared__ uint32_t h[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t n = *n_ptr, prefix = st->prefix;
    const int shift = st->shift, top = shift + st->width;
    const uint64_t dmask = (1ull << st->width) - 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    constexpr int R = 4;
    for (; i + (R - 1) * stride < n; i += R * stride) {
        uint64_t k[R];
#pragma unroll
        for (int r = 0; r < R; ++r) k[r] = keys[i + r * stride];
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (top >= 64 || (k[r] >> top) == prefix) atomicAdd(&h[(k[r] >> shift) & dmask], 1u);
    }
    for (; i < n; i += stride) {
        const uint64_t k = keys[i];
        if (top >= 64 || (k >> top) == prefix) atomicAdd(&h[(k >> shift) & dmask], 1u);
    }
    __syncthreads();
    uint64_t *gh = hist + (int64_t)blockIdx.y * 2048;
    for (int i = threadIdx.x; i < 2048; i += blockDim.x)
        if (h[i]) atomicAdd((unsigned long long *)&gh[i], (unsigned long long)h[i]);
}

__global__ void __launch_bounds__(1024) radix_decide_batch_kernel(const sdp_select_task *tasks, int round,
                                                                  uint64_t *hist) {
    const sdp_select_task t = tasks[blockIdx.x];
    const uint64_t *c, *cn;
    uint64_t *o, *on;
    task_io(t, round, c, cn, o, on);
    // (the decide body of the single-select path; a task that finished in an
    // earlier round returns at once)
    SelState *st = task_state(t);
    if (st->done) return;
    uint64_t *hh = hist + (int64_t)blockIdx.x * 2048;
    __shared__ uint64_t sm[1024];
    __shared__ int s_j;
    __shared__ uint64_t s_before;
    const int th = threadIdx.x;
    const uint64_t a = hh[2 * th], b = hh[2 * th + 1];
    sm[th] = a + b;
    if (th == 0) { s_j = -1; s_before = 0; }
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const uint64_t v = th >= off ? sm[th - off] : 0;
        __syncthreads();
        sm[th] += v;
        __syncthreads();
    }
    const uint64_t k = (uint64_t)st->k;
    const uint64_t excl = sm[th] - a - b;
    if (excl <= k && k < sm[th]) {
        s_j = k < excl + a ? 2 * th : 2 * th + 1;
        s_before = k < excl + a ? excl : excl + a;
    }
    __syncthreads();
    hh[2 * th] = 0;
    hh[2 * th + 1] = 0;
    if (th == 0) {
        if (s_j < 0) {
            st->done = 1;
            st->result = EMPTY64;
            *t.d_result = EMPTY64;
        } else {
            st->k = (int64_t)(k - s_before);
            st->prefix = (st->shift + st->width >= 64 ? 0ull : (st->prefix << st->width)) | (uint64_t)s_j;
            if (st->shift == 0) {
                st->done = 1;
                st->result = st->prefix;
                *t.d_result = st->prefix;
            } else {
                st->width = st->shift < 11 ? st->shift : 11;
                st->shift -= st->width;
            }
        }
        *on = 0;                                   // the next round's survivor count
    }
}

__global__ void radix_filter_hist_batch_kernel(const sdp_select_task *tasks, int round, uint64_t *hist) {
    const sdp_select_task t = tasks[blockIdx.y];
    const SelState *st = task_state(t);
    if (st->done) return;
    const uint64_t *keys, *n_ptr;
    uint64_t *out, *out_n;
    task_io(t, round, keys, n_ptr, out, out_n);
    __shared__ uint64_t s_buf[STAGE];
    __shared__ uint32_t s_cnt;
    __shared__ uint64_t s_gbase;
    __shared__ uint32_t h[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) h[i] = 0;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    Stager sg{s_buf, &s_cnt, &s_gbase};
    const uint64_t n = *n_ptr, prefix = st->prefix;
    const int shift = st->shift, top = shift + st->width;
    const uint64_t dmask = (1ull << st->width) - 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // R keys per thread loaded before any is pushed: R loads in flight, not one
    constexpr int R = 4;
    const uint64_t iters = (n + R * stride - 1) / (R * stride);
    for (uint64_t it = 0; it < iters; ++it) {
        const uint64_t i0 = it * R * stride + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        uint64_t k[R];
#pragma unroll
        for (int r = 0; r < R; ++r) k[r] = i0 + r * stride < n ? keys[i0 + r * stride] : 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool keep = i0 + r * stride < n && (top >= 64 || (k[r] >> top) == prefix);
            if (keep) atomicAdd(&h[(k[r] >> shift) & dmask], 1u);
            stage_push(sg, keep, k[r], out, (unsigned long long *)out_n, it + 1 == iters && r == R - 1);
        }
    }
    __syncthreads();
    uint64_t *gh = hist + (int64_t)blockIdx.y * 2048;
    for (int i = threadIdx.x; i < 2048; i += blockDim.x)
        if (h[i]) atomicAdd((unsigned long long *)&gh[i], (unsigned long long)h[i]);
}

// Batched candidate compaction: task i scans its segment counts (one
// workgroup) and copies its segments (grid.x workgroups) -- two launches for
// every window of every column.
__global__ void __launch_bounds__(1024) scan_counts_batch_kernel(const sdp_compact_task *tasks) {
    const sdp_compact_task t = tasks[blockIdx.x];
    __shared__ uint64_t sm[1024];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t base = 0; base < t.nseg; base += 1024) {
        const int64_t i = base + threadIdx.x;
        const uint64_t v = i < t.nseg ? t.d_counts[i] : 0;
        sm[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const uint64_t x = threadIdx.x >= o ? sm[threadIdx.x - o] : 0;
            __syncthreads();
            sm[threadIdx.x] += x;
            __syncthreads();
        }
        if (i < t.nseg) t.d_offsets_work[i] = carry + sm[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += sm[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *t.d_out_count = carry;
}

__global__ void copy_segments_batch_kernel(const sdp_compact_task *tasks) {
    const sdp_compact_task t = tasks[blockIdx.y];
    for (int64_t b = blockIdx.x; b < t.nseg; b += gridDim.x) {
        const uint32_t c = t.d_counts[b];
        const uint64_t base = t.d_offsets_work[b];
        const uint64_t *src = t.d_cand + b * t.cap;
        for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) t.d_out[base + i] = src[i];
    }
}

static int select_batch_blocks(int32_t q) {
    int hb = (16384 + q - 1) / q;      // ~16 K workgroups: the largest windows get enough of them
    return hb < 16 ? 16 : (hb > 512 ? 512 : hb);
}

extern "C" int sdp_compact_batch(const sdp_compact_task *d_tasks, int32_t q, int64_t max_nseg, void *stream) {
    if (q < 1 || max_nseg < 1) return set_error(SDP_EINVAL, "sdp_compact_batch: q %d max_nseg %lld", q,
                                                 (long long)max_nseg);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(scan_counts_batch_kernel, dim3((unsigned)q), dim3(1024), 0, s, d_tasks);
    int rc = check_launch("scan_counts_batch_kernel");
    if (rc) return rc;
    const int64_t gx = max_nseg < 1024 ? max_nseg : 1024;
    hipLaunchKernelGGL(copy_segments_batch_kernel, dim3((unsigned)gx, (unsigned)q), dim3(256), 0, s, d_tasks);
    return check_launch("copy_segments_batch_kernel");
}

extern "C" int sdp_select_batch_init(const sdp_select_task *d_tasks, int32_t q, uint64_t *d_hist, void *stream) {
    if (q < 1 || d_hist == nullptr) return set_error(SDP_EINVAL, "sdp_select_batch_init: q %d", q);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(select_init_batch_kernel, dim3((unsigned)q), dim3(256), 0, s, d_tasks, d_hist);
    int rc = check_launch("select_init_batch_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(radix_hist_batch_kernel, dim3((unsigned)select_batch_blocks(q), (unsigned)q), dim3(256), 0, s,
                       d_tasks, 0, d_hist);
    return check_launch("radix_hist_batch_kernel");
}

extern "C" int sdp_select_batch_step(const sdp_select_task *d_tasks, int32_t q, int32_t round, int32_t last,
                                     uint64_t *d_hist, void *stream) {
    if (q < 1 || round < 0 || round > 5 || d_hist == nullptr)
        return set_error(SDP_EINVAL, "sdp_select_batch_step: q %d round %d", q, round);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(radix_decide_batch_kernel, dim3((unsigned)q), dim3(1024), 0, s, d_tasks, round, d_hist);
    int rc = check_launch("radix_decide_batch_kernel");
    if (rc || last) return rc;
    hipLaunchKernelGGL(radix_filter_hist_batch_kernel, dim3((unsigned)select_batch_blocks(q), (unsigned)q), dim3(256),
                       0, s, d_tasks, round, d_hist);
    return check_launch("radix_filter_hist_batch_kernel");
}

extern "C" int sdp_select_batch(const sdp_select_task *d_tasks, int32_t q, int32_t rounds, uint64_t *d_hist,
                                void *stream) {
    if (rounds < 1 || rounds > 6) return set_error(SDP_EINVAL, "sdp_select_batch: rounds %d", rounds);
    int rc = sdp_select_batch_init(d_tasks, q, d_hist, stream);
    for (int r = 0; r < rounds && !rc; ++r) rc = sdp_select_batch_step(d_tasks, q, r, r == rounds - 1, d_hist, stream);
    return rc;
}

extern "C" int sdp_sort_small(uint64_t *d_keys, const uint64_t *d_n, void *stream) {
    hipLaunchKernelGGL(sort_small_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_keys, d_n);
    return check_launch("sort_small_kernel");
}

extern "C" int sdp_sort_small_batch(uint64_t *d_keys, int32_t n_each, int32_t n_sets, void *stream) {
    if (n_each < 1 || n_each > SORT_MAX || n_sets < 1)
        return set_error(SDP_EINVAL, "sdp_sort_small_batch: n_each %d n_sets %d", n_each, n_sets);
    hipLaunchKernelGGL(sort_small_batch_kernel, dim3(n_sets), dim3(1024), 0, (hipStream_t)stream, d_keys, n_each);
    return check_launch("sort_small_batch_kernel");
}

extern "C" int sdp_column_keys_range(const sdp_column *col, uint64_t lo_key, uint64_t hi_key, uint64_t *d_out,
                                     uint64_t *d_out_n, void *stream) {
    int rc = check_col(col, "sdp_column_keys_range");
    if (rc) return rc;
    if (d_out == nullptr || d_out_n == nullptr) return set_error(SDP_EINVAL, "sdp_column_keys_range: outputs");
    hipStream_t s = (hipStream_t)stream;
    SDP_DISPATCH_NUMERIC(col->dtype,
        hipLaunchKernelGGL(column_keys_kernel<T>, dim3(1024), dim3(256), 0, s, *col, lo_key, hi_key, d_out, d_out_n));
    return check_launch("column_keys_kernel");
}

extern "C" int sdp_sorted_distinct(const sdp_column *col, uint64_t *d_out, void *stream) {
    int rc = check_col(col, "sdp_sorted_distinct");
    if (rc) return rc;
    if (d_out == nullptr) return set_error(SDP_EINVAL, "sdp_sorted_distinct: output");
    hipStream_t s = (hipStream_t)stream;
    // (check_col has rejected every dtype SDP_DISPATCH_NUMERIC lacks, so no
    // kernel below is queued for a column that then fails dispatch)
    hipLaunchKernelGGL(sorted_distinct_init_kernel, dim3(1), dim3(1), 0, s, d_out);
    rc = check_launch("sorted_distinct_init_kernel");
    if (rc) return rc;
    const int64_t groups = (col->length + SD_V - 1) / SD_V;
    // (2048 workgroups: one resident round, eight per CU)
    const int grid = (int)std::min<int64_t>(std::max<int64_t>((groups + SD_T - 1) / SD_T, 1), 2048);
    SDP_DISPATCH_NUMERIC(col->dtype,
        hipLaunchKernelGGL(sorted_distinct_kernel<T>, dim3(grid), dim3(SD_T), 0, s, *col, d_out);
        hipLaunchKernelGGL(sorted_distinct_final_kernel<T>, dim3(1), dim3(1), 0, s, *col, d_out));
    return check_launch("sorted_distinct_kernel");
}

extern "C" int sdp_column_keys(const sdp_column *col, uint64_t *d_out, uint64_t *d_out_n, void *stream) {
    return sdp_column_keys_range(col, 0ull, ~0ull, d_out, d_out_n, stream);
}

extern "C" int64_t sdp_pass2_count_workspace_bytes(int64_t length, int32_t bins) {
    if (length < 0 || bins < 1) return -1;
    const int64_t rpb = sdp_part_rows_per_block(length, 0);
    const int64_t g = (length + rpb - 1) / rpb < 1 ? 1 : (length + rpb - 1) / rpb;
    return g * (int64_t)sizeof(double) + g * (int64_t)(3 + bins) * (int64_t)sizeof(uint64_t);
}

extern "C" int sdp_pass2_count(const sdp_column *col, double mean, const double *d_edges, int32_t bins,
                               int32_t edges_monotone, double hi_t, double lo_t, void *d_work, int64_t work_bytes,
                               sdp_pass2_result *d_result, uint64_t *d_hist, const sdp_heavy *heavy, int32_t b1,
                               uint32_t *d_part_hist, uint64_t *d_heavy_counts, uint64_t *d_stats, void *stream) {
    int rc = check_col(col, "sdp_pass2_count");
    if (rc) return rc;
    if (bins < 2 || bins > 8192) return set_error(SDP_EINVAL, "sdp_pass2_count: bins %d", bins);
    if (b1 < 0 || b1 > 10 || d_part_hist == nullptr || d_stats == nullptr)
        return set_error(SDP_EINVAL, "sdp_pass2_count: b1 %d / outputs", b1);
    HeavyArg hv{nullptr, nullptr, nullptr, nullptr, 0};
    if (heavy && heavy->n > 0) {
        if (heavy->n > HEAVY_MAX || d_heavy_counts == nullptr)
            return set_error(SDP_EINVAL, "sdp_pass2_count: %d heavy keys", heavy->n);
        hv = HeavyArg{heavy->d_h, nullptr, nullptr, nullptr, heavy->n};
    }
    const int64_t n = col->length;
    const int64_t rpb = sdp_part_rows_per_block(n, 0);
    const int grid = (int)((n + rpb - 1) / rpb < 1 ? 1 : (n + rpb - 1) / rpb);
    const int64_t need = sdp_pass2_count_workspace_bytes(n, bins);
    if (work_bytes < need) return set_error(SDP_ECAP, "sdp_pass2_count: workspace %lld < %lld",
                                            (long long)work_bytes, (long long)need);
    double *pm = (double *)d_work;
    uint64_t *pc = (uint64_t *)((char *)d_work + (int64_t)grid * sizeof(double));
    const size_t lds = (size_t)bins * (sizeof(double) + sizeof(uint32_t)) + 16;
    hipStream_t s = (hipStream_t)stream;
#define SDP_P2C(SM, MO, ...) \
    hipLaunchKernelGGL((pass2_count_kernel<T, SM, MO, ##__VA_ARGS__>), dim3(grid), dim3(P2_BLOCK), lds, s, *col, mean, \
                       d_edges, bins, edges_monotone, hi_t, lo_t, pm, pc, hv, b1, rpb, d_part_hist, d_heavy_counts, \
                       d_stats)
    if (bins <= 10 && edges_monotone) {
        SDP_DISPATCH_NUMERIC(col->dtype, SDP_P2C(true, true, 10));
    } else if (bins <= P2_SMALL_BINS && edges_monotone) {
        SDP_DISPATCH_NUMERIC(col->dtype, SDP_P2C(true, true));
    } else if (bins <= P2_SMALL_BINS) {
        SDP_DISPATCH_NUMERIC(col->dtype, SDP_P2C(true, false));
    } else {
        SDP_DISPATCH_NUMERIC(col->dtype, SDP_P2C(false, false));
    }
#undef SDP_P2C
    rc = check_launch("pass2_count_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(pass2_merge_kernel, dim3(1), dim3(MERGE_T), 0, s, pm, pc, grid, bins, d_result, d_hist);
    return check_launch("pass2_merge_kernel");
}

extern "C" int sdp_pass2_count_batch(const sdp_pass2_task *d_tasks, int32_t ntasks, int32_t dtype, int32_t bins,
                                     int32_t edges_monotone, int32_t max_grid, void *stream) {
    if (d_tasks == nullptr || ntasks < 1 || ntasks > 65535 || max_grid < 1 || bins < 2 || bins > 8192)
        return set_error(SDP_EINVAL, "sdp_pass2_count_batch: args");
    if (elem_size(dtype) <= 0) return set_error(SDP_EINVAL, "sdp_pass2_count_batch: dtype %d", dtype);
    const size_t lds = (size_t)bins * (sizeof(double) + sizeof(uint32_t)) + 16;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(max_grid, ntasks);
#define SDP_P2CB(SM, MO, ...) \
    hipLaunchKernelGGL((pass2_count_batch_kernel<T, SM, MO, ##__VA_ARGS__>), grid, dim3(P2_BLOCK), lds, s, d_tasks)
    if (bins <= 10 && edges_monotone) {
        SDP_DISPATCH_NUMERIC(dtype, SDP_P2CB(true, true, 10));
    } else if (bins <= P2_SMALL_BINS && edges_monotone) {
        SDP_DISPATCH_NUMERIC(dtype, SDP_P2CB(true, true));
    } else if (bins <= P2_SMALL_BINS) {
        SDP_DISPATCH_NUMERIC(dtype, SDP_P2CB(true, false));
    } else {
        SDP_DISPATCH_NUMERIC(dtype, SDP_P2CB(false, false));
    }
#undef SDP_P2CB
    int rc = check_launch("pass2_count_batch_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(pass2_merge_batch_kernel, dim3(ntasks), dim3(MERGE_T), 0, s, d_tasks);
    return check_launch("pass2_merge_batch_kernel");
}

extern "C" int sdp_pass2(const sdp_column *col, double mean, const double *d_edges, int32_t bins,
                         int32_t edges_monotone, double hi_t, double lo_t, void *d_work, int64_t work_bytes,
                         sdp_pass2_result *d_result, uint64_t *d_hist, void *stream) {
    int rc = check_col(col, "sdp_pass2");
    if (rc) return rc;
    if (bins < 2 || bins > 8192) return set_error(SDP_EINVAL, "sdp_pass2: bins %d", bins);
    const int grid = p2_grid(col->length, col->dtype);
    const int64_t need = sdp_pass2_workspace_bytes(col->length, col->dtype, bins);
    if (work_bytes < need) return set_error(SDP_ECAP, "sdp_pass2: workspace %lld < %lld", (long long)work_bytes,
                                            (long long)need);
    double *pm = (double *)d_work;
    uint64_t *pc = (uint64_t *)((char *)d_work + (int64_t)grid * sizeof(double));
    const size_t lds = (size_t)bins * (sizeof(double) + sizeof(uint32_t)) + 16;
    hipStream_t s = (hipStream_t)stream;
    if (bins <= 10 && edges_monotone) {          // describe()'s default bins=10
        SDP_DISPATCH_NUMERIC(col->dtype,
            hipLaunchKernelGGL((pass2_kernel<T, true, true, 10>), dim3(grid), dim3(P2_BLOCK), lds, s, *col, mean,
                               d_edges, bins, edges_monotone, hi_t, lo_t, pm, pc));
    } else if (bins <= P2_SMALL_BINS && edges_monotone) {
        SDP_DISPATCH_NUMERIC(col->dtype,
            hipLaunchKernelGGL((pass2_kernel<T, true, true>), dim3(grid), dim3(P2_BLOCK), lds, s, *col, mean,
                               d_edges, bins, edges_monotone, hi_t, lo_t, pm, pc));
    } else if (bins <= P2_SMALL_BINS) {
        SDP_DISPATCH_NUMERIC(col->dtype,
            hipLaunchKernelGGL((pass2_kernel<T, true, false>), dim3(grid), dim3(P2_BLOCK), lds, s, *col, mean,
                               d_edges, bins, edges_monotone, hi_t, lo_t, pm, pc));
    } else {
        SDP_DISPATCH_NUMERIC(col->dtype,
            hipLaunchKernelGGL((pass2_kernel<T, false, false>), dim3(grid), dim3(P2_BLOCK), lds, s, *col, mean,
                               d_edges, bins, edges_monotone, hi_t, lo_t, pm, pc));
    }
    rc = check_launch("pass2_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(pass2_merge_kernel, dim3(1), dim3(MERGE_T), 0, s, pm, pc, grid, bins, d_result, d_hist);
    return check_launch("pass2_merge_kernel");
}

// ============================================================================
// Spark 2.x percentile_approx emulation (opt-in; describe(quantile_mode='gk'))
// ============================================================================
// Replaces describe.py:205-206's percentile_approx(c, p) element by element
// for a given partitioning: ApproximatePercentile's QuantileSummaries
// (relativeError = 1/accuracy, head buffer 50000, compress threshold 10000),
// restated from Spark 2.1-2.4 (oracle/gk.py holds the CPU restatement the
// tests compare against, bit for bit).  One workgroup per Spark partition walks
// the partition's rows in order: every 50000 non-null, non-NaN values form a
// head batch, sorted in LDS chunks and merged; the batch is merged into the
// samples by binary-search ranks (all threads), then compressImmut's greedy
// scan runs on one thread (it is sequential by definition).  A second kernel
// merges the partition summaries in partition order and answers the queries.
// The GK state is tiny; the cost is the sequential compress scans, which makes
// this a correctness mode, not the default (the default returns the exact
// element at rank ceil(pN), inside Spark's rank window).
constexpr int GK_T = 1024;
constexpr int GK_HEAD = 50000;          // QuantileSummaries.defaultHeadSize
constexpr int GK_COMPRESS = 10000;      // defaultCompressThreshold (every full head exceeds it)
constexpr int GK_CHUNK = 12500;         // a head is sorted as four LDS chunks (<= SORT_MAX)
constexpr int64_t GK_CAP = 1 << 18;     // samples per partition buffer
constexpr int64_t GK_HBUF = 65536;      // head keys per buffer

struct GkPart {                         // one partition's state in the workspace
    int64_t len, count, which, status;  // samples, values seen, current buffer (0/1), error
};
struct GkView {                         // structure-of-arrays samples
    double *v;
    int64_t *g, *d;
};

__device__ __forceinline__ uint64_t gk_key(double v) {          // java.lang.Double.compare order
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double gk_val(uint64_t k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k));
}

// workspace layout: [P] GkPart | per partition: headA, headB (GK_HBUF u64 each),
// two sample buffers (GK_CAP x (v, g, d)) | merge: two buffers of 2*GK_CAP samples
__host__ __device__ inline int64_t gk_part_bytes() { return 2 * GK_HBUF * 8 + 2 * GK_CAP * 24; }
__host__ __device__ inline int64_t gk_head_off(int P) { return ((int64_t)P * (int64_t)sizeof(GkPart) + 255) / 256 * 256; }
__device__ GkView gk_view(uint8_t *base, int64_t cap) {
    GkView w;
    w.v = (double *)base;
    w.g = (int64_t *)(base + cap * 8);
    w.d = (int64_t *)(base + cap * 16);
    return w;
}

// number of a[0..n) (numerically non-decreasing) with a[i] < x (strict) or <= x
__device__ __forceinline__ int64_t gk_count_lt(const double *a, int64_t n, double x, bool le) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (le ? (a[mid] <= x) : (a[mid] < x)) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int64_t gk_count_key(const uint64_t *a, int64_t n, uint64_t x, bool le) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (le ? (a[mid] <= x) : (a[mid] < x)) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// compressImmut(in[0..L), thr) by thread 0 into out[w..L) (written from the end);
// the caller copies it to the front.  Returns w (all threads).
__device__ int64_t gk_compress(const GkView in, int64_t L, double thr, GkView out, int64_t *s_w) {
    if (threadIdx.x == 0) {
        int64_t w = L;
        if (L > 0) {
            double hv = in.v[L - 1];
            int64_t hg = in.g[L - 1], hd = in.d[L - 1];
            for (int64_t i = L - 2; i >= 1; --i) {
                const int64_t g1 = in.g[i];
                if ((double)(g1 + hg + hd) < thr) {
                    hg += g1;
                } else {
                    --w; out.v[w] = hv; out.g[w] = hg; out.d[w] = hd;
                    hv = in.v[i]; hg = g1; hd = in.d[i];
                }
            }
            --w; out.v[w] = hv; out.g[w] = hg; out.d[w] = hd;
            if (in.v[0] <= hv && L > 1) { --w; out.v[w] = in.v[0]; out.g[w] = in.g[0]; out.d[w] = in.d[0]; }
        }
        *s_w = w;
    }
    __syncthreads();
    return *s_w;
}
__device__ void gk_copy(const GkView src, int64_t from, int64_t n, GkView dst) {
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        dst.v[i] = src.v[from + i]; dst.g[i] = src.g[from + i]; dst.d[i] = src.d[from + i];
    }
    __syncthreads();
}

// sorted head keys (hn) merged into samples cur[0..len) -> nxt[0..len + hn)
// (withHeadBufferInserted), count = values before this head
__device__ void gk_insert(const uint64_t *H, int64_t hn, const GkView cur, int64_t len, int64_t count, double eps,
                          GkView nxt) {
    for (int64_t i = threadIdx.x; i < len; i += blockDim.x) {
        // batch values strictly below s_i come first (s_i <= x emits s_i before x)
        int64_t lo = 0, hi = hn;
        const double s = cur.v[i];
        while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (gk_val(H[mid]) < s) lo = mid + 1; else hi = mid; }
        const int64_t p = i + lo;
        nxt.v[p] = s; nxt.g[p] = cur.g[i]; nxt.d[p] = cur.d[i];
    }
    for (int64_t j = threadIdx.x; j < hn; j += blockDim.x) {
        const double x = gk_val(H[j]);
        const int64_t c = gk_count_lt(cur.v, len, x, true);
        const int64_t p = j + c;
        const bool zero = p == 0 || (j == hn - 1 && c == len);
        nxt.v[p] = x; nxt.g[p] = 1;
        nxt.d[p] = zero ? 0 : (int64_t)floor(2 * eps * (double)(count + j + 1));
    }
    __syncthreads();
}

// sort H[0..hn) (hn <= GK_HEAD): four LDS chunks, then two rounds of merges via B
__device__ void gk_sort_head(uint64_t *H, uint64_t *B, int64_t hn, uint64_t *s) {
    int64_t cs[5];
    int nc = 0;
    for (int64_t st = 0; st < hn; st += GK_CHUNK) {
        const int m = (int)min((int64_t)GK_CHUNK, hn - st);
        for (int i = threadIdx.x; i < m; i += blockDim.x) s[i] = H[st + i];
        __syncthreads();
        block_sort_keys(s, m);
        for (int i = threadIdx.x; i < m; i += blockDim.x) H[st + i] = s[i];
        __syncthreads();
        cs[nc++] = st;
    }
    cs[nc] = hn;
    uint64_t *src = H, *dst = B;
    for (int width = 1; width < nc; width <<= 1) {
        for (int a = 0; a < nc; a += 2 * width) {
            const int64_t l0 = cs[a], l1 = cs[min(a + width, nc)], r1 = cs[min(a + 2 * width, nc)];
            const int64_t nl = l1 - l0, nr = r1 - l1;
            for (int64_t i = threadIdx.x; i < nl + nr; i += blockDim.x) {
                if (i < nl) {
                    const uint64_t x = src[l0 + i];
                    dst[l0 + i + gk_count_key(src + l1, nr, x, false)] = x;
                } else {
                    const int64_t j = i - nl;
                    const uint64_t x = src[l1 + j];
                    dst[l0 + j + gk_count_key(src + l0, nl, x, true)] = x;
                }
            }
        }
        __syncthreads();
        uint64_t *t = src; src = dst; dst = t;
    }
    if (src != H) {
        for (int64_t i = threadIdx.x; i < hn; i += blockDim.x) H[i] = src[i];
        __syncthreads();
    }
}

template <typename T>
__global__ void __launch_bounds__(GK_T) gk_partition_kernel(sdp_column col, int32_t P, double eps, uint8_t *work) {
    __shared__ uint64_t s[SORT_MAX];
    __shared__ uint32_t s_wsum[GK_T / WAVE];
    __shared__ int64_t s_next, s_w;
    const int p = blockIdx.x, t = threadIdx.x, lane = lane_id(), wv = t / WAVE;
    GkPart *parts = (GkPart *)work;
    uint8_t *mine = work + gk_head_off(P) + (int64_t)p * gk_part_bytes();
    uint64_t *H = (uint64_t *)mine, *B = H + GK_HBUF;
    GkView buf[2] = {gk_view(mine + 2 * GK_HBUF * 8, GK_CAP), gk_view(mine + 2 * GK_HBUF * 8 + GK_CAP * 24, GK_CAP)};
    const int64_t n = col.length;
    const int64_t r1 = (int64_t)(((__int128)(p + 1) * n) / P);
    int64_t row = (int64_t)(((__int128)p * n) / P);
    int64_t len = 0, count = 0, status = 0;
    int cur = 0;
    bool any = false;
    const T *vals = (const T *)col.d_values;
    while (true) {
        // next head: up to GK_HEAD non-null, non-NaN values in row order
        int64_t hn = 0;
        while (hn < GK_HEAD && row < r1) {
            const int64_t i = row + t;
            bool ok = false;
            double x = 0.0;
            if (i < r1 && valid_bit(col.d_validity, col.validity_bit_offset, i)) {
                x = Elem<T>::d(vals[i]);
                ok = !(x != x);
            }
            const uint64_t m = __ballot(ok);
            if (lane == 0) s_wsum[wv] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t before = 0, total = 0;
            for (int k = 0; k < GK_T / WAVE; ++k) { const uint32_t c = s_wsum[k]; before += k < wv ? c : 0; total += c; }
            const int64_t take = min((int64_t)total, GK_HEAD - hn);
            const int64_t rk = before + lane_rank(m);
            if (ok && rk < take) H[hn + rk] = gk_key(x);
            if (ok && rk == take - 1 && take < (int64_t)total) s_next = i + 1;
            if (t == 0 && take == (int64_t)total) s_next = min(row + GK_T, r1);
            __syncthreads();
            row = s_next;
            hn += take;
            __syncthreads();
        }
        const bool full = hn == GK_HEAD;
        if (hn > 0) {
            any = true;
            if (len + hn > GK_CAP) { status = 1; break; }
            gk_sort_head(H, B, hn, s);
            gk_insert(H, hn, buf[cur], len, count, eps, buf[cur ^ 1]);
            len += hn;
            count += hn;
            // compress (every full head reaches the threshold; a final partial head is
            // compressed by the serializing compress() below)
            if (full && len >= GK_COMPRESS) {
                const int64_t w = gk_compress(buf[cur ^ 1], len, 2 * eps * (double)count, buf[cur], &s_w);
                gk_copy(buf[cur], w, len - w, buf[cur ^ 1]);
                len -= w;
            }
            cur ^= 1;
        }
        if (!full) break;
    }
    if (status == 0 && any) {               // the partial aggregate is serialized compressed
        const int64_t w = gk_compress(buf[cur], len, 2 * eps * (double)count, buf[cur ^ 1], &s_w);
        gk_copy(buf[cur ^ 1], w, len - w, buf[cur]);
        len -= w;
    }
    if (t == 0) {
        parts[p].len = len;
        parts[p].count = count;
        parts[p].which = cur;
        parts[p].status = status;
    }
}

// one workgroup: stable-merge the partition summaries in partition order
// (QuantileSummaries.merge), then query every probability
__device__ void gk_zero_fix(GkView a, int64_t n, GkView tmp) {
    // numerically sorted samples may hold 0.0 before -0.0: put the zero run in
    // Double.compare order (stable), as sortBy(_.value) sees it
    if (threadIdx.x == 0) {
        const int64_t z0 = gk_count_lt(a.v, n, 0.0, false), z1 = gk_count_lt(a.v, n, 0.0, true);
        int64_t k = 0;
        for (int pass = 0; pass < 2; ++pass)
            for (int64_t i = z0; i < z1; ++i) {
                const bool neg = (__double_as_longlong(a.v[i]) >> 63) != 0;
                if (neg == (pass == 0)) { tmp.v[k] = a.v[i]; tmp.g[k] = a.g[i]; tmp.d[k] = a.d[i]; ++k; }
            }
        for (int64_t i = 0; i < k; ++i) { a.v[z0 + i] = tmp.v[i]; a.g[z0 + i] = tmp.g[i]; a.d[z0 + i] = tmp.d[i]; }
    }
    __syncthreads();
}
__global__ void __launch_bounds__(GK_T) gk_merge_query_kernel(int32_t P, double eps, uint8_t *work,
                                                              const double *probs, int32_t np, double *out,
                                                              int64_t *status) {
    __shared__ int64_t s_w;
    GkPart *parts = (GkPart *)work;
    uint8_t *mbase = work + gk_head_off(P) + (int64_t)P * gk_part_bytes();
    const int64_t MC = 2 * GK_CAP;
    GkView M = gk_view(mbase, MC), X = gk_view(mbase + MC * 24, MC);
    int64_t m = 0, cm = 0, st = 0;
    for (int p = 0; p < P; ++p) {
        const GkPart gp = parts[p];
        if (gp.status) { st = gp.status; break; }
        if (gp.count == 0) continue;
        uint8_t *mine = work + gk_head_off(P) + (int64_t)p * gk_part_bytes();
        GkView pv = gk_view(mine + 2 * GK_HBUF * 8 + gp.which * GK_CAP * 24, GK_CAP);
        if (cm == 0) {
            gk_copy(pv, 0, gp.len, M);
            m = gp.len;
            cm = gp.count;
            continue;
        }
        if (m + gp.len > MC) { st = 2; break; }
        gk_zero_fix(M, m, X);
        gk_zero_fix(pv, gp.len, X);
        // stable merge by Double.compare: M's samples first among equal keys
        for (int64_t i = threadIdx.x; i < m + gp.len; i += blockDim.x) {
            int64_t q;
            double v;
            int64_t g, d;
            if (i < m) {
                v = M.v[i]; g = M.g[i]; d = M.d[i];
                const uint64_t k = gk_key(v);
                int64_t lo = 0, hi = gp.len;
                while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (gk_key(pv.v[mid]) < k) lo = mid + 1; else hi = mid; }
                q = i + lo;
            } else {
                const int64_t j = i - m;
                v = pv.v[j]; g = pv.g[j]; d = pv.d[j];
                const uint64_t k = gk_key(v);
                int64_t lo = 0, hi = m;
                while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (gk_key(M.v[mid]) <= k) lo = mid + 1; else hi = mid; }
                q = j + lo;
            }
            X.v[q] = v; X.g[q] = g; X.d[q] = d;
        }
        __syncthreads();
        const int64_t L = m + gp.len;
        const int64_t w = gk_compress(X, L, 2 * eps * (double)cm, M, &s_w);   // threshold: the receiver's count
        gk_copy(M, w, L - w, X);
        gk_copy(X, 0, L - w, M);
        m = L - w;
        cm += gp.count;
    }
    if (threadIdx.x != 0) return;
    status[0] = st;
    status[1] = cm;
    status[2] = m;
    for (int k = 0; k < np; ++k) {
        const double q = probs[k];
        double r = __builtin_nan("");
        if (st == 0 && m > 0) {
            if (q <= eps) {
                r = M.v[0];
            } else if (q >= 1 - eps) {
                r = M.v[m - 1];
            } else {
                // Scala's Double.toInt saturates at Int.MaxValue (reachable once
                // q * count >= 2^31; an out-of-range C++ cast would be undefined)
                const double rr = ceil(q * (double)cm);
                const int64_t rank = rr >= 2147483647.0 ? (int64_t)2147483647 : (int64_t)(int32_t)rr;
                const double target = ceil(eps * (double)cm);
                int64_t min_rank = 0;
                r = M.v[m - 1];
                for (int64_t i = 1; i < m - 1; ++i) {
                    min_rank += M.g[i];
                    const int64_t max_rank = min_rank + M.d[i];
                    if ((double)max_rank - target <= (double)rank && (double)rank <= (double)min_rank + target) {
                        r = M.v[i];
                        break;
                    }
                }
            }
        }
        out[k] = r;
    }
}

extern "C" int64_t sdp_gk_workspace_bytes(int32_t n_partitions) {
    if (n_partitions < 1) return -1;
    return gk_head_off(n_partitions) + (int64_t)n_partitions * gk_part_bytes() + 2 * (2 * GK_CAP) * 24;
}

extern "C" int sdp_gk_layout(int32_t n_partitions, int64_t *out4) {
    if (n_partitions < 1 || out4 == nullptr) return set_error(SDP_EINVAL, "sdp_gk_layout: args");
    out4[0] = gk_head_off(n_partitions);        // partition p's state at out4[0] + p * out4[1]
    out4[1] = gk_part_bytes();
    out4[2] = 2 * GK_HBUF * 8;                  // sample buffer b of a partition at + out4[2] + b * out4[3] * 24
    out4[3] = GK_CAP;                           // (v[cap] f64, g[cap] i64, d[cap] i64)
    return SDP_OK;
}

extern "C" int sdp_gk_partitions(const sdp_column *col, int32_t n_partitions, int32_t accuracy, void *d_work,
                                 int64_t work_bytes, void *stream) {
    int rc = check_col(col, "sdp_gk_partitions");
    if (rc) return rc;
    if (n_partitions < 1 || n_partitions > 65535) return set_error(SDP_EINVAL, "sdp_gk_partitions: n_partitions %d", n_partitions);
    if (accuracy < 1) return set_error(SDP_EINVAL, "sdp_gk_partitions: accuracy %d", accuracy);
    if (work_bytes < sdp_gk_workspace_bytes(n_partitions))
        return set_error(SDP_ECAP, "sdp_gk_partitions: workspace %lld < %lld", (long long)work_bytes,
                         (long long)sdp_gk_workspace_bytes(n_partitions));
    const double eps = 1.0 / (double)accuracy;
    hipStream_t s = (hipStream_t)stream;
    switch (col->dtype) {
    case SDP_F64:
        hipLaunchKernelGGL(gk_partition_kernel<double>, dim3(n_partitions), dim3(GK_T), 0, s, *col, n_partitions, eps,
                           (uint8_t *)d_work);
        break;
    case SDP_F32:
        hipLaunchKernelGGL(gk_partition_kernel<float>, dim3(n_partitions), dim3(GK_T), 0, s, *col, n_partitions, eps,
                           (uint8_t *)d_work);
        break;
    default: return set_error(SDP_EINVAL, "sdp_gk_partitions: dtype %d is not float/double", col->dtype);
    }
    return check_launch("gk_partition_kernel");
}

extern "C" int sdp_gk_merge(int32_t n_partitions, int32_t accuracy, const double *d_probs, int32_t n_probs,
                            void *d_work, int64_t work_bytes, double *d_out, int64_t *d_status, void *stream) {
    if (n_partitions < 1 || n_partitions > 65535 || accuracy < 1) return set_error(SDP_EINVAL, "sdp_gk_merge: args");
    if (n_probs < 0 || d_out == nullptr || d_status == nullptr || (n_probs > 0 && d_probs == nullptr))
        return set_error(SDP_EINVAL, "sdp_gk_merge: outputs");
    if (work_bytes < sdp_gk_workspace_bytes(n_partitions)) return set_error(SDP_ECAP, "sdp_gk_merge: workspace");
    hipLaunchKernelGGL(gk_merge_query_kernel, dim3(1), dim3(GK_T), 0, (hipStream_t)stream, n_partitions,
                       1.0 / (double)accuracy, (uint8_t *)d_work, d_probs, n_probs, d_out, d_status);
    return check_launch("gk_merge_query_kernel");
}

extern "C" int sdp_gk_quantiles(const sdp_column *col, int32_t n_partitions, int32_t accuracy, const double *d_probs,
                                int32_t n_probs, void *d_work, int64_t work_bytes, double *d_out, int64_t *d_status,
                                void *stream) {
    int rc = check_col(col, "sdp_gk_quantiles");
    if (rc) return rc;
    if (n_partitions < 1 || n_partitions > 65535) return set_error(SDP_EINVAL, "sdp_gk_quantiles: n_partitions %d", n_partitions);
    if (accuracy < 1) return set_error(SDP_EINVAL, "sdp_gk_quantiles: accuracy %d", accuracy);
    if (n_probs < 0 || d_out == nullptr || d_status == nullptr || (n_probs > 0 && d_probs == nullptr))
        return set_error(SDP_EINVAL, "sdp_gk_quantiles: outputs");
    if (work_bytes < sdp_gk_workspace_bytes(n_partitions))
        return set_error(SDP_ECAP, "sdp_gk_quantiles: workspace %lld < %lld", (long long)work_bytes,
                         (long long)sdp_gk_workspace_bytes(n_partitions));
    const double eps = 1.0 / (double)accuracy;
    hipStream_t s = (hipStream_t)stream;
    switch (col->dtype) {
    case SDP_F64:
        hipLaunchKernelGGL(gk_partition_kernel<double>, dim3(n_partitions), dim3(GK_T), 0, s, *col, n_partitions, eps,
                           (uint8_t *)d_work);
        break;
    case SDP_F32:
        hipLaunchKernelGGL(gk_partition_kernel<float>, dim3(n_partitions), dim3(GK_T), 0, s, *col, n_partitions, eps,
                           (uint8_t *)d_work);
        break;
    default: return set_error(SDP_EINVAL, "sdp_gk_quantiles: dtype %d is not float/double", col->dtype);
    }
    rc = check_launch("gk_partition_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(gk_merge_query_kernel, dim3(1), dim3(GK_T), 0, s, n_partitions, eps, (uint8_t *)d_work, d_probs,
                       n_probs, d_out, d_status);
    return check_launch("gk_merge_query_kernel");
}
