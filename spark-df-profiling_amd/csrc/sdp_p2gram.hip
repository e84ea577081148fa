// sdp_p2gram.hip -- pass 2 of every NUM column and their Pearson Gram in ONE
// read of the table (round 5).
//
// The reference computes pass 2 per column (describe.py:215-223 mad and the
// outlier counts, :49 the CASE-WHEN histogram) and the Pearson matrix with one
// Spark job per column pair over df.na.drop(how='any') (utils.py:27-31).  The
// engine already folds each counted column's level-1 partition count
// (describe.py:143 countDistinct) into its pass-2 read; the Gram was a separate
// read of every NUM column (sdp_gram, ~89 GB per 1e9-row C3 step).  Here one
// kernel streams all <= 16 NUM columns of a table row-block by row-block in the
// Gram's lane layout -- lane (q, c): rows 4q..4q+3 of every 16-row k-block of
// column c -- so each lane holds ONE column's values: that column's pass-2
// state (mad, outliers, cumulative bin counts against its edges) and level-1
// count (LDS histogram, heavy keys) stay per lane, and the same values feed
// v_mfma_f64_16x16x4f64 for G = (X-K)^T (X-K) over the rows every Gram column
// keeps (validity AND not-NaN, AND-reduced over the 16 lanes of a row group).
//
// Lanes of one MFMA wave would hold 16 different columns (dtypes, count modes,
// heavy tables): measured first (lane = column, every lane running every
// column kind's path) it took 99.8 ms per C3 step against 51 ms for the
// separate launches.  So the work is split by wave instead: wave c of a
// workgroup owns column c and runs its pass-2 and count work on 256-row tiles
// exactly as sdp_pass2_count does (lanes = rows, the column's edges and mode
// wave-uniform), writing (x - K) of the rows it keeps into an LDS tile
// Y[c][row] and the 'kept' ballots; after one barrier every wave takes
// 16-row k-blocks of the tile and runs the MFMAs from LDS, each row masked by
// the AND of all Gram columns' ballots (listwise deletion).  Y is double
// buffered, so each 256-row tile costs one workgroup barrier.
//
// Outputs are exactly those of sdp_pass2_count_batch per column (the block
// partials pass2_merge_batch_kernel sums, the level-1 histogram / heavy counts /
// stats of sdp_part_rows phase 0 or sdp_distinct32's level-1 count) plus the
// Gram partials gram_reduce_kernel<16> sums -- so the merge and the grouping
// that follow are unchanged.  Block g covers the partition row block g
// (rows_per_block of sdp_part_rows_per_block), one 16-wave workgroup per CU.
#include "sdp_common.h"
#include "sdp_heavy.h"
#include "sdp_internal.h"

namespace sdp {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int PG_C = 16;                   // column slots (the MFMA tile), one wave each
constexpr int PG_R = 256;                  // rows per tile: 4 per lane of a column wave
constexpr int PG_KB = PG_R / 16;           // 16-row k-blocks per tile
constexpr int PG_P = 258;                  // Y row pitch (doubles): 16-B rows, 2-way banking at worst
constexpr int PG_POOL = 64 * 1024;         // LDS for the level-1 histograms and heavy tables
constexpr int PG_NONE = -2;                // b1 of a column without a level-1 count
constexpr int P2G_MAX_BINS = 10;           // bins per column (describe()'s default, bins=10)

struct PgLds {
    double y[2][PG_C][PG_P];               // (x - K) of kept rows, 0 otherwise; double buffered
    uint64_t okm[2][PG_C][4];              // column c, element m: bit l = row 4l + m kept by c
    alignas(16) unsigned char pool[PG_POOL];
    double cs[PG_C][PG_C];                 // epilogue: per-wave column sums
    double nk[PG_C];
};

struct PgArgs {
    int32_t ncols;
    uint32_t gram_mask;                    // columns in the Pearson matrix
    int32_t hist_off[PG_C];                // pool byte offset of column c's histogram (-1: no count)
    int32_t heavy_off[PG_C];               // pool byte offset of its heavy table (-1: none)
    int64_t n, rows_per_block;
    int32_t grid;
    int32_t _pad;
};

// a column wave's pass-2 state (per lane; summed over the wave at the end)
template <int NB>
struct PgState {
    double mad;
    uint32_t high, low, okc, rows, special;
    uint32_t bc[NB];
};

// a column's context, wave-uniform
template <int NB>
struct PgCol {
    const uint8_t *vals, *vmap;
    int64_t vbit, lo32;
    double mean, hi_t, lo_t;
    double ev[NB];
    int b1, shift, nheavy;
    bool in_gram;
    uint32_t *hist;
    HeavyLdsT<false> *hv;
};

// one tile of column wave c: rows tr + 4 lane + m (m < 4) whose raw bytes are
// `lo` (and `hi`, 8-byte types); `vb` their validity bits
template <typename T, int NB>
__device__ __forceinline__ void pg_tile(const PgCol<NB> &cc, PgState<NB> &st, u32x4 lo, u32x4 hi, uint32_t vb,
                                        double *yrow, uint64_t *okm, int lane) {
    T x[4];
    if constexpr (sizeof(T) == 8) {
        const uint64_t b[4] = {((uint64_t)lo[1] << 32) | lo[0], ((uint64_t)lo[3] << 32) | lo[2],
                               ((uint64_t)hi[1] << 32) | hi[0], ((uint64_t)hi[3] << 32) | hi[2]};
#pragma unroll
        for (int m = 0; m < 4; ++m) memcpy(&x[m], &b[m], 8);
    } else {
#pragma unroll
        for (int m = 0; m < 4; ++m) { const uint32_t b = lo[m]; memcpy(&x[m], &b, 4); }
    }
    double y[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const bool valid = (vb >> m) & 1u;
        const double xd = Elem<T>::d(x[m]);
        const bool ok = valid && !(Elem<T>::is_float && xd != xd);
        // pass 2 (describe.py:215-223, :49; sdp_pass2_count's SMALL / MONO path)
        st.high += (uint32_t)(valid && spark_gt(xd, cc.hi_t));
        st.low += (uint32_t)(valid && spark_lt(xd, cc.lo_t));
        st.okc += (uint32_t)ok;
        st.mad += ok ? fabs(xd - cc.mean) : 0.0;
        const double xv = ok ? xd : -__builtin_inf();
#pragma unroll
        for (int j = 0; j < NB; ++j) st.bc[j] += (uint32_t)(xv >= cc.ev[j]);
        // the level-1 count (sdp_part_rows phase 0 / sdp_distinct32's)
        if (valid) {
            ++st.rows;
            if (cc.b1 == -1) {
                if constexpr (!std::is_same<T, double>::value)
                    atomicAdd(&cc.hist[mix32(key32_rel<T>(x[m], cc.lo32)) >> (32 - D32_B1)], 1u);
            } else if (cc.b1 >= 0) {
                const uint64_t h = mix64(key_of<T>(x[m]));
                const int hv = cc.nheavy ? heavy_find_u64(*cc.hv, cc.nheavy, h) : -1;
                if (hv >= 0) atomicAdd(&cc.hv->cnt[hv], 1u);
                else if (h == EMPTY64) ++st.special;
                else atomicAdd(&cc.hist[cc.b1 ? (int)(h >> cc.shift) : 0], 1u);
            }
        }
        y[m] = (cc.in_gram && ok) ? xd - cc.mean : 0.0;
        const uint64_t bal = __ballot(ok);
        if (lane == 0) okm[m] = cc.in_gram ? bal : ~0ull;
    }
    double2 *yp = (double2 *)(yrow + 4 * lane);
    yp[0] = make_double2(y[0], y[1]);
    yp[1] = make_double2(y[2], y[3]);
}

// wave-uniform values in scalar registers (the column's context)
__device__ __forceinline__ double sgpr_f64(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ int64_t sgpr_i64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <typename P>
__device__ __forceinline__ P *sgpr_ptr(P *p) { return (P *)sgpr_i64((int64_t)p); }
__device__ __forceinline__ int sgpr_i32(int v) { return __builtin_amdgcn_readfirstlane(v); }

template <int NB>
__global__ void __launch_bounds__(PG_C * WAVE, 1) pass2_gram_kernel(const sdp_pass2_task *tasks, PgArgs a,
                                                                    double *part_g, double *part_cs,
                                                                    double *part_n) {
    __shared__ PgLds L;
    const int t = threadIdx.x, lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane(t / WAVE);          // this wave's column
    const int NW = a.ncols;                                           // (blockDim.x = 64 ncols)
    const int g = blockIdx.x;
    const int q = lane >> 4, cl = lane & 15;

    // ---- LDS: the counted columns' histograms, the heavy tables ----
    for (int c = 0; c < NW; ++c) {
        const int b1 = tasks[c].b1;
        const int nb = b1 == -1 ? D32_NB1 : (b1 >= 0 ? 1 << b1 : 0);
        uint32_t *h = (uint32_t *)(L.pool + (a.hist_off[c] > 0 ? a.hist_off[c] : 0));
        for (int b = t; b < nb; b += blockDim.x) h[b] = 0;
    }
    for (int c = 0; c < NW; ++c)
        if (a.heavy_off[c] >= 0) {
            const sdp_pass2_task &hk = tasks[c];
            heavy_build<false>(*(HeavyLdsT<false> *)(L.pool + a.heavy_off[c]),
                               HeavyArg{hk.heavy.d_h, nullptr, nullptr, nullptr, hk.heavy.n});
        }
    lds_barrier();

    // ---- this wave's column ----
    const sdp_pass2_task &tk = tasks[w];
    const int dt = sgpr_i32(tk.col.dtype);
    const int width = (dt == SDP_F64 || dt == SDP_I64) ? 8 : 4;
    PgCol<NB> cc;
    cc.vals = sgpr_ptr((const uint8_t *)tk.col.d_values);
    cc.vmap = sgpr_ptr(tk.col.d_validity);
    cc.vbit = sgpr_i64(tk.col.validity_bit_offset);
    cc.lo32 = sgpr_i64(tk.key32_lo);
    cc.mean = sgpr_f64(tk.mean);
    cc.hi_t = sgpr_f64(tk.hi_t);
    cc.lo_t = sgpr_f64(tk.lo_t);
    const int bins = sgpr_i32(tk.bins);
#pragma unroll
    for (int j = 0; j < NB; ++j) cc.ev[j] = sgpr_f64(j < bins ? tk.d_edges[j] : __builtin_inf());
    cc.b1 = sgpr_i32(tk.b1);
    cc.shift = cc.b1 > 0 ? 64 - cc.b1 : 0;
    cc.nheavy = a.heavy_off[w] >= 0 ? sgpr_i32(tk.heavy.n) : 0;
    cc.in_gram = (a.gram_mask >> w) & 1u;
    cc.hist = (uint32_t *)(L.pool + (a.hist_off[w] > 0 ? a.hist_off[w] : 0));
    cc.hv = (HeavyLdsT<false> *)(L.pool + (a.heavy_off[w] > 0 ? a.heavy_off[w] : 0));
    PgState<NB> st;
    st.mad = 0.0;
    st.high = st.low = st.okc = st.rows = st.special = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j) st.bc[j] = 0;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    double csum = 0.0, nkeep = 0.0;

    const int64_t n = a.n;
    const int64_t r0 = (int64_t)g * a.rows_per_block;
    const int64_t r1 = min(n, r0 + a.rows_per_block);
    // raw loads of a tile (rows tr + 4 lane .. + 3): whole 16-byte vectors
    // inside the block, element loads in the block's last partial tile
    auto load = [&](int64_t tr, u32x4 &lo, u32x4 &hi, uint32_t &vb) {
        const int64_t r = tr + 4 * lane;
        if (tr + PG_R <= r1) {
            const __attribute__((address_space(1))) u32x4 *p =
                (const __attribute__((address_space(1))) u32x4 *)(cc.vals + r * width);
            lo = p[0];
            hi = width == 8 ? p[1] : lo;
            vb = valid_bits(cc.vmap, cc.vbit, r, 4);
        } else {
            uint32_t wd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            vb = 0;
            for (int m = 0; m < 4; ++m) {
                const int64_t i = r + m;
                if (i < r1) {
                    if (width == 8) {
                        const uint64_t v = ((const uint64_t *)cc.vals)[i];
                        wd[2 * m] = (uint32_t)v;
                        wd[2 * m + 1] = (uint32_t)(v >> 32);
                    } else {
                        wd[m] = ((const uint32_t *)cc.vals)[i];
                    }
                    vb |= (valid_bit(cc.vmap, cc.vbit, i) ? 1u : 0u) << m;
                }
            }
            lo = u32x4{wd[0], wd[1], wd[2], wd[3]};
            hi = u32x4{wd[4], wd[5], wd[6], wd[7]};
        }
    };
    u32x4 lo, hi;
    uint32_t vb = 0;
    if (r0 < r1) load(r0, lo, hi, vb);
    int buf = 0;
    for (int64_t tr = r0; tr < r1; tr += PG_R, buf ^= 1) {
        // next tile's loads in flight while this one is worked on
        u32x4 nlo = lo, nhi = hi;
        uint32_t nvb = 0;
        if (tr + PG_R < r1) load(tr + PG_R, nlo, nhi, nvb);
        // ---- phase 1: this wave's column over the tile ----
        double *yrow = L.y[buf][w];
        uint64_t *okm = L.okm[buf][w];
        switch (dt) {
        case SDP_F64: pg_tile<double, NB>(cc, st, lo, hi, vb, yrow, okm, lane); break;
        case SDP_F32: pg_tile<float, NB>(cc, st, lo, hi, vb, yrow, okm, lane); break;
        case SDP_I64: pg_tile<int64_t, NB>(cc, st, lo, hi, vb, yrow, okm, lane); break;
        default: pg_tile<int32_t, NB>(cc, st, lo, hi, vb, yrow, okm, lane); break;
        }
        lds_barrier();
        // ---- phase 2: the Gram over the tile's k-blocks (every wave) ----
        uint64_t km[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            uint64_t v = cl < NW ? L.okm[buf][cl][m] : ~0ull;
            v &= __shfl_xor(v, 1, WAVE);
            v &= __shfl_xor(v, 2, WAVE);
            v &= __shfl_xor(v, 4, WAVE);
            v &= __shfl_xor(v, 8, WAVE);
            km[m] = v;                       // bit l: row 4l + m kept by every Gram column
        }
        const double *yc = L.y[buf][cl < NW ? cl : 0];
        for (int kb = w; kb < PG_KB; kb += NW) {
            const int l = 4 * kb + q;
            uint32_t kbits = 0;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const bool keep = (km[m] >> l) & 1u;
                kbits |= (keep ? 1u : 0u) << m;
                const double yv = yc[16 * kb + 4 * q + m];
                const double y = (keep && cl < NW) ? yv : 0.0;
                csum += y;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, acc, 0, 0, 0);
            }
            if (cl == 0) nkeep += (double)__popc(kbits);
        }
        lo = nlo;
        hi = nhi;
        vb = nvb;
    }

    // ---- column wave: pass-2 partial of the block (sdp_pass2_count's layout) ----
    {
        const double md = wave_sum_f64(st.mad);
        const uint64_t hi_ = wave_sum_u64(st.high), lo_ = wave_sum_u64(st.low), okc = wave_sum_u64(st.okc);
        const uint64_t rows = wave_sum_u64(st.rows), sp = wave_sum_u64(st.special);
        uint64_t bcs[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) bcs[j] = wave_sum_u64(st.bc[j]);
        const int stride = 3 + bins;
        if (lane == 0) {
            double *pm = (double *)tk.d_work;
            uint64_t *pc = (uint64_t *)((char *)tk.d_work + (int64_t)tk.grid * sizeof(double)) + (int64_t)g * stride;
            pm[g] = md;
            pc[0] = hi_;
            pc[1] = lo_;
            pc[2] = okc - bcs[0];                         // ok rows below e_0
#pragma unroll
            for (int j = 0; j < NB; ++j)                  // CASE-WHEN bins from the cumulative counts
                if (j < bins) pc[3 + j] = j + 1 < bins ? bcs[j] - bcs[j + 1] : bcs[j];
            if (tk.b1 == -1) {
                if (rows) atomicAdd((unsigned long long *)&tk.d_stats[1], (unsigned long long)rows);
            } else if (tk.b1 >= 0) {
                if (rows) atomicAdd((unsigned long long *)&tk.d_stats[0], (unsigned long long)rows);
                if (sp) atomicAdd((unsigned long long *)&tk.d_stats[1], (unsigned long long)sp);
            }
        }
    }
    // ---- the level-1 count outputs (every thread has passed its last LDS atomic) ----
    lds_barrier();
    if (tk.b1 != PG_NONE) {
        const int nb = tk.b1 == -1 ? D32_NB1 : 1 << tk.b1;
        for (int b = lane; b < nb; b += WAVE) tk.d_part_hist[(int64_t)b * a.grid + g] = cc.hist[b];
        if (cc.nheavy)
            for (int i = lane; i < cc.nheavy; i += WAVE)
                if (cc.hv->cnt[i])
                    atomicAdd((unsigned long long *)&tk.d_heavy_counts[i], (unsigned long long)cc.hv->cnt[i]);
    }
    // ---- the Gram tile, column sums and kept rows of the block ----
    double *ep = &L.y[0][0][0];                           // (every wave is past its last Y read)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) ep[w * 256 + (q + 4 * rr) * 16 + cl] = acc[rr];
    {
        double v = csum;
        v += __shfl_xor(v, 16, WAVE);
        v += __shfl_xor(v, 32, WAVE);
        if (q == 0) L.cs[w][cl] = v;
        const double nk = wave_sum_f64(nkeep);
        if (lane == 0) L.nk[w] = nk;
    }
    __syncthreads();
    for (int e = t; e < 256 + PG_C + 1; e += blockDim.x) {
        double v = 0.0;
        if (e < 256) {
            for (int ww = 0; ww < NW; ++ww) v += ep[ww * 256 + e];
            part_g[(int64_t)g * 256 + e] = v;
        } else if (e < 256 + PG_C) {
            for (int ww = 0; ww < NW; ++ww) v += L.cs[ww][e - 256];
            part_cs[(int64_t)g * PG_C + (e - 256)] = v;
        } else {
            for (int ww = 0; ww < NW; ++ww) v += L.nk[ww];
            part_n[g] = v;
        }
    }
}

}  // namespace
}  // namespace sdp

using namespace sdp;

extern "C" int64_t sdp_pass2_gram_workspace_bytes(int64_t length, int32_t ncols) {
    if (length < 0 || ncols < 1 || ncols > PG_C) return -1;
    const int64_t rpb = sdp_part_rows_per_block(length > 0 ? length : 1, 0);
    const int64_t grid = (length + rpb - 1) / rpb < 1 ? 1 : (length + rpb - 1) / rpb;
    return grid * (256 + PG_C + 1) * (int64_t)sizeof(double) + 3 * 256;
}

extern "C" int sdp_pass2_gram(const sdp_pass2_task *h_tasks, const sdp_pass2_task *d_tasks, int32_t ntasks,
                              uint32_t gram_mask, void *d_work, int64_t work_bytes, double *d_gram, double *d_colsum,
                              double *d_n, void *stream) {
    if (h_tasks == nullptr || d_tasks == nullptr || ntasks < 1 || ntasks > PG_C || d_work == nullptr ||
        d_gram == nullptr || d_colsum == nullptr || d_n == nullptr)
        return set_error(SDP_EINVAL, "sdp_pass2_gram: args");
    const int64_t n = h_tasks[0].col.length;
    const int64_t rpb = sdp_part_rows_per_block(n > 0 ? n : 1, 0);
    const int64_t grid = (n + rpb - 1) / rpb < 1 ? 1 : (n + rpb - 1) / rpb;
    PgArgs a{};
    a.ncols = ntasks;
    int pool = 0;
    a.gram_mask = gram_mask & ((1u << ntasks) - 1u);
    a.n = n;
    a.rows_per_block = rpb;
    a.grid = (int32_t)grid;
    int heavy_cols = 0, max_bins = 0;
    for (int i = 0; i < ntasks; ++i) {
        const sdp_pass2_task &t = h_tasks[i];
        const int dt = t.col.dtype;
        if (t.col.length != n) return set_error(SDP_EINVAL, "sdp_pass2_gram: column lengths differ");
        if (dt != SDP_F64 && dt != SDP_F32 && dt != SDP_I64 && dt != SDP_I32)
            return set_error(SDP_EINVAL, "sdp_pass2_gram: column %d dtype %d", i, dt);
        if (n > 0 && !aligned16(t.col.d_values)) return set_error(SDP_EALIGN, "sdp_pass2_gram: column %d alignment", i);
        if (t.bins < 2 || t.bins > P2G_MAX_BINS || !t.edges_monotone)
            return set_error(SDP_EINVAL, "sdp_pass2_gram: column %d needs 2..%d monotone bins", i, P2G_MAX_BINS);
        if (t.rows_per_block != rpb || t.grid != grid)
            return set_error(SDP_EINVAL, "sdp_pass2_gram: column %d geometry (rows_per_block / grid)", i);
        if (t.b1 < PG_NONE || t.b1 > 10) return set_error(SDP_EINVAL, "sdp_pass2_gram: column %d b1 %d", i, t.b1);
        if (t.b1 == -1 && dt == SDP_F64) return set_error(SDP_EINVAL, "sdp_pass2_gram: b1 = -1 on a double column");
        if (t.b1 != PG_NONE && (t.d_part_hist == nullptr || t.d_stats == nullptr))
            return set_error(SDP_EINVAL, "sdp_pass2_gram: column %d count outputs", i);
        // LDS pool: the column's histogram, then its heavy table
        a.hist_off[i] = a.heavy_off[i] = -1;
        const int nb = t.b1 == -1 ? D32_NB1 : (t.b1 >= 0 ? 1 << t.b1 : 0);
        if (nb) {
            a.hist_off[i] = pool;
            pool += (nb * 4 + 15) / 16 * 16;
        }
        if (t.b1 >= 0 && t.heavy.n > 0) {
            if (t.heavy.n > HEAVY_MAX || t.d_heavy_counts == nullptr || t.heavy.d_h == nullptr)
                return set_error(SDP_EINVAL, "sdp_pass2_gram: column %d heavy keys", i);
            a.heavy_off[i] = pool;
            pool += ((int)sizeof(HeavyLdsT<false>) + 15) / 16 * 16;
            ++heavy_cols;
        }
        if (pool > PG_POOL)
            return set_error(SDP_ECAP, "sdp_pass2_gram: %d bytes of histograms and heavy tables > %d", pool, PG_POOL);
        if (t.bins > max_bins) max_bins = t.bins;
    }
    for (int i = ntasks; i < PG_C; ++i) a.hist_off[i] = a.heavy_off[i] = -1;
    (void)heavy_cols;
    if (work_bytes < sdp_pass2_gram_workspace_bytes(n, ntasks))
        return set_error(SDP_ECAP, "sdp_pass2_gram: workspace too small");
    double *pg = (double *)d_work;
    double *pcs = pg + grid * 256;
    double *pn = pcs + grid * PG_C;
    hipStream_t s = (hipStream_t)stream;
    if (max_bins <= 10)
        hipLaunchKernelGGL(pass2_gram_kernel<10>, dim3((unsigned)grid), dim3(WAVE * ntasks), 0, s, d_tasks, a, pg,
                           pcs, pn);
    else
        hipLaunchKernelGGL(pass2_gram_kernel<P2G_MAX_BINS>, dim3((unsigned)grid), dim3(WAVE * ntasks), 0, s, d_tasks,
                           a, pg, pcs, pn);
    int rc = check_launch("pass2_gram_kernel");
    if (rc) return rc;
    rc = launch_pass2_merge_batch(d_tasks, ntasks, s);
    if (rc) return rc;
    return launch_gram_reduce16(pg, pcs, pn, ntasks, (int)grid, d_gram, d_colsum, d_n, s);
}
