// sdp_gram.hip -- Pearson matrix support (utils.py:20-36 corr_matrix) on gfx950.
//
// The reference issues one Spark `df.stat.corr(x, y)` job per ordered column pair
// over `df.na.drop(how='any')` (utils.py:27-31), i.e. C^2 full scans.  Here the
// listwise-deletion mask is built once (sdp_rowmask) and the whole matrix comes
// from one shifted Gram product G = (X-K)^T (X-K) over the kept rows on the fp64
// matrix cores (v_mfma_f64_16x16x4_f64); rho = C_xy / sqrt(C_xx C_yy) with
// C = G - s s^T / n is formed by the host from (G, s, n).
//
// Decomposition: the upper-triangular TILE x TILE output tiles x S row chunks;
// each wave owns the full tile for every 4th 16-row k-block of its chunk and
// keeps (TILE/16)^2 accumulators.  Rows are permuted inside a k-block (lane
// group q reads rows 4q..4q+3, MFMA m uses row 4q+m) so each lane's loads are
// contiguous; a permutation of the summation order leaves G unchanged.  Chunk
// partials are summed in chunk order by gram_reduce_kernel (deterministic).
#include "sdp_common.h"

namespace sdp {

typedef double d4 __attribute__((ext_vector_type(4)));
// the LDS images' rows sit on 16-byte (not 32-byte) boundaries (pitches of
// G16_P / GW_PITCH doubles): accessed through this 16-byte-aligned type, so no
// access assumes d4's natural 32-byte alignment (ds_*_b128 pairs either way)
typedef double d4u __attribute__((ext_vector_type(4), aligned(16)));

constexpr int G_WAVES = 4;
constexpr int G_BLOCK = G_WAVES * WAVE;

// ---- row mask ------------------------------------------------------------------
struct MaskCol {
    sdp_column c;
    int32_t check_nan;
    int32_t _pad;
};

__device__ __forceinline__ double load_as_double(const void *p, int dt, int64_t i) {
    switch (dt) {
    case SDP_F64: return ((const double *)p)[i];
    case SDP_F32: return (double)((const float *)p)[i];
    case SDP_I64: return (double)((const int64_t *)p)[i];
    case SDP_I32: return (double)((const int32_t *)p)[i];
    case SDP_I16: return (double)((const int16_t *)p)[i];
    case SDP_I8: return (double)((const int8_t *)p)[i];
    case SDP_U32: return (double)((const uint32_t *)p)[i];
    case SDP_U16: return (double)((const uint16_t *)p)[i];
    case SDP_U8: return (double)((const uint8_t *)p)[i];
    default: return 0.0;
    }
}

__global__ void rowmask_kernel(const MaskCol *cols, int ncols, int64_t n, uint32_t *keep) {
    const int64_t nwords = (n + 31) / 32;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords;
         w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r0 = w * 32;
        const int cnt = (int)min((int64_t)32, n - r0);
        uint32_t k = cnt >= 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u);
        for (int c = 0; c < ncols && k; ++c) {
            const MaskCol &mc = cols[c];
            k &= valid_bits(mc.c.d_validity, mc.c.validity_bit_offset, r0, cnt);
            if (mc.check_nan) {
                for (int b = 0; b < cnt; ++b) {
                    const double x = load_as_double(mc.c.d_values, mc.c.dtype, r0 + b);
                    if (x != x) k &= ~(1u << b);
                }
            }
        }
        keep[w] = k;
    }
}

// ---- column descriptors into device memory, stream-ordered ----------------------
// K descriptors per launch ride in the kernel arguments (copied at launch), so
// the host array can be freed at once: no pageable copy and no
// hipStreamSynchronize, which drained the caller's whole queue before the row
// mask and again before the Gram (r06s's bench measured 5.8 ms of HIP-event
// time around the 0.69 ms row-mask kernel; a same-box A/B on another box was
// even, profiles/r06aa_*).
template <typename D, int K> struct DescBatch {
    D d[K];
};
template <typename D, int K> __global__ void put_desc_kernel(DescBatch<D, K> b, int count, D *dst) {
    const int i = threadIdx.x;
    if (i < count) dst[i] = b.d[i];
}
template <typename D, int K> static hipError_t put_descs(const D *h, int n, D *d_dst, hipStream_t s) {
    static_assert(sizeof(DescBatch<D, K>) <= 2048, "kernel argument block");
    for (int i0 = 0; i0 < n; i0 += K) {
        DescBatch<D, K> b;
        const int c = n - i0 < K ? n - i0 : K;
        for (int i = 0; i < K; ++i) b.d[i] = h[i0 + (i < c ? i : 0)];
        hipLaunchKernelGGL((put_desc_kernel<D, K>), dim3(1), dim3(K), 0, s, b, c, d_dst + i0);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---- Gram ----------------------------------------------------------------------
struct GramCol {
    const void *p;
    int32_t dtype;
    int32_t width;             // bytes per value
};

// 4 consecutive rows [r, r+4) of a column: raw bytes first, doubles after.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct Raw4 {
    u32x4 lo, hi;
};
// Rows [r, r + 32) lie inside the column (the fast path's margin), so every
// lane loads the same two 16-byte words whatever its dtype -- one load form
// per register, no divergent branch between loads, no waits until conv4.
// Lanes of columns absent from the tile read column 0 (cache hits) as dtype 0.
__device__ __forceinline__ void raw4(const GramCol &gc, int64_t r, Raw4 &x) {
    // (4-byte types use only `lo`; their `hi` is the next lane group's rows, a cache hit)
    const __attribute__((address_space(1))) u32x4 *b =
        (const __attribute__((address_space(1))) u32x4 *)((const char *)gc.p + r * gc.width);
    x.lo = b[0];
    x.hi = b[1];
}
__device__ __forceinline__ void conv4(int dt, const Raw4 &x, double out[4]) {
    const uint32_t w[8] = {x.lo[0], x.lo[1], x.lo[2], x.lo[3], x.hi[0], x.hi[1], x.hi[2], x.hi[3]};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const uint64_t u64 = ((uint64_t)w[2 * m + 1] << 32) | w[2 * m];
        double v;
        switch (dt) {
        case SDP_F64: v = __longlong_as_double((long long)u64); break;
        case SDP_I64: v = (double)(int64_t)u64; break;
        case SDP_F32: v = (double)__uint_as_float(w[m]); break;
        case SDP_I32: v = (double)(int32_t)w[m]; break;
        case SDP_U32: v = (double)w[m]; break;
        case SDP_I16: v = (double)(int16_t)(w[m >> 1] >> (16 * (m & 1))); break;
        case SDP_U16: v = (double)(uint16_t)(w[m >> 1] >> (16 * (m & 1))); break;
        case SDP_I8: v = (double)(int8_t)(w[0] >> (8 * m)); break;
        case SDP_U8: v = (double)(uint8_t)(w[0] >> (8 * m)); break;
        default: v = 0.0;
        }
        out[m] = v;
    }
}
// The four common dtypes without a per-lane branch (lanes of one wave hold
// different columns): both conversions of the 8-byte and of the 4-byte
// interpretation are formed and selected.  Integer -> double is exact below
// 2^53 and correctly rounded above (one rounding in the final add).
__device__ __forceinline__ void conv4_common(bool is8, bool isf, const Raw4 &x, double out[4]) {
    const uint32_t w[8] = {x.lo[0], x.lo[1], x.lo[2], x.lo[3], x.hi[0], x.hi[1], x.hi[2], x.hi[3]};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const uint32_t lo = w[2 * m], hi = w[2 * m + 1];
        const double f64 = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
        const double i64 = __builtin_fma((double)(int32_t)hi, 4294967296.0, (double)lo);
        const double f32 = (double)__uint_as_float(w[m]);
        const double i32 = (double)(int32_t)w[m];
        out[m] = is8 ? (isf ? f64 : i64) : (isf ? f32 : i32);
    }
}
__device__ __forceinline__ bool common_dtype(int dt) {
    return dt == SDP_F64 || dt == SDP_I64 || dt == SDP_F32 || dt == SDP_I32 || dt == 0;
}

// element-wise (the column's last rows); 0 beyond n and for dtype 0
__device__ __forceinline__ void load4_tail(const GramCol &gc, int64_t r, int64_t n, double out[4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
        out[m] = r + m < n ? load_as_double(gc.p, gc.dtype, r + m) : 0.0;
}

template <int TILE>
__global__ void __launch_bounds__(G_BLOCK) gram_kernel(const GramCol *cols, int ncols, const double *shift,
                                                       const uint32_t *keep, int64_t n, int ntiles_side, int T,
                                                       int64_t rows_per_chunk, double *part_g, double *part_cs,
                                                       double *part_n) {
    constexpr int NT = TILE / 16;
    const int t = blockIdx.x % T;
    const int s = blockIdx.x / T;
    // tile t -> (ti, tj), tj >= ti, row-major over the upper triangle
    int ti = 0, rem = t;
    while (rem >= ntiles_side - ti) { rem -= ntiles_side - ti; ++ti; }
    const int tj = ti + rem;
    const bool diag = ti == tj;
    const int lane = lane_id(), wid = threadIdx.x / WAVE;
    const int q = lane >> 4, cl = lane & 15;

    GramCol ca[NT], cb[NT];
    double ka[NT], kb[NT];
    bool va[NT], vb[NT];
#pragma unroll
    for (int a = 0; a < NT; ++a) {
        const int ci = ti * TILE + 16 * a + cl, cj = tj * TILE + 16 * a + cl;
        va[a] = ci < ncols;
        vb[a] = cj < ncols;
        ca[a] = va[a] ? cols[ci] : GramCol{cols[0].p, 0, cols[0].width};   // dtype 0 converts to 0.0
        cb[a] = vb[a] ? cols[cj] : GramCol{cols[0].p, 0, cols[0].width};
        ka[a] = va[a] ? shift[ci] : 0.0;
        kb[a] = vb[a] ? shift[cj] : 0.0;
    }
    // per-lane conversion selectors; `common` is wave-uniform
    bool a8[NT], af[NT], b8[NT], bf[NT], all_common = true;
#pragma unroll
    for (int a = 0; a < NT; ++a) {
        a8[a] = ca[a].width == 8 && ca[a].dtype != 0;
        af[a] = ca[a].dtype == SDP_F64 || ca[a].dtype == SDP_F32;
        b8[a] = cb[a].width == 8 && cb[a].dtype != 0;
        bf[a] = cb[a].dtype == SDP_F64 || cb[a].dtype == SDP_F32;
        all_common = all_common && common_dtype(ca[a].dtype) && common_dtype(cb[a].dtype);
    }
    const bool common = __all(all_common);
    d4 acc[NT][NT];
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    double csum[NT];
#pragma unroll
    for (int a = 0; a < NT; ++a) csum[a] = 0.0;
    double nkeep = 0.0;

    // UNR k-blocks per iteration.  Away from the column end (a wave-uniform
    // test) every lane issues the raw 16-byte loads of all UNR blocks back to
    // back -- no dtype branch sits between a load and the next one, so nothing
    // waits on memory before the conversions -- and only then converts; the
    // last blocks of the column take the element-wise path.
    constexpr int UNR = TILE == 16 ? 4 : (TILE == 32 ? 2 : 1);
    const int64_t c0 = (int64_t)s * rows_per_chunk;
    const int64_t c1 = min(n, c0 + rows_per_chunk);
    auto consume = [&](const double (&xa)[NT][4], const double (&xb)[NT][4], int64_t r, uint32_t kw) {
        uint32_t kbits = 0;
        if (r < c1) {
            kbits = (kw >> (r & 31)) & 0xFu;
            if (r + 4 > c1) kbits &= (1u << (int)(c1 - r)) - 1u;   // chunk boundary
        }
        if (diag && cl == 0) nkeep += (double)__popc(kbits);
        double ya[NT][4], yb[NT][4];
#pragma unroll
        for (int a = 0; a < NT; ++a) {
#pragma unroll
            for (int m = 0; m < 4; ++m) ya[a][m] = ((kbits >> m) & 1u) ? xa[a][m] - ka[a] : 0.0;
            if (diag) {
#pragma unroll
                for (int m = 0; m < 4; ++m) csum[a] += ya[a][m];
            }
        }
        if (!diag) {
#pragma unroll
            for (int b = 0; b < NT; ++b)
#pragma unroll
                for (int m = 0; m < 4; ++m) yb[b][m] = ((kbits >> m) & 1u) ? xb[b][m] - kb[b] : 0.0;
        }
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int a = 0; a < NT; ++a)
#pragma unroll
                for (int b = 0; b < NT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya[a][m], diag ? ya[b][m] : yb[b][m], acc[a][b],
                                                                      0, 0, 0);
    };
    for (int64_t rb = c0 + (int64_t)wid * 16 * UNR; rb < c1; rb += (int64_t)G_WAVES * 16 * UNR) {
        if (rb + 16 * UNR + 32 <= n) {
            uint32_t kw[UNR];
            Raw4 ra[UNR][NT], rbw[UNR][NT];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int64_t r = rb + 16 * u + 4 * q;
                kw[u] = r < c1 ? keep[r >> 5] : 0u;
#pragma unroll
                for (int a = 0; a < NT; ++a) raw4(ca[a], r, ra[u][a]);
                if (!diag) {
#pragma unroll
                    for (int b = 0; b < NT; ++b) raw4(cb[b], r, rbw[u][b]);
                }
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                double xa[NT][4], xb[NT][4];
                if (common) {
#pragma unroll
                    for (int a = 0; a < NT; ++a) conv4_common(a8[a], af[a], ra[u][a], xa[a]);
                    if (!diag) {
#pragma unroll
                        for (int b = 0; b < NT; ++b) conv4_common(b8[b], bf[b], rbw[u][b], xb[b]);
                    }
                } else {
#pragma unroll
                    for (int a = 0; a < NT; ++a) conv4(ca[a].dtype, ra[u][a], xa[a]);
                    if (!diag) {
#pragma unroll
                        for (int b = 0; b < NT; ++b) conv4(cb[b].dtype, rbw[u][b], xb[b]);
                    }
                }
                consume(xa, xb, rb + 16 * u + 4 * q, kw[u]);
            }
        } else {
            for (int u = 0; u < UNR; ++u) {
                const int64_t r = rb + 16 * u + 4 * q;
                double xa[NT][4], xb[NT][4];
#pragma unroll
                for (int a = 0; a < NT; ++a) load4_tail(ca[a], r, n, xa[a]);
                if (!diag) {
#pragma unroll
                    for (int b = 0; b < NT; ++b) load4_tail(cb[b], r, n, xb[b]);
                }
                consume(xa, xb, r, r < c1 ? keep[r >> 5] : 0u);
            }
        }
    }

    // ---- combine the 4 waves through LDS (fixed order), write the chunk partial ----
    __shared__ double s_acc[G_WAVES][TILE * TILE];
    __shared__ double s_cs[G_WAVES][TILE];
    __shared__ double s_n[G_WAVES];
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int i = 16 * a + q + 4 * rr, j = 16 * b + cl;   // f64 C/D map
                s_acc[wid][i * TILE + j] = acc[a][b][rr];
            }
    if (diag) {
#pragma unroll
        for (int a = 0; a < NT; ++a) {
            double v = csum[a];
            v += __shfl_xor(v, 16, WAVE);
            v += __shfl_xor(v, 32, WAVE);
            if (q == 0) s_cs[wid][16 * a + cl] = v;
        }
        const double nk = wave_sum_f64(nkeep);
        if (lane == 0) s_n[wid] = nk;
    }
    __syncthreads();
    double *pg = part_g + (int64_t)blockIdx.x * TILE * TILE;
    for (int e = threadIdx.x; e < TILE * TILE; e += G_BLOCK) {
        double v = 0.0;
        for (int w = 0; w < G_WAVES; ++w) v += s_acc[w][e];
        pg[e] = v;
    }
    if (diag) {
        for (int e = threadIdx.x; e < TILE; e += G_BLOCK) {
            double v = 0.0;
            for (int w = 0; w < G_WAVES; ++w) v += s_cs[w][e];
            part_cs[((int64_t)s * ntiles_side + ti) * TILE + e] = v;
        }
        if (ti == 0 && threadIdx.x == 0) {
            double v = 0.0;
            for (int w = 0; w < G_WAVES; ++w) v += s_n[w];
            part_n[s] = v;
        }
    }
}

// ---- wide tables (C > 64): 128 x 128 output tiles staged through LDS ---------
//
// One 512-thread workgroup owns output tile (ti, tj) (ti <= tj, 128 columns
// each) for one row chunk.  Per k-step of GW_KR = 32 rows the workgroup stages
// both column panels ONCE into LDS as shifted, masked fp64 ((x - K) or 0 for a
// dropped row), so the dtype conversion is paid once per element per tile
// instead of once per wave; every wave then runs its MFMAs from LDS.  Wave w
// owns the 64 x 32 quadrant (qa = w >> 2, qb = w & 3) of the tile: 8
// accumulators, no cross-wave reduction (each wave writes its quadrant of the
// chunk partial).  On a diagonal tile the waves share out the 36 upper-
// triangle 16x16 blocks instead (GW_DIAG_BLK; the reduce mirrors them).  The next
// k-step's raw loads are issued before the MFMA phase, so HBM latency hides
// behind the matrix work (v2: double-buffered panels, each slot's
// convert/store and its next load interleaved between MFMA groups, one
// barrier per k-step).  Blocks are mapped XCD-major: the tiles of one row
// chunk run on one XCD and share its L2 for the column reads.
//
// LDS panel layout [col][row] with a pitch of 34 doubles (68 dwords = 4 mod 64
// banks): an MFMA operand read (lane (q, cl) -> col 16a + cl, row 4kk + q)
// touches 64 distinct banks per 32-lane group.
constexpr int GW_TILE = 128;
constexpr int GW_WAVES = 8;
constexpr int GW_BLOCK = GW_WAVES * WAVE;
constexpr int GW_KR = 32;                              // rows per k-step
constexpr int GW_PITCH = 34;                           // doubles per column (32 rows + pad)
constexpr int GW_SLOTS = 2 * GW_TILE * (GW_KR / 4) / GW_BLOCK;   // (col, 4-row quad) per thread: 4

struct GwRaw {
    u32x4 lo, hi;
};

// Diagonal tiles: the 36 16x16 blocks (bi <= bj) of the upper triangle dealt
// round-robin to the 8 waves (5 or 4 each), so no SIMD carries more than ~10
// blocks per k-step against 16 on an off-diagonal tile.  Entry = bi * 8 + bj.
__constant__ uint8_t GW_DIAG_BLK[GW_WAVES][5] = {
    {0, 9, 19, 30, 47}, {1, 10, 20, 31, 54}, {2, 11, 21, 36, 55}, {3, 12, 22, 37, 63},
    {4, 13, 23, 38, 0}, {5, 14, 27, 39, 0}, {6, 15, 28, 45, 0}, {7, 18, 29, 46, 0}};
__constant__ uint8_t GW_DIAG_N[GW_WAVES] = {5, 5, 5, 5, 4, 4, 4, 4};

__device__ __forceinline__ void gw_load(const GramCol &gc, int64_t r, int64_t n, GwRaw &x) {
    if (gc.dtype == 0) return;
    const char *base = (const char *)gc.p + r * gc.width;
    if (r + 4 <= n) {
        switch (gc.width) {
        case 8: {
            const __attribute__((address_space(1))) u32x4 *b = (const __attribute__((address_space(1))) u32x4 *)base;
            x.lo = b[0];
            x.hi = b[1];
        } break;
        case 4: x.lo = *(const __attribute__((address_space(1))) u32x4 *)base; break;
        case 2: {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 v = *(const __attribute__((address_space(1))) u32x2 *)base;
            x.lo[0] = v[0];
            x.lo[1] = v[1];
        } break;
        default: x.lo[0] = *(const __attribute__((address_space(1))) uint32_t *)base;
        }
        return;
    }
    // column end: element-wise into the same byte image (beyond n -> zero bytes)
    uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int m = 0; m < 4 && r + m < n; ++m) {
        const unsigned char *e = (const unsigned char *)base + m * gc.width;
        for (int b = 0; b < gc.width; ++b) w[(m * gc.width + b) >> 2] |= (uint32_t)e[b] << (8 * ((m * gc.width + b) & 3));
    }
    x.lo = u32x4{w[0], w[1], w[2], w[3]};
    x.hi = u32x4{w[4], w[5], w[6], w[7]};
}

// ---- narrow tables (C <= 16): whole columns per wave while staging ---------------
//
// gram_kernel<16> converts in the MFMA operand layout, where the 16 lanes of a
// lane group hold 16 different columns: every lane forms all four common
// conversions and selects (SQ counters, profiles/r04s_gram_sq_pmc.txt: ~100
// VALU instructions per 16-row k-block, wait_inst 0.53 of wave cycles -- issue
// bound, not memory bound).  Here a 256-row k-step is staged into LDS first,
// each wave converting four whole columns (column, dtype and shift are
// wave-uniform: a uniform branch per column and k-step, then one conversion
// per element or none), and then every wave runs the MFMAs of its four 16-row
// groups from LDS.  The next k-step's raw loads are issued right after the
// staging, so they are in flight during the MFMAs; four workgroups per CU.
// Only the chunk's last k-step can be ragged (a wave-uniform test): the others
// load without per-lane bounds checks.
// LDS [col][row] with a pitch of 258 doubles (2 * 258 = 4 mod 64 banks): the
// 16 lanes of an operand read (column cl, 4 consecutive rows) touch 64
// distinct banks.  (A 16-wave form with one column per wave and its k-loop
// instantiated per dtype ran 23.0 ms against this form's 19.1 on 1e9 x 13
// columns: one workgroup per CU left the HBM idle during its barriers.)
constexpr int G16_W = 4;                        // waves per workgroup
constexpr int G16_BLOCK = G16_W * WAVE;
// (G16_Q = 2 -- 512-row k-steps, two workgroups per CU at 224 VGPRs -- measured
// 27.2 vs 17.7 ms on 1e9 x 13 columns, profiles/r05ab_gram16_two_quads_rejected_ab.log)
#ifndef G16_Q
#define G16_Q 1
#endif
constexpr int G16_QN = G16_Q;                   // 4-row quads per lane and column per k-step
constexpr int G16_R = 4 * WAVE * G16_QN;        // rows per k-step (quad k of lane l: rows 4 l + 256 k)
constexpr int G16_P = G16_R + 2;                // LDS pitch in doubles
constexpr int G16_CPW = 16 / G16_W;             // columns staged per wave

// stage 4 rows of a column of dtype DT: convert, shift, mask, sum, store
template <int DT>
__device__ __forceinline__ void g16_stage(const GwRaw &x, uint32_t kb, double K, double &csum, double *dst) {
    double v[4];
    if (DT == SDP_F64) {
        v[0] = __longlong_as_double((long long)(((uint64_t)x.lo[1] << 32) | x.lo[0]));
        v[1] = __longlong_as_double((long long)(((uint64_t)x.lo[3] << 32) | x.lo[2]));
        v[2] = __longlong_as_double((long long)(((uint64_t)x.hi[1] << 32) | x.hi[0]));
        v[3] = __longlong_as_double((long long)(((uint64_t)x.hi[3] << 32) | x.hi[2]));
    } else if (DT == SDP_I64) {
        v[0] = (double)(int64_t)(((uint64_t)x.lo[1] << 32) | x.lo[0]);
        v[1] = (double)(int64_t)(((uint64_t)x.lo[3] << 32) | x.lo[2]);
        v[2] = (double)(int64_t)(((uint64_t)x.hi[1] << 32) | x.hi[0]);
        v[3] = (double)(int64_t)(((uint64_t)x.hi[3] << 32) | x.hi[2]);
    } else if (DT == SDP_F32) {
#pragma unroll
        for (int m = 0; m < 4; ++m) v[m] = (double)__uint_as_float(x.lo[m]);
    } else if (DT == SDP_I32) {
#pragma unroll
        for (int m = 0; m < 4; ++m) v[m] = (double)(int32_t)x.lo[m];
    } else {
        conv4(DT, Raw4{x.lo, x.hi}, v);
    }
    double y[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) y[m] = ((kb >> m) & 1u) ? v[m] - K : 0.0;
    csum += (y[0] + y[1]) + (y[2] + y[3]);
    *(d4u *)dst = d4u{y[0], y[1], y[2], y[3]};
}
__device__ __forceinline__ void g16_stage_any(int dt, const GwRaw &x, uint32_t kb, double K, double &csum,
                                              double *dst) {
    switch (dt) {                                      // wave-uniform
    case SDP_F64: g16_stage<SDP_F64>(x, kb, K, csum, dst); break;
    case SDP_I64: g16_stage<SDP_I64>(x, kb, K, csum, dst); break;
    case SDP_F32: g16_stage<SDP_F32>(x, kb, K, csum, dst); break;
    case SDP_I32: g16_stage<SDP_I32>(x, kb, K, csum, dst); break;
    case SDP_U32: g16_stage<SDP_U32>(x, kb, K, csum, dst); break;
    case SDP_I16: g16_stage<SDP_I16>(x, kb, K, csum, dst); break;
    case SDP_U16: g16_stage<SDP_U16>(x, kb, K, csum, dst); break;
    case SDP_I8: g16_stage<SDP_I8>(x, kb, K, csum, dst); break;
    case SDP_U8: g16_stage<SDP_U8>(x, kb, K, csum, dst); break;
    default: *(d4u *)dst = d4u{0.0, 0.0, 0.0, 0.0};   // padding column
    }
}

__global__ void __launch_bounds__(G16_BLOCK, 4 / G16_Q) gram16_kernel(const GramCol *cols, int ncols, const double *shift,
                                                            const uint32_t *keep, int64_t n, int64_t rows_per_chunk,
                                                            double *part_g, double *part_cs, double *part_n) {
    __shared__ double s_y[16 * G16_P];
    const int s = blockIdx.x;
    const int lane = lane_id();
    const int wid = (int)uniform_u32(threadIdx.x / WAVE);
    const int q = lane >> 4, cl = lane & 15;
    const int64_t c0 = (int64_t)s * rows_per_chunk;
    const int64_t c1 = min(n, c0 + rows_per_chunk);

    // the wave's columns wid, wid + 4, wid + 8, wid + 12 (dtype 0: padding, staged as zeros)
    GramCol gc[G16_CPW];
    double K[G16_CPW];
#pragma unroll
    for (int j = 0; j < G16_CPW; ++j) {
        const int c = wid + G16_W * j;
        gc[j] = c < ncols ? cols[c] : GramCol{nullptr, 0, 0};
        K[j] = c < ncols ? shift[c] : 0.0;
    }
    double csum[G16_CPW];
#pragma unroll
    for (int j = 0; j < G16_CPW; ++j) csum[j] = 0.0;
    double nkeep = 0.0;
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};   // (one chain: the f64 MFMA issue rate, not its latency, bounds it)

    GwRaw raw[G16_QN][G16_CPW];
    uint32_t kw[G16_QN];
    auto load = [&](int64_t r0) {
        const bool whole = r0 + G16_R <= c1;           // wave-uniform: a whole k-step
#pragma unroll
        for (int k = 0; k < G16_QN; ++k) {
            const int64_t r = r0 + 4 * lane + 4 * WAVE * k;
            if (whole) {
                kw[k] = keep[r >> 5];
#pragma unroll
                for (int j = 0; j < G16_CPW; ++j) {
                    const char *b = (const char *)gc[j].p + r * gc[j].width;
                    switch (gc[j].width) {
                    case 8:
                        raw[k][j].lo = *(const __attribute__((address_space(1))) u32x4 *)b;
                        raw[k][j].hi = *(const __attribute__((address_space(1))) u32x4 *)(b + 16);
                        break;
                    case 4: raw[k][j].lo = *(const __attribute__((address_space(1))) u32x4 *)b; break;
                    case 2: {
                        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                        const u32x2 v = *(const __attribute__((address_space(1))) u32x2 *)b;
                        raw[k][j].lo[0] = v[0];
                        raw[k][j].lo[1] = v[1];
                    } break;
                    case 1: raw[k][j].lo[0] = *(const __attribute__((address_space(1))) uint32_t *)b; break;
                    default: break;                    // padding column
                    }
                }
            } else {
                kw[k] = r < c1 ? keep[r >> 5] : 0u;
#pragma unroll
                for (int j = 0; j < G16_CPW; ++j) {
                    raw[k][j].lo = u32x4{0, 0, 0, 0};
                    raw[k][j].hi = u32x4{0, 0, 0, 0};
                    if (r < n) gw_load(gc[j], r, n, raw[k][j]);
                }
            }
        }
    };
    if (c0 < c1) load(c0);
    for (int64_t r0 = c0; r0 < c1; r0 += G16_R) {
        uint32_t kb[G16_QN];
#pragma unroll
        for (int k = 0; k < G16_QN; ++k) {
            const int64_t r = r0 + 4 * lane + 4 * WAVE * k;
            kb[k] = (kw[k] >> (r & 31)) & 0xFu;
            if (r0 + G16_R > c1) kb[k] &= r >= c1 ? 0u : (r + 4 > c1 ? (1u << (int)(c1 - r)) - 1u : 0xFu);
            if (wid == 0) nkeep += (double)__popc(kb[k]);
        }
        // (LDS-only barriers: __syncthreads()' release fence waited vmcnt(0),
        // draining the next k-step's loads issued just before the second one --
        // the prefetch never overlapped the MFMAs)
        lds_barrier();                                 // the previous k-step's operand reads are done
#pragma unroll
        for (int k = 0; k < G16_QN; ++k)
#pragma unroll
            for (int j = 0; j < G16_CPW; ++j)
                g16_stage_any(gc[j].dtype, raw[k][j], kb[k], K[j], csum[j],
                              &s_y[(wid + G16_W * j) * G16_P + 4 * lane + 4 * WAVE * k]);
        if (r0 + G16_R < c1) load(r0 + G16_R);
        lds_barrier();
        // this wave's row groups wid + 4 g: MFMA m takes row 4q + m of the group
#pragma unroll
        for (int g = 0; g < 4 * G16_QN; ++g) {
            const d4u v = *(const d4u *)&s_y[cl * G16_P + 16 * (wid + G16_W * g) + 4 * q];
#pragma unroll
            for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v[m], v[m], acc, 0, 0, 0);
        }
    }
    // ---- combine the 4 waves (fixed order), write the chunk partial ----
    __syncthreads();
    double *s_acc = s_y;                               // 4 x 256 doubles
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_acc[wid * 256 + (q + 4 * rr) * 16 + cl] = acc[rr];
    __syncthreads();
    {
        const int e = threadIdx.x;                     // G16_BLOCK == 256 entries
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < G16_W; ++w) v += s_acc[w * 256 + e];
        part_g[(int64_t)s * 256 + e] = v;
    }
    // column sums: wave wid holds columns wid + 4 j
#pragma unroll
    for (int j = 0; j < G16_CPW; ++j) {
        const double v = wave_sum_f64(csum[j]);
        if (lane == 0) part_cs[(int64_t)s * 16 + wid + G16_W * j] = v;
    }
    if (wid == 0) {
        const double v = wave_sum_f64(nkeep);
        if (lane == 0) part_n[s] = v;
    }
}

// KIND: GW_GENERIC (any dtype mix, element-wise tail), GW_F32 / GW_F64 (every
// column of the tile has that dtype and the chunk holds no ragged tail: the
// staging is branch-free -- row addresses are clamped into the column and the
// rows past n are zeroed by their keep bits, absent columns read column 0 and
// are zeroed by their slot mask -- so the k-loop stays one basic block and the
// compiler can hoist the next group's LDS operand reads over the MFMAs).
constexpr int GW_GENERIC = 0, GW_F32 = 1, GW_F64 = 2;

template <bool DIAG, int KIND>
__device__ __forceinline__ void gram_wide_unit(int L, const GramCol *cols, int ncols, const double *shift,
                                               const uint32_t *keep, int64_t n, int side, int T,
                                               int64_t rows_per_chunk, double *part_g, double *part_cs,
                                               double *part_n, double (*pa)[GW_TILE * GW_PITCH],
                                               double (*pb)[GW_TILE * GW_PITCH]) {
    const int s = L / T, t = L % T;
    int ti = 0, rem = t;
    while (rem >= side - ti) { rem -= side - ti; ++ti; }
    const int tj = ti + rem;
    constexpr bool diag = DIAG;
    const int tid = threadIdx.x, lane = lane_id();
    const int wid = (int)uniform_u32(tid / WAVE);
    const int q = lane >> 4, cl = lane & 15;
    const int qa = wid >> 2, qb = wid & 3;
    constexpr int NSLOT = DIAG ? GW_SLOTS / 2 : GW_SLOTS;    // diagonal tiles stage panel A only
    const int squad = tid & 7;                         // the same quad in every slot

    GramCol sc[NSLOT];
    double sk[NSLOT];
    uint32_t smask[NSLOT];                             // 0xF for a real column, 0 for padding
#pragma unroll
    for (int i = 0; i < NSLOT; ++i) {
        const int c = (tid + GW_BLOCK * i) >> 3;
        const int gc = (c >= GW_TILE ? tj : ti) * GW_TILE + (c & (GW_TILE - 1));
        const bool v = gc < ncols;
        sc[i] = v ? cols[gc] : (KIND == GW_GENERIC ? GramCol{nullptr, 0, 0} : cols[0]);
        sk[i] = v ? shift[gc] : 0.0;
        smask[i] = v ? 0xFu : 0u;
    }
    double csum[NSLOT];
#pragma unroll
    for (int i = 0; i < NSLOT; ++i) csum[i] = 0.0;
    double nkeep = 0.0;

    // off-diagonal: acc[2a + b] is block (a, b) of the 64 x 32 quadrant;
    // diagonal: acc[j] is block GW_DIAG_BLK[wid][j] of the tile
    constexpr int NACC = DIAG ? 5 : 8;
    d4 acc[NACC];
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = d4{0.0, 0.0, 0.0, 0.0};
    const int dn = diag ? (int)GW_DIAG_N[wid] : 0;
    int dbi[5], dbj[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int blk = diag ? (int)GW_DIAG_BLK[wid][j] : 0;
        dbi[j] = blk >> 3;
        dbj[j] = blk & 7;
    }

    const int64_t c0 = (int64_t)s * rows_per_chunk;
    const int64_t c1 = min(n, c0 + rows_per_chunk);
    const int64_t rlast = (n & ~(int64_t)3) - 4;       // last whole 4-row group (fast kinds: n >= 4)
    GwRaw raw[NSLOT];
    auto load_slot = [&](int i, int64_t r0) {
        const int64_t r = r0 + 4 * squad;
        if (KIND == GW_F32) {
            const int64_t rc = r < rlast ? r : rlast;
            raw[i].lo = *(const __attribute__((address_space(1))) u32x4 *)((const char *)sc[i].p + rc * 4);
        } else if (KIND == GW_F64) {
            const int64_t rc = r < rlast ? r : rlast;
            const __attribute__((address_space(1))) u32x4 *b =
                (const __attribute__((address_space(1))) u32x4 *)((const char *)sc[i].p + rc * 8);
            raw[i].lo = b[0];
            raw[i].hi = b[1];
        } else {
            raw[i].lo = u32x4{0, 0, 0, 0};
            raw[i].hi = u32x4{0, 0, 0, 0};
            gw_load(sc[i], r, n, raw[i]);
        }
    };
    // converts slot i (rows of the k-step whose keep word is kw) into buffer `buf`
    auto stage_slot = [&](int i, uint32_t kw, int buf) {
        const int c = (tid + GW_BLOCK * i) >> 3;
        const uint32_t kb = (kw >> (4 * squad)) & smask[i];
        double x[4];
        if (KIND == GW_F32) {
#pragma unroll
            for (int m = 0; m < 4; ++m) x[m] = (double)__uint_as_float(raw[i].lo[m]);
        } else if (KIND == GW_F64) {
            x[0] = __longlong_as_double((long long)(((uint64_t)raw[i].lo[1] << 32) | raw[i].lo[0]));
            x[1] = __longlong_as_double((long long)(((uint64_t)raw[i].lo[3] << 32) | raw[i].lo[2]));
            x[2] = __longlong_as_double((long long)(((uint64_t)raw[i].hi[1] << 32) | raw[i].hi[0]));
            x[3] = __longlong_as_double((long long)(((uint64_t)raw[i].hi[3] << 32) | raw[i].hi[2]));
        } else if (common_dtype(sc[i].dtype)) {
            conv4_common(sc[i].width == 8, sc[i].dtype == SDP_F64 || sc[i].dtype == SDP_F32,
                         Raw4{raw[i].lo, raw[i].hi}, x);
        } else {
            conv4(sc[i].dtype, Raw4{raw[i].lo, raw[i].hi}, x);
        }
        double y[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) y[m] = ((kb >> m) & 1u) ? x[m] - sk[i] : 0.0;
        if (diag) csum[i] += (y[0] + y[1]) + (y[2] + y[3]);
        double *dst = (c < GW_TILE ? pa[buf] : pb[buf]) + (c & (GW_TILE - 1)) * GW_PITCH + 4 * squad;
        *(d4u *)dst = d4u{y[0], y[1], y[2], y[3]};
    };
    // MFMA operands of 4-row group kk out of buffer `buf`
    auto read_ops = [&](int buf, int kk, double (&va)[4], double (&vb)[4]) {
        const double *A = pa[buf];
        const double *B = diag ? pa[buf] : pb[buf];
        if (!diag) {
#pragma unroll
            for (int a = 0; a < 4; ++a) va[a] = A[(64 * qa + 16 * a + cl) * GW_PITCH + 4 * kk + q];
#pragma unroll
            for (int b = 0; b < 2; ++b) vb[b] = B[(32 * qb + 16 * b + cl) * GW_PITCH + 4 * kk + q];
        }
    };

    if (c0 < c1) {
        // prologue: k-step 0 staged, k-step 1 in flight
        const uint32_t kw0 = keep[c0 >> 5];
#pragma unroll
        for (int i = 0; i < NSLOT; ++i) load_slot(i, c0);
#pragma unroll
        for (int i = 0; i < NSLOT; ++i) {
            stage_slot(i, kw0, 0);
            if (c0 + GW_KR < c1) load_slot(i, c0 + GW_KR);
        }
        if (diag && ti == 0 && tid == 0) nkeep += (double)__popc(kw0);
        lds_barrier();
    }
    int cur = 0;
    for (int64_t r0 = c0; r0 < c1; r0 += GW_KR) {
        const bool has1 = r0 + GW_KR < c1, has2 = r0 + 2 * GW_KR < c1;
        const uint32_t kw1 = has1 ? keep[(r0 + GW_KR) >> 5] : 0u;
        double va[2][4], vb[2][4];
        read_ops(cur, 0, va[0], vb[0]);
#pragma unroll
        for (int kk = 0; kk < GW_KR / 4; ++kk) {
            if (kk + 1 < GW_KR / 4) read_ops(cur, kk + 1, va[(kk + 1) & 1], vb[(kk + 1) & 1]);
            if (!diag) {
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc[2 * a + b] = __builtin_amdgcn_mfma_f64_16x16x4f64(va[kk & 1][a], vb[kk & 1][b],
                                                                              acc[2 * a + b], 0, 0, 0);
            } else {
                const double *A = pa[cur];
#pragma unroll
                for (int j = 0; j < NACC; ++j) {
                    if (j < dn) {                      // wave-uniform
                        const double x = A[(16 * dbi[j] + cl) * GW_PITCH + 4 * kk + q];
                        const double y = A[(16 * dbj[j] + cl) * GW_PITCH + 4 * kk + q];
                        acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[j], 0, 0, 0);
                    }
                }
            }
            // between MFMA groups: convert one slot of the next k-step, then
            // reuse its registers for the k-step after that (a full k-step of
            // matrix work before they are needed)
            constexpr int EVERY = (GW_KR / 4) / NSLOT;
            if ((kk % EVERY) == EVERY - 1 && has1) {
                const int i = kk / EVERY;
                stage_slot(i, kw1, cur ^ 1);
                if (has2) load_slot(i, r0 + 2 * GW_KR);
            }
        }
        if (has1 && diag && ti == 0 && tid == 0) nkeep += (double)__popc(kw1);
        lds_barrier();                                 // next buffer written, this one read by all waves
        cur ^= 1;
    }

    // this wave's blocks of the chunk partial
    double *pg = part_g + (int64_t)L * GW_TILE * GW_TILE;
    if (!diag) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int i = 64 * qa + 16 * a + q + 4 * rr, j = 32 * qb + 16 * b + cl;
                    pg[i * GW_TILE + j] = acc[2 * a + b][rr];
                }
    } else {
#pragma unroll
        for (int jb = 0; jb < NACC; ++jb)
            if (jb < dn) {
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int i = 16 * dbi[jb] + q + 4 * rr, j = 16 * dbj[jb] + cl;
                    pg[i * GW_TILE + j] = acc[jb][rr];
                }
            }
        // column sums: the 8 quads of a column are 8 consecutive lanes
#pragma unroll
        for (int i = 0; i < NSLOT; ++i) {
            double v = csum[i];
            v += __shfl_xor(v, 1, WAVE);
            v += __shfl_xor(v, 2, WAVE);
            v += __shfl_xor(v, 4, WAVE);
            const int c = (tid + GW_BLOCK * i) >> 3;
            if (squad == 0) part_cs[((int64_t)s * side + ti) * GW_TILE + c] = v;
        }
        if (ti == 0 && tid == 0) part_n[s] = nkeep;
    }
}

// Persistent workgroups (one per CU, 136 KiB of LDS each) pull units -- one
// (row chunk, tile) pair each, chunk-major so that concurrently running units
// share their rows in the L2/Infinity Cache -- from an atomic counter until
// none is left.  Units are ~1/16 of a workgroup's share, so the diagonal tiles'
// lighter units and the tail balance out; each unit writes its own partial,
// so the result does not depend on which workgroup ran it.
__global__ void __launch_bounds__(GW_BLOCK, 2) gram_wide_kernel(const GramCol *cols, int ncols, const double *shift,
                                                              const uint32_t *keep, int64_t n, int side, int T,
                                                              int S, int64_t rows_per_chunk, double *part_g,
                                                              double *part_cs, double *part_n,
                                                              unsigned int *next_unit) {
    __shared__ double pa[2][GW_TILE * GW_PITCH];
    __shared__ double pb[2][GW_TILE * GW_PITCH];
    __shared__ int s_unit;
    const int U = S * T;
    // XCD-affine: workgroup b runs on XCD b % 8 (the usual round-robin; for
    // speed only -- any placement is correct) and first drains that XCD's
    // contiguous eighth of the chunk-major units, so the tiles of one row chunk
    // share the XCD's L2; then it helps the other XCDs' ranges.
    const int x0 = (int)(blockIdx.x & 7);
    int d = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            int L = -1;
            while (d < 8) {
                const int x = (x0 + d) & 7;
                const int lo = (int)((int64_t)U * x / 8), hi = (int)((int64_t)U * (x + 1) / 8);
                const int u = lo + (int)atomicAdd(&next_unit[16 * x], 1u);
                if (u < hi) { L = u; break; }
                ++d;                                   // this range is drained (counters only grow)
            }
            s_unit = L;
        }
        __syncthreads();
        const int L = s_unit;
        __syncthreads();                           // everyone has read s_unit before it is rewritten
        if (L < 0) return;
        int ti = 0, rem = L % T;                   // diagonal tiles take their own instantiation
        while (rem >= side - ti) { rem -= side - ti; ++ti; }
        const int tj = ti + rem;
        // uniform dtype kind of the tile's columns (padding columns count as any kind)
        int f32 = 1, f64 = 1;
        for (int c = threadIdx.x; c < 2 * GW_TILE; c += GW_BLOCK) {
            const int gc = (c >= GW_TILE ? tj : ti) * GW_TILE + (c & (GW_TILE - 1));
            if (gc < ncols) {
                f32 &= cols[gc].dtype == SDP_F32;
                f64 &= cols[gc].dtype == SDP_F64;
            }
        }
        f32 = __syncthreads_and(f32);
        f64 = __syncthreads_and(f64);
        const int64_t c1 = min(n, (int64_t)(L / T) * rows_per_chunk + rows_per_chunk);
        const bool whole = n >= 4 && c1 <= (n & ~(int64_t)3);   // no ragged tail rows in this chunk
        const int kind = whole && f32 ? GW_F32 : (whole && f64 ? GW_F64 : GW_GENERIC);
#define GW_CALL(D, K) gram_wide_unit<D, K>(L, cols, ncols, shift, keep, n, side, T, rows_per_chunk, part_g, part_cs, \
                                          part_n, pa, pb)
        if (rem == 0) {
            if (kind == GW_F32) GW_CALL(true, GW_F32);
            else if (kind == GW_F64) GW_CALL(true, GW_F64);
            else GW_CALL(true, GW_GENERIC);
        } else {
            if (kind == GW_F32) GW_CALL(false, GW_F32);
            else if (kind == GW_F64) GW_CALL(false, GW_F64);
            else GW_CALL(false, GW_GENERIC);
        }
#undef GW_CALL
        __syncthreads();                           // the unit's LDS reads are done before the next unit stages
    }
}

// Sum of the S chunk partials of every output entry.  A block owns R_EB
// entries of one tile; each entry's S partials are split into R_P contiguous
// parts summed by separate threads, and the parts are added in part order
// (deterministic for a given S).  One thread per entry looping over S = 8192
// partials took 7 ms; this takes well under 0.1 ms.
constexpr int R_EB = 16;
constexpr int R_P = 16;
__device__ __forceinline__ double sum_parts(const double *base, int64_t stride, int S, double (*red)[R_EB]) {
    const int el = threadIdx.x % R_EB, p = threadIdx.x / R_EB;
    const int s0 = (int)((int64_t)S * p / R_P), s1 = (int)((int64_t)S * (p + 1) / R_P);
    double v = 0.0;
    for (int s = s0; s < s1; ++s) v += base[(int64_t)s * stride];
    red[p][el] = v;
    __syncthreads();
    double tot = 0.0;
    if (p == 0)
        for (int k = 0; k < R_P; ++k) tot += red[k][el];
    __syncthreads();
    return tot;
}

template <int TILE>
__global__ void __launch_bounds__(R_EB * R_P) gram_reduce_kernel(const double *part_g, const double *part_cs,
                                                                const double *part_n, int ncols, int ntiles_side,
                                                                int T, int S, double *G, double *colsum, double *nout) {
    constexpr int EGROUPS = TILE * TILE / R_EB;
    __shared__ double red[R_P][R_EB];
    const int t = blockIdx.x / EGROUPS, eg = blockIdx.x % EGROUPS;
    int ti = 0, rem = t;
    while (rem >= ntiles_side - ti) { rem -= ntiles_side - ti; ++ti; }
    const int tj = ti + rem;
    const int el = threadIdx.x % R_EB, p = threadIdx.x / R_EB;
    const int e = eg * R_EB + el;
    const double v = sum_parts(part_g + (int64_t)t * TILE * TILE + e, (int64_t)T * TILE * TILE, S, red);
    if (p == 0) {
        const int i = ti * TILE + e / TILE, j = tj * TILE + e % TILE;
        // diagonal tiles: the upper triangle (the wide kernel leaves the lower
        // quadrants unwritten; the narrow kernels' are bitwise mirrors)
        if (i < ncols && j < ncols && (ti != tj || i <= j)) {
            G[(int64_t)i * ncols + j] = v;
            G[(int64_t)j * ncols + i] = v;
        }
    }
    if (ti == tj && eg < TILE / R_EB) {       // column sums of this diagonal tile
        const double c = sum_parts(part_cs + (int64_t)ti * TILE + e, (int64_t)ntiles_side * TILE, S, red);
        if (p == 0 && ti * TILE + e < ncols) colsum[ti * TILE + e] = c;
    }
    if (t == 0 && eg == 0) {                  // kept rows
        const double c = sum_parts(part_n, 1, S, red);
        if (threadIdx.x == 0) *nout = c;
    }
}

struct GramGeom {
    int tile, side, T, S;
    int64_t rows_per_chunk;
};

static GramGeom gram_geom(int64_t n, int ncols) {
    GramGeom g;
    if (ncols > 64) {
        // wide kernel: ~4096 (chunk, tile) units pulled by 256 persistent
        // workgroups, chunks of whole k-steps
        g.tile = GW_TILE;
        g.side = (ncols + GW_TILE - 1) / GW_TILE;
        g.T = g.side * (g.side + 1) / 2;
        int64_t S = (4096 + g.T - 1) / g.T;
        const int64_t max_s = (n + 4095) / 4096;
        if (S > max_s) S = max_s;
        if (S < 1) S = 1;
        int64_t rpc = (n + S - 1) / S;
        rpc = (rpc + GW_KR - 1) / GW_KR * GW_KR;
        if (rpc < GW_KR) rpc = GW_KR;
        g.S = (int)((n + rpc - 1) / rpc);
        if (g.S < 1) g.S = 1;
        g.rows_per_chunk = rpc;
        return g;
    }
    g.tile = ncols <= 16 ? 16 : (ncols <= 32 ? 32 : 64);
    g.side = (ncols + g.tile - 1) / g.tile;
    g.T = g.side * (g.side + 1) / 2;
    // enough workgroups for several rounds at full occupancy (a single
    // 1024-workgroup round left a tail when fewer than 4 waves/SIMD fit)
    const int64_t target = 4096;
    int64_t S = (target + g.T - 1) / g.T;
    const int64_t min_rows = 4096;
    const int64_t max_s = (n + min_rows - 1) / min_rows;
    if (S > max_s) S = max_s;
    if (S < 1) S = 1;
    int64_t rpc = (n + S - 1) / S;
    const int64_t kstep = g.tile == 16 ? G16_R : 64;   // whole k-steps (gram16) / k-blocks per wave group
    rpc = (rpc + kstep - 1) / kstep * kstep;
    if (rpc < kstep) rpc = kstep;
    g.S = (int)((n + rpc - 1) / rpc);
    if (g.S < 1) g.S = 1;
    g.rows_per_chunk = rpc;
    return g;
}

static int gram_width(int dt) {
    switch (dt) {
    case SDP_F64: case SDP_I64: return 8;
    case SDP_F32: case SDP_I32: case SDP_U32: return 4;
    case SDP_I16: case SDP_U16: return 2;
    default: return 1;
    }
}

static int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }

}  // namespace sdp

using namespace sdp;

extern "C" int64_t sdp_gram_workspace_bytes(int64_t length, int32_t ncols) {
    if (ncols < 1 || length < 0) return -1;
    const GramGeom g = gram_geom(length, ncols);
    int64_t b = align256((int64_t)ncols * sizeof(GramCol));
    b += align256((int64_t)g.S * g.T * g.tile * g.tile * sizeof(double));
    b += align256((int64_t)g.S * g.side * g.tile * sizeof(double));
    b += align256((int64_t)g.S * sizeof(double));
    b += align256((int64_t)ncols * sizeof(MaskCol));
    b += 512;                                       // wide kernel's per-XCD unit counters
    return b;
}

extern "C" int sdp_rowmask(const sdp_column *cols, const int32_t *check_nan, int32_t ncols, void *d_work,
                              int64_t work_bytes, uint32_t *d_keep, void *stream) {
    if (ncols < 1) return set_error(SDP_EINVAL, "sdp_rowmask: ncols %d", ncols);
    const int64_t n = cols[0].length;
    for (int i = 1; i < ncols; ++i)
        if (cols[i].length != n) return set_error(SDP_EINVAL, "sdp_rowmask: column lengths differ");
    if (work_bytes < (int64_t)ncols * (int64_t)sizeof(MaskCol)) return set_error(SDP_ECAP, "sdp_rowmask: workspace");
    MaskCol *h = (MaskCol *)malloc(sizeof(MaskCol) * ncols);
    for (int i = 0; i < ncols; ++i) { h[i].c = cols[i]; h[i].check_nan = check_nan ? check_nan[i] : 1; h[i]._pad = 0; }
    hipStream_t s = (hipStream_t)stream;
    const hipError_t e = put_descs<MaskCol, 32>(h, ncols, (MaskCol *)d_work, s);
    free(h);
    if (e != hipSuccess) return set_error(SDP_EHIP, "sdp_rowmask: %s", hipGetErrorString(e));
    const int64_t nwords = (n + 31) / 32;
    int64_t grid = (nwords + 255) / 256;
    if (grid > 4096) grid = 4096;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(rowmask_kernel, dim3((unsigned)grid), dim3(256), 0, s, (const MaskCol *)d_work, ncols, n, d_keep);
    return check_launch("rowmask_kernel");
}

extern "C" int sdp_gram(const sdp_column *cols, int32_t ncols, const uint32_t *d_keep, const double *d_shift,
                        void *d_work, int64_t work_bytes, double *d_gram, double *d_colsum, double *d_n,
                        void *stream) {
    if (ncols < 1) return set_error(SDP_EINVAL, "sdp_gram: ncols %d", ncols);
    const int64_t n = cols[0].length;
    for (int i = 0; i < ncols; ++i) {
        if (cols[i].length != n) return set_error(SDP_EINVAL, "sdp_gram: column lengths differ");
        if (!aligned16(cols[i].d_values)) return set_error(SDP_EALIGN, "sdp_gram: column %d not 16-B aligned", i);
        if (cols[i].dtype == SDP_U64 || cols[i].dtype == SDP_BOOL || cols[i].dtype < SDP_I8 || cols[i].dtype > SDP_U32)
            return set_error(SDP_EINVAL, "sdp_gram: column %d dtype %d", i, cols[i].dtype);
    }
    const int64_t need = sdp_gram_workspace_bytes(n, ncols);
    if (work_bytes < need) return set_error(SDP_ECAP, "sdp_gram: workspace %lld < %lld", (long long)work_bytes,
                                            (long long)need);
    const GramGeom g = gram_geom(n, ncols);
    char *w = (char *)d_work;
    GramCol *d_cols = (GramCol *)w;
    w += align256((int64_t)ncols * sizeof(GramCol));
    double *pg = (double *)w;
    w += align256((int64_t)g.S * g.T * g.tile * g.tile * sizeof(double));
    double *pcs = (double *)w;
    w += align256((int64_t)g.S * g.side * g.tile * sizeof(double));
    double *pn = (double *)w;
    GramCol *h = (GramCol *)malloc(sizeof(GramCol) * ncols);
    for (int i = 0; i < ncols; ++i) { h[i].p = cols[i].d_values; h[i].dtype = cols[i].dtype; h[i].width = gram_width(cols[i].dtype); }
    hipStream_t s = (hipStream_t)stream;
    const hipError_t e = put_descs<GramCol, 128>(h, ncols, d_cols, s);
    free(h);
    if (e != hipSuccess) return set_error(SDP_EHIP, "sdp_gram: %s", hipGetErrorString(e));
    if (g.tile == GW_TILE) {
        // per-XCD unit counters (64 B apart): the last 512 bytes of the workspace
        unsigned int *ctr = (unsigned int *)((char *)d_work + sdp_gram_workspace_bytes(n, ncols) - 512);
        hipError_t me = hipMemsetAsync(ctr, 0, 512, s);
        if (me != hipSuccess) return set_error(SDP_EHIP, "sdp_gram: %s", hipGetErrorString(me));
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
        const int G = g.S * g.T;
        const int wg = cus < G ? cus : G;
        hipLaunchKernelGGL(gram_wide_kernel, dim3((unsigned)wg), dim3(GW_BLOCK), 0, s, d_cols, ncols, d_shift, d_keep,
                           n, g.side, g.T, g.S, g.rows_per_chunk, pg, pcs, pn, ctr);
        int rcw = check_launch("gram_wide_kernel");
        if (rcw) return rcw;
        hipLaunchKernelGGL(gram_reduce_kernel<GW_TILE>, dim3(g.T * (GW_TILE * GW_TILE / R_EB)), dim3(R_EB * R_P), 0, s,
                           pg, pcs, pn, ncols, g.side, g.T, g.S, d_gram, d_colsum, d_n);
        return check_launch("gram_reduce_kernel");
    }
    const dim3 grid((unsigned)(g.S * g.T));
    switch (g.tile) {
    case 16:
        hipLaunchKernelGGL(gram16_kernel, grid, dim3(G16_BLOCK), 0, s, d_cols, ncols, d_shift, d_keep, n,
                           g.rows_per_chunk, pg, pcs, pn);
        break;
    case 32:
        hipLaunchKernelGGL(gram_kernel<32>, grid, dim3(G_BLOCK), 0, s, d_cols, ncols, d_shift, d_keep, n, g.side, g.T,
                           g.rows_per_chunk, pg, pcs, pn);
        break;
    default:
        hipLaunchKernelGGL(gram_kernel<64>, grid, dim3(G_BLOCK), 0, s, d_cols, ncols, d_shift, d_keep, n, g.side, g.T,
                           g.rows_per_chunk, pg, pcs, pn);
    }
    int rc = check_launch("gram_kernel");
    if (rc) return rc;
    switch (g.tile) {
    case 16:
        hipLaunchKernelGGL(gram_reduce_kernel<16>, dim3(g.T * (16 * 16 / R_EB)), dim3(R_EB * R_P), 0, s, pg, pcs, pn, ncols, g.side, g.T, g.S,
                           d_gram, d_colsum, d_n);
        break;
    case 32:
        hipLaunchKernelGGL(gram_reduce_kernel<32>, dim3(g.T * (32 * 32 / R_EB)), dim3(R_EB * R_P), 0, s, pg, pcs, pn, ncols, g.side, g.T, g.S,
                           d_gram, d_colsum, d_n);
        break;
    default:
        hipLaunchKernelGGL(gram_reduce_kernel<64>, dim3(g.T * (64 * 64 / R_EB)), dim3(R_EB * R_P), 0, s, pg, pcs, pn, ncols, g.side, g.T, g.S,
                           d_gram, d_colsum, d_n);
    }
    return check_launch("gram_reduce_kernel");
}
