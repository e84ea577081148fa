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

// ---- Gram ----------------------------------------------------------------------
struct GramCol {
    const void *p;
    int32_t dtype;
    int32_t _pad;
};

// 4 consecutive rows [r, r+4) of column c as doubles (0 beyond n)
__device__ __forceinline__ void load4(const GramCol &gc, int64_t r, int64_t n, double out[4]) {
    if (r + 4 <= n) {
        switch (gc.dtype) {
        case SDP_F64: {
            const double2 *q = (const double2 *)((const double *)gc.p + r);
            const double2 a = q[0], b = q[1];
            out[0] = a.x; out[1] = a.y; out[2] = b.x; out[3] = b.y;
            return;
        }
        case SDP_F32: {
            const float4 a = *(const float4 *)((const float *)gc.p + r);
            out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
            return;
        }
        case SDP_I64: {
            const longlong2 *q = (const longlong2 *)((const int64_t *)gc.p + r);
            const longlong2 a = q[0], b = q[1];
            out[0] = (double)a.x; out[1] = (double)a.y; out[2] = (double)b.x; out[3] = (double)b.y;
            return;
        }
        case SDP_I32: {
            const int4 a = *(const int4 *)((const int32_t *)gc.p + r);
            out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
            return;
        }
        default:
            break;
        }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) out[m] = (r + m < n) ? load_as_double(gc.p, gc.dtype, r + m) : 0.0;
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
        ca[a] = va[a] ? cols[ci] : GramCol{nullptr, 0, 0};
        cb[a] = vb[a] ? cols[cj] : GramCol{nullptr, 0, 0};
        ka[a] = va[a] ? shift[ci] : 0.0;
        kb[a] = vb[a] ? shift[cj] : 0.0;
    }
    d4 acc[NT][NT];
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    double csum[NT];
#pragma unroll
    for (int a = 0; a < NT; ++a) csum[a] = 0.0;
    double nkeep = 0.0;

    const int64_t c0 = (int64_t)s * rows_per_chunk;
    const int64_t c1 = min(n, c0 + rows_per_chunk);
    for (int64_t r0 = c0 + (int64_t)wid * 16; r0 < c1; r0 += (int64_t)G_WAVES * 16) {
        const int64_t r = r0 + 4 * q;
        uint32_t kbits = 0;
        if (r < n) {
            const uint32_t w = keep[r >> 5];
            kbits = (w >> (r & 31)) & 0xFu;
            if (r + 4 > c1) kbits &= (1u << (int)(c1 - r)) - 1u;   // chunk boundary
        }
        if (diag && cl == 0) nkeep += (double)__popc(kbits);
        double xa[NT][4], xb[NT][4];
#pragma unroll
        for (int a = 0; a < NT; ++a) {
            if (va[a]) load4(ca[a], r, n, xa[a]);
            else { xa[a][0] = xa[a][1] = xa[a][2] = xa[a][3] = 0.0; }
#pragma unroll
            for (int m = 0; m < 4; ++m) xa[a][m] = ((kbits >> m) & 1u) ? xa[a][m] - ka[a] : 0.0;
            if (diag) {
#pragma unroll
                for (int m = 0; m < 4; ++m) csum[a] += xa[a][m];
            }
        }
        if (!diag) {
#pragma unroll
            for (int b = 0; b < NT; ++b) {
                if (vb[b]) load4(cb[b], r, n, xb[b]);
                else { xb[b][0] = xb[b][1] = xb[b][2] = xb[b][3] = 0.0; }
#pragma unroll
                for (int m = 0; m < 4; ++m) xb[b][m] = ((kbits >> m) & 1u) ? xb[b][m] - kb[b] : 0.0;
            }
        }
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int a = 0; a < NT; ++a)
#pragma unroll
                for (int b = 0; b < NT; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[a][m], diag ? xa[b][m] : xb[b][m],
                                                                      acc[a][b], 0, 0, 0);
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

template <int TILE>
__global__ void gram_reduce_kernel(const double *part_g, const double *part_cs, const double *part_n, int ncols,
                                   int ntiles_side, int T, int S, double *G, double *colsum, double *nout) {
    const int t = blockIdx.x;
    int ti = 0, rem = t;
    while (rem >= ntiles_side - ti) { rem -= ntiles_side - ti; ++ti; }
    const int tj = ti + rem;
    for (int e = threadIdx.x; e < TILE * TILE; e += blockDim.x) {
        const int i = ti * TILE + e / TILE, j = tj * TILE + e % TILE;
        if (i >= ncols || j >= ncols) continue;
        double v = 0.0;
        for (int s = 0; s < S; ++s) v += part_g[((int64_t)s * T + t) * TILE * TILE + e];
        G[(int64_t)i * ncols + j] = v;
        G[(int64_t)j * ncols + i] = v;
    }
    if (ti == tj) {
        for (int e = threadIdx.x; e < TILE; e += blockDim.x) {
            const int i = ti * TILE + e;
            if (i >= ncols) continue;
            double v = 0.0;
            for (int s = 0; s < S; ++s) v += part_cs[((int64_t)s * ntiles_side + ti) * TILE + e];
            colsum[i] = v;
        }
        if (ti == 0 && threadIdx.x == 0) {
            double v = 0.0;
            for (int s = 0; s < S; ++s) v += part_n[s];
            *nout = v;
        }
    }
}

struct GramGeom {
    int tile, side, T, S;
    int64_t rows_per_chunk;
};

static GramGeom gram_geom(int64_t n, int ncols) {
    GramGeom g;
    g.tile = ncols <= 16 ? 16 : (ncols <= 32 ? 32 : 64);
    g.side = (ncols + g.tile - 1) / g.tile;
    g.T = g.side * (g.side + 1) / 2;
    int64_t S = (1024 + g.T - 1) / g.T;
    const int64_t min_rows = 4096;
    const int64_t max_s = (n + min_rows - 1) / min_rows;
    if (S > max_s) S = max_s;
    if (S < 1) S = 1;
    int64_t rpc = (n + S - 1) / S;
    rpc = (rpc + 63) / 64 * 64;                 // whole k-blocks per wave group
    if (rpc < 64) rpc = 64;
    g.S = (int)((n + rpc - 1) / rpc);
    if (g.S < 1) g.S = 1;
    g.rows_per_chunk = rpc;
    return g;
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
    hipError_t e = hipMemcpyAsync(d_work, h, sizeof(MaskCol) * ncols, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);   // h is pageable and freed below
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
    for (int i = 0; i < ncols; ++i) { h[i].p = cols[i].d_values; h[i].dtype = cols[i].dtype; h[i]._pad = 0; }
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemcpyAsync(d_cols, h, sizeof(GramCol) * ncols, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    free(h);
    if (e != hipSuccess) return set_error(SDP_EHIP, "sdp_gram: %s", hipGetErrorString(e));
    const dim3 grid((unsigned)(g.S * g.T));
    switch (g.tile) {
    case 16:
        hipLaunchKernelGGL(gram_kernel<16>, grid, dim3(G_BLOCK), 0, s, d_cols, ncols, d_shift, d_keep, n, g.side, g.T,
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
        hipLaunchKernelGGL(gram_reduce_kernel<16>, dim3(g.T), dim3(256), 0, s, pg, pcs, pn, ncols, g.side, g.T, g.S,
                           d_gram, d_colsum, d_n);
        break;
    case 32:
        hipLaunchKernelGGL(gram_reduce_kernel<32>, dim3(g.T), dim3(256), 0, s, pg, pcs, pn, ncols, g.side, g.T, g.S,
                           d_gram, d_colsum, d_n);
        break;
    default:
        hipLaunchKernelGGL(gram_reduce_kernel<64>, dim3(g.T), dim3(256), 0, s, pg, pcs, pn, ncols, g.side, g.T, g.S,
                           d_gram, d_colsum, d_n);
    }
    return check_launch("gram_reduce_kernel");
}
