// sdp_bitmap.hip -- exact countDistinct of small-range integral columns.
//
// Replaces countDistinct (describe.py:143) for tinyint/smallint/int/bigint and
// date columns whose value range R = max - min + 1 (known from pass 1) is at
// most SDP_BITMAP_MAX_BITS.  One bit per possible value instead of a hash table:
//
//   bitmap_rows   each workgroup streams a contiguous row range with 16-byte
//                 loads and ORs bit (v - lo) into an LDS bitmap (ds_or_b32, no
//                 global atomics), then writes the bitmap to its own slice of
//                 the workspace (coalesced, no atomics)
//   bitmap_reduce OR of the slices word by word + popcount
//
// The kernel reads the column once (w + 1/8 bytes per row) and writes
// grid x R/8 bytes of partial bitmaps; it is HBM-bound for R up to 2^20.
#include "sdp_common.h"

namespace sdp {

constexpr int BM_T = 1024;                       // threads per bitmap workgroup
constexpr int BM_SMALL_WORDS = 2048;             // 64 K values, 8 KB of LDS
constexpr int BM_LARGE_WORDS = SDP_BITMAP_MAX_BITS / 32;   // 1 M values, 128 KB
constexpr int BM_UNROLL = 4;                     // 16-byte loads in flight per lane

template <typename T, int WORDS>
__global__ void __launch_bounds__(BM_T) bitmap_rows_kernel(sdp_column col, int64_t lo, int64_t range,
                                                           int64_t rows_per_block, uint32_t *partial) {
    __shared__ uint32_t bm[WORDS];
    const int t = threadIdx.x;
    const int nw = (int)((range + 31) >> 5);
    for (int i = t; i < nw; i += BM_T) bm[i] = 0u;
    __syncthreads();
    constexpr int VPT = Vec16<T>::N;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(col.length, r0 + rows_per_block);
    const Vec16<T> *vals = (const Vec16<T> *)col.d_values;
    // r0 is a multiple of VPT (rows_per_block is); full vectors first
    const int64_t v0 = r0 / VPT, v1 = r1 / VPT;
    for (int64_t vb = v0; vb < v1; vb += (int64_t)BM_T * BM_UNROLL) {
        Vec16<T> v[BM_UNROLL];
        uint32_t ok[BM_UNROLL];
#pragma unroll
        for (int u = 0; u < BM_UNROLL; ++u) {
            const int64_t vi = vb + (int64_t)u * BM_T + t;
            ok[u] = 0;
            if (vi < v1) {
                v[u] = vals[vi];
                ok[u] = valid_bits(col.d_validity, col.validity_bit_offset, vi * VPT, VPT);
            }
        }
#pragma unroll
        for (int u = 0; u < BM_UNROLL; ++u)
#pragma unroll
            for (int e = 0; e < VPT; ++e)
                if ((ok[u] >> e) & 1u) {
                    const uint64_t d = (uint64_t)((int64_t)v[u].v[e] - lo);
                    if (d < (uint64_t)range) atomicOr(&bm[d >> 5], 1u << (d & 31));
                }
    }
    // tail rows (fewer than one vector)
    for (int64_t i = v1 * VPT + t; i < r1; i += BM_T) {
        if (!valid_bit(col.d_validity, col.validity_bit_offset, i)) continue;
        const uint64_t d = (uint64_t)((int64_t)((const T *)col.d_values)[i] - lo);
        if (d < (uint64_t)range) atomicOr(&bm[d >> 5], 1u << (d & 31));
    }
    __syncthreads();
    uint32_t *dst = partial + (int64_t)blockIdx.x * nw;
    for (int i = t; i < nw; i += BM_T) dst[i] = bm[i];
}

__global__ void __launch_bounds__(256) bitmap_reduce_kernel(const uint32_t *partial, int nw, int nparts,
                                                            uint32_t *d_bitmap, uint64_t *d_out) {
    const int w = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    if (w < nw) {
        for (int p = 0; p < nparts; ++p) acc |= partial[(int64_t)p * nw + w];
        if (d_bitmap) d_bitmap[w] = acc;
    }
    uint64_t c = wave_sum_u64((uint64_t)__popc(acc));
    if (lane_id() == 0 && c) atomicAdd((unsigned long long *)d_out, (unsigned long long)c);
}

static int bitmap_grid(int64_t length, int64_t range) {
    // one 128 KB workgroup per CU for large ranges; several per CU for small ones
    const int64_t per_cu = range <= (int64_t)BM_SMALL_WORDS * 32 ? 2 : 1;   // 16 waves each
    int64_t g = 256 * per_cu;
    const int64_t min_rows = (int64_t)BM_T * 16 * 4;       // keep >= 64 K rows per block
    if (length / min_rows < g) g = length / min_rows;
    return (int)(g < 1 ? 1 : g);
}

template <typename T>
static void launch_bitmap(const sdp_column &c, int64_t lo, int64_t range, int grid, int64_t rpb, uint32_t *partial,
                          hipStream_t s) {
    if (range <= (int64_t)BM_SMALL_WORDS * 32)
        hipLaunchKernelGGL((bitmap_rows_kernel<T, BM_SMALL_WORDS>), dim3(grid), dim3(BM_T), 0, s, c, lo, range, rpb,
                           partial);
    else
        hipLaunchKernelGGL((bitmap_rows_kernel<T, BM_LARGE_WORDS>), dim3(grid), dim3(BM_T), 0, s, c, lo, range, rpb,
                           partial);
}

}  // namespace sdp

using namespace sdp;

extern "C" {

int64_t sdp_bitmap_workspace_bytes(int64_t length, int64_t range) {
    if (range < 1) range = 1;
    return (int64_t)bitmap_grid(length, range) * ((range + 31) / 32) * 4;
}

int sdp_distinct_bitmap(const sdp_column *col, int64_t lo, int64_t range, void *d_work, int64_t work_bytes,
                        uint32_t *d_bitmap, uint64_t *d_out, void *stream) {
    if (col == nullptr || d_out == nullptr || range < 1 || range > SDP_BITMAP_MAX_BITS)
        return set_error(SDP_EINVAL, "distinct_bitmap: args (range %lld)", (long long)range);
    if (work_bytes < sdp_bitmap_workspace_bytes(col->length, range))
        return set_error(SDP_ECAP, "distinct_bitmap: workspace too small");
    if (!aligned16(col->d_values)) return set_error(SDP_EALIGN, "distinct_bitmap: values not 16-byte aligned");
    if (col->length < 1) return 0;
    const int grid = bitmap_grid(col->length, range);
    // rows per block: a multiple of 16 so every block starts on a vector boundary
    int64_t rpb = (col->length + grid - 1) / grid;
    rpb = (rpb + 15) & ~(int64_t)15;
    const int nblocks = (int)((col->length + rpb - 1) / rpb);
    uint32_t *partial = (uint32_t *)d_work;
    hipStream_t s = (hipStream_t)stream;
    switch (col->dtype) {
    case SDP_I64: launch_bitmap<int64_t>(*col, lo, range, nblocks, rpb, partial, s); break;
    case SDP_I32: launch_bitmap<int32_t>(*col, lo, range, nblocks, rpb, partial, s); break;
    case SDP_I16: launch_bitmap<int16_t>(*col, lo, range, nblocks, rpb, partial, s); break;
    case SDP_I8: launch_bitmap<int8_t>(*col, lo, range, nblocks, rpb, partial, s); break;
    case SDP_U32: launch_bitmap<uint32_t>(*col, lo, range, nblocks, rpb, partial, s); break;
    case SDP_U16: launch_bitmap<uint16_t>(*col, lo, range, nblocks, rpb, partial, s); break;
    case SDP_U8: launch_bitmap<uint8_t>(*col, lo, range, nblocks, rpb, partial, s); break;
    default: return set_error(SDP_EINVAL, "distinct_bitmap: dtype %d is not integral", col->dtype);
    }
    if (check_launch("bitmap_rows_kernel")) return SDP_EHIP;
    const int nw = (int)((range + 31) / 32);
    hipLaunchKernelGGL(bitmap_reduce_kernel, dim3((nw + 255) / 256), dim3(256), 0, s, partial, nw, nblocks, d_bitmap,
                       d_out);
    return check_launch("bitmap_reduce_kernel");
}

int sdp_bitmap_reduce(const uint32_t *d_parts, int32_t nparts, int64_t nwords, uint32_t *d_bitmap, uint64_t *d_out,
                      void *stream) {
    if (d_parts == nullptr || d_out == nullptr || nparts < 1 || nwords < 1 || nwords > SDP_BITMAP_MAX_BITS / 32)
        return set_error(SDP_EINVAL, "bitmap_reduce: args");
    hipLaunchKernelGGL(bitmap_reduce_kernel, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       d_parts, (int)nwords, nparts, d_bitmap, d_out);
    return check_launch("bitmap_reduce_kernel");
}

}  // extern "C"
