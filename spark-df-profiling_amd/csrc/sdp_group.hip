// sdp_group.hip -- exact distinct counts / value counts by radix-partitioned
// aggregation, all de-duplication in LDS (gfx950).
//
// Replaces countDistinct (describe.py:143) and the groupBy+count of
// describe_categorical_1d (describe.py:251) for columns of any cardinality.
// A global open-addressing table costs one random HBM atomic per row; here the
// rows stream through three kernels and every probe hits LDS:
//
//   part_rows   column -> L1 buckets: each block de-duplicates a 2048-row tile in
//               an LDS table (hot keys of skewed columns collapse to one record
//               per tile), then appends the tile's groups to 2^b1 buckets chosen
//               by the top hash bits (one global atomic per bucket per tile).
//   part_recs   L1 bucket -> L2 buckets by the next b2 hash bits, again with an
//               LDS de-duplication of each 2048-record chunk.
//   dedup       one block per L2 bucket (~2k records): the bucket's groups in an
//               LDS table; group count out, groups compacted in place.
//
// Records are structure-of-arrays: key (u64 key, or the 64-bit hash of a byte
// key), row (byte keys: a representative row for byte comparison), count.
// Byte keys are equal only after a byte-for-byte comparison, so counts are exact.
// The bucket index doubles as the owner rank for the multi-GPU all-to-all.
#include "sdp_common.h"

namespace sdp {

constexpr int GB = 256;               // threads per block
constexpr int GT = 2048;              // rows / records per LDS round
constexpr int GL = 4096;              // LDS table slots (load <= 0.5)
constexpr int GMAXB = 1024;           // max buckets per partition level (b <= 10)
constexpr uint64_t RMASK = (1ull << 40) - 1ull;

// ---- helpers shared with sdp_hash.hip (duplicated as inline device code) ------
__device__ __forceinline__ bool g_fetch_key(const sdp_column &c, int64_t i, uint64_t &key) {
    const bool valid = valid_bit(c.d_validity, c.validity_bit_offset, i);
    switch (c.dtype) {
    case SDP_I8: key = Elem<int8_t>::key(((const int8_t *)c.d_values)[i]); break;
    case SDP_I16: key = Elem<int16_t>::key(((const int16_t *)c.d_values)[i]); break;
    case SDP_I32: key = Elem<int32_t>::key(((const int32_t *)c.d_values)[i]); break;
    case SDP_I64: key = Elem<int64_t>::key(((const int64_t *)c.d_values)[i]); break;
    case SDP_U8: key = ((const uint8_t *)c.d_values)[i]; break;
    case SDP_U16: key = ((const uint16_t *)c.d_values)[i]; break;
    case SDP_U32: key = ((const uint32_t *)c.d_values)[i]; break;
    case SDP_U64: key = ((const uint64_t *)c.d_values)[i]; break;
    case SDP_F32: key = Elem<float>::key(((const float *)c.d_values)[i]); break;
    case SDP_F64: key = Elem<double>::key(((const double *)c.d_values)[i]); break;
    case SDP_BOOL: {
        const int64_t b = c.validity_bit_offset + i;
        key = (((const uint8_t *)c.d_values)[b >> 3] >> (b & 7)) & 1u;
        break;
    }
    default: key = 0;
    }
    return valid;
}

struct BRef {
    const uint8_t *p;
    int64_t len;
};

__device__ __forceinline__ BRef g_bytes_at(const sdp_bytes_column &c, int64_t row) {
    BRef r;
    if (c.fixed_width > 0) {
        r.p = c.d_data + row * (int64_t)c.fixed_width;
        r.len = c.fixed_width;
    } else if (c.offset_width == 8) {
        const int64_t *o = (const int64_t *)c.d_offsets;
        r.p = c.d_data + o[row];
        r.len = o[row + 1] - o[row];
    } else {
        const int32_t *o = (const int32_t *)c.d_offsets;
        r.p = c.d_data + o[row];
        r.len = (int64_t)o[row + 1] - (int64_t)o[row];
    }
    return r;
}

__device__ __forceinline__ uint64_t g_load8(const uint8_t *p, int64_t avail) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    const int sh = (int)(a & 3) * 8;
    const uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    uint64_t v = lo >> sh;
    if (sh) v |= (uint64_t)w[2] << (64 - sh);
    if (avail < 8) v = avail <= 0 ? 0 : (v & ((1ull << (8 * avail)) - 1ull));
    return v;
}

__device__ __forceinline__ uint64_t g_hash_bytes(BRef s) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)s.len * 0xFF51AFD7ED558CCDull);
    int64_t i = 0;
    for (; i + 8 <= s.len; i += 8) h = mix64(h ^ g_load8(s.p + i, 8)) + 0x632BE59BD9B4E019ull;
    if (i < s.len) h = mix64(h ^ g_load8(s.p + i, s.len - i) ^ 0xA0761D6478BD642Full);
    return mix64(h);
}

__device__ __forceinline__ bool g_bytes_equal(BRef a, BRef b) {
    if (a.len != b.len) return false;
    for (int64_t i = 0; i < a.len; i += 8)
        if (g_load8(a.p + i, a.len - i) != g_load8(b.p + i, b.len - i)) return false;
    return true;
}

// ---- LDS group table ----------------------------------------------------------
// u64 keys:  tkey = key (EMPTY64 = empty), thash unused.
// byte keys: tkey = (tag24 << 40) | (row + 1) (0 = empty), thash = full hash.
template <bool BYTES>
struct LTab {
    uint64_t *tkey;
    uint64_t *thash;
    uint32_t *tcnt;
};

template <bool BYTES>
__device__ __forceinline__ void ltab_clear(LTab<BYTES> t) {
    for (int i = threadIdx.x; i < GL; i += blockDim.x) {
        t.tkey[i] = BYTES ? 0ull : EMPTY64;
        t.tcnt[i] = 0;
    }
}

__device__ __forceinline__ bool ltab_empty_u64(uint64_t v) { return v == EMPTY64; }

// returns false only when the table is full (probe wrapped)
__device__ __forceinline__ bool ltab_insert_u64(LTab<false> t, uint64_t key, uint64_t h, uint32_t c) {
    uint32_t pos = (uint32_t)(h & (GL - 1));
    for (int probe = 0; probe < GL; ++probe) {
        const uint64_t old = atomicCAS((unsigned long long *)&t.tkey[pos], (unsigned long long)EMPTY64,
                                       (unsigned long long)key);
        if (old == EMPTY64 || old == key) {
            atomicAdd(&t.tcnt[pos], c);
            return true;
        }
        pos = (pos + 1) & (GL - 1);
    }
    return false;
}

__device__ __forceinline__ bool ltab_insert_bytes(LTab<true> t, const sdp_bytes_column &bc, uint64_t h, int64_t row,
                                                  uint32_t c) {
    const uint64_t tag = h >> 40;
    const uint64_t mine = (tag << 40) | (uint64_t)(row + 1);
    const BRef me = g_bytes_at(bc, row);
    uint32_t pos = (uint32_t)(h & (GL - 1));
    for (int probe = 0; probe < GL; ++probe) {
        uint64_t cur = t.tkey[pos];
        if (cur == 0) {
            const uint64_t old = atomicCAS((unsigned long long *)&t.tkey[pos], 0ull, (unsigned long long)mine);
            if (old == 0) {
                t.thash[pos] = h;
                atomicAdd(&t.tcnt[pos], c);
                return true;
            }
            cur = old;
        }
        if ((cur >> 40) == tag && g_bytes_equal(me, g_bytes_at(bc, (int64_t)(cur & RMASK) - 1))) {
            atomicAdd(&t.tcnt[pos], c);
            return true;
        }
        pos = (pos + 1) & (GL - 1);
    }
    return false;
}

// ---- bucket output buffers ------------------------------------------------------
struct Buckets {
    uint64_t *key;      // [nb][cap]
    uint64_t *row;      // bytes only
    uint64_t *cnt;      // counts (nullable when !COUNTS)
    uint32_t *fill;     // [nb] records appended (may exceed cap: overflow)
    int64_t cap;
};

// Append every occupied LDS slot to bucket ((h >> shift) & (nb-1)) + base_bucket.
template <bool BYTES, bool COUNTS>
__device__ void flush_groups(LTab<BYTES> t, Buckets out, int shift, int nb, int64_t base_bucket,
                             uint32_t *s_hist, uint32_t *s_base, uint32_t *overflow) {
    for (int i = threadIdx.x; i < nb; i += blockDim.x) s_hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < GL; i += blockDim.x) {
        const uint64_t k = t.tkey[i];
        const bool occ = BYTES ? (k != 0) : (k != EMPTY64);
        if (occ) {
            uint64_t h;
            if constexpr (BYTES) h = t.thash[i]; else h = mix64(k);
            atomicAdd(&s_hist[(int)((h >> shift) & (uint64_t)(nb - 1))], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += blockDim.x) {
        const uint32_t c = s_hist[i];
        s_base[i] = c ? atomicAdd(&out.fill[base_bucket + i], c) : 0u;
        s_hist[i] = 0;   // reused as the per-bucket cursor
    }
    __syncthreads();
    for (int i = threadIdx.x; i < GL; i += blockDim.x) {
        const uint64_t k = t.tkey[i];
        const bool occ = BYTES ? (k != 0) : (k != EMPTY64);
        if (occ) {
            uint64_t h;
            if constexpr (BYTES) h = t.thash[i]; else h = mix64(k);
            const int b = (int)((h >> shift) & (uint64_t)(nb - 1));
            const uint32_t r = atomicAdd(&s_hist[b], 1u);
            const int64_t idx = (int64_t)s_base[b] + r;
            if (idx < out.cap) {
                const int64_t o = (base_bucket + b) * out.cap + idx;
                if constexpr (BYTES) { out.key[o] = h; out.row[o] = (k & RMASK) - 1; }
                else out.key[o] = k;
                if (COUNTS) out.cnt[o] = t.tcnt[i];
            } else {
                *overflow = 1u;
            }
        }
    }
    __syncthreads();
}

// stats layout (u64): [0] rows inserted, [1] rows whose key == EMPTY64 (u64 only),
// [2] overflow flag, [3] LDS-full flag
template <bool COUNTS>
__global__ void __launch_bounds__(GB) part_rows_u64_kernel(sdp_column col, Buckets out, int b1, uint64_t *stats) {
    __shared__ uint64_t s_key[GL];
    __shared__ uint32_t s_cnt[GL];
    __shared__ uint32_t s_hist[GMAXB], s_base[GMAXB];
    __shared__ uint32_t s_ovf;
    LTab<false> t{s_key, nullptr, s_cnt};
    if (threadIdx.x == 0) s_ovf = 0;
    const int nb = 1 << b1;
    const int shift = 64 - b1;
    const int64_t n = col.length;
    const int64_t ntiles = (n + GT - 1) / GT;
    uint64_t rows = 0, maxk = 0;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        ltab_clear(t);
        __syncthreads();
        const int64_t base = tile * GT;
        for (int k = threadIdx.x; k < GT; k += blockDim.x) {
            const int64_t i = base + k;
            if (i >= n) break;
            uint64_t key;
            if (!g_fetch_key(col, i, key)) continue;
            ++rows;
            if (key == EMPTY64) { ++maxk; continue; }
            ltab_insert_u64(t, key, mix64(key), 1u);   // a tile has <= GT/2 of GL slots
        }
        __syncthreads();
        flush_groups<false, COUNTS>(t, out, b1 ? shift : 63, b1 ? nb : 1, 0, s_hist, s_base, &s_ovf);
    }
    rows = wave_sum_u64(rows);
    maxk = wave_sum_u64(maxk);
    if (lane_id() == 0) {
        if (rows) atomicAdd((unsigned long long *)&stats[0], (unsigned long long)rows);
        if (maxk) atomicAdd((unsigned long long *)&stats[1], (unsigned long long)maxk);
    }
    if (threadIdx.x == 0 && s_ovf) atomicOr((unsigned long long *)&stats[2], 1ull);
}

__global__ void __launch_bounds__(GB) part_rows_bytes_kernel(sdp_bytes_column col, Buckets out, int b1,
                                                             uint64_t *stats) {
    __shared__ uint64_t s_key[GL];
    __shared__ uint64_t s_hash[GL];
    __shared__ uint32_t s_cnt[GL];
    __shared__ uint32_t s_hist[GMAXB], s_base[GMAXB];
    __shared__ uint32_t s_ovf;
    LTab<true> t{s_key, s_hash, s_cnt};
    if (threadIdx.x == 0) s_ovf = 0;
    const int nb = 1 << b1;
    const int shift = 64 - b1;
    const int64_t n = col.length;
    const int64_t ntiles = (n + GT - 1) / GT;
    uint64_t rows = 0;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        ltab_clear(t);
        __syncthreads();
        const int64_t base = tile * GT;
        for (int k = threadIdx.x; k < GT; k += blockDim.x) {
            const int64_t row = base + k;
            if (row >= n) break;
            if (!valid_bit(col.d_validity, col.validity_bit_offset, row)) continue;
            ++rows;
            ltab_insert_bytes(t, col, g_hash_bytes(g_bytes_at(col, row)), row, 1u);
        }
        __syncthreads();
        flush_groups<true, true>(t, out, b1 ? shift : 63, b1 ? nb : 1, 0, s_hist, s_base, &s_ovf);
    }
    rows = wave_sum_u64(rows);
    if (lane_id() == 0 && rows) atomicAdd((unsigned long long *)&stats[0], (unsigned long long)rows);
    if (threadIdx.x == 0 && s_ovf) atomicOr((unsigned long long *)&stats[2], 1ull);
}

// L1 bucket records -> L2 buckets.  Work item = (L1 bucket, chunk of GT records).
template <bool BYTES, bool COUNTS>
__global__ void __launch_bounds__(GB) part_recs_kernel(Buckets in, int nb1, Buckets out, int b1, int b2,
                                                       sdp_bytes_column bc, int64_t chunks_per_bucket,
                                                       uint64_t *stats) {
    __shared__ uint64_t s_key[GL];
    __shared__ uint64_t s_hash[BYTES ? GL : 1];
    __shared__ uint32_t s_cnt[GL];
    __shared__ uint32_t s_hist[GMAXB], s_base[GMAXB];
    __shared__ uint32_t s_ovf;
    LTab<BYTES> t{s_key, BYTES ? s_hash : nullptr, s_cnt};
    if (threadIdx.x == 0) s_ovf = 0;
    const int nb2 = 1 << b2;
    const int shift = 64 - b1 - b2;
    const int64_t items = (int64_t)nb1 * chunks_per_bucket;
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const int64_t p = it % nb1, ch = it / nb1;
        const int64_t fill = min((int64_t)in.fill[p], in.cap);
        const int64_t r0 = ch * GT;
        if (r0 >= fill) continue;                       // uniform per block
        ltab_clear(t);
        __syncthreads();
        const int64_t r1 = min(fill, r0 + GT);
        for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
            const int64_t o = p * in.cap + r;
            const uint32_t c = COUNTS ? (uint32_t)in.cnt[o] : 1u;
            if constexpr (BYTES) ltab_insert_bytes(t, bc, in.key[o], (int64_t)in.row[o], c);
            else ltab_insert_u64(t, in.key[o], mix64(in.key[o]), c);
        }
        __syncthreads();
        flush_groups<BYTES, COUNTS>(t, out, shift, nb2, p * nb2, s_hist, s_base, &s_ovf);
    }
    if (threadIdx.x == 0 && s_ovf) atomicOr((unsigned long long *)&stats[2], 1ull);
}

// One block per bucket: distinct groups in LDS; groups written back in place
// (bucket region [0, groups)); per-bucket group count to ngroups[b]; the group
// total accumulated into stats[4 + (b & 63)] (64 spread counters).
template <bool BYTES, bool COUNTS>
__global__ void __launch_bounds__(GB) dedup_kernel(Buckets in, int64_t nbuckets, sdp_bytes_column bc,
                                                   uint32_t *ngroups, uint64_t *stats) {
    __shared__ uint64_t s_key[GL];
    __shared__ uint64_t s_hash[BYTES ? GL : 1];
    __shared__ uint32_t s_cnt[GL];
    __shared__ uint32_t s_n, s_full;
    LTab<BYTES> t{s_key, BYTES ? s_hash : nullptr, s_cnt};
    for (int64_t b = blockIdx.x; b < nbuckets; b += gridDim.x) {
        const int64_t fill = min((int64_t)in.fill[b], in.cap);
        if (fill == 0) {
            if (threadIdx.x == 0) ngroups[b] = 0;
            continue;
        }
        ltab_clear(t);
        if (threadIdx.x == 0) { s_n = 0; s_full = 0; }
        __syncthreads();
        bool ok = true;
        for (int64_t r = threadIdx.x; r < fill; r += blockDim.x) {
            const int64_t o = b * in.cap + r;
            const uint32_t c = COUNTS ? (uint32_t)in.cnt[o] : 1u;
            if constexpr (BYTES) ok &= ltab_insert_bytes(t, bc, in.key[o], (int64_t)in.row[o], c);
            else ok &= ltab_insert_u64(t, in.key[o], mix64(in.key[o]), c);
        }
        if (!ok) s_full = 1;
        __syncthreads();
        // write the groups back to the bucket's region (every read is done)
        for (int i = threadIdx.x; i < GL; i += blockDim.x) {
            const uint64_t k = t.tkey[i];
            const bool occ = BYTES ? (k != 0) : (k != EMPTY64);
            if (occ) {
                const uint32_t pos = atomicAdd(&s_n, 1u);
                const int64_t o = b * in.cap + pos;
                in.key[o] = k;                 // bytes: (tag << 40 | row + 1)
                if (COUNTS) in.cnt[o] = t.tcnt[i];
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            ngroups[b] = s_n;
            atomicAdd((unsigned long long *)&stats[4 + (b & 63)], (unsigned long long)s_n);
            if (s_full) atomicOr((unsigned long long *)&stats[3], 1ull);
        }
        __syncthreads();
    }
}

static int gridcap(int64_t items, int maxg) {
    if (items < 1) return 1;
    return (int)(items < maxg ? items : maxg);
}

}  // namespace sdp

using namespace sdp;

extern "C" {

static Buckets to_b(const sdp_buckets *b) {
    Buckets r;
    r.key = b->d_key;
    r.row = b->d_row;
    r.cnt = b->d_cnt;
    r.fill = b->d_fill;
    r.cap = b->capacity;
    return r;
}

int sdp_group_part_rows_u64(const sdp_column *col, int32_t b1, int32_t with_counts, const sdp_buckets *out,
                            uint64_t *d_stats, void *stream) {
    if (col == nullptr || out == nullptr || b1 < 0 || b1 > 10) return set_error(SDP_EINVAL, "part_rows_u64: args");
    const int grid = gridcap((col->length + GT - 1) / GT, 2048);
    if (with_counts)
        hipLaunchKernelGGL(part_rows_u64_kernel<true>, dim3(grid), dim3(GB), 0, (hipStream_t)stream, *col, to_b(out),
                           b1, d_stats);
    else
        hipLaunchKernelGGL(part_rows_u64_kernel<false>, dim3(grid), dim3(GB), 0, (hipStream_t)stream, *col,
                           to_b(out), b1, d_stats);
    return check_launch("part_rows_u64_kernel");
}

int sdp_group_part_rows_bytes(const sdp_bytes_column *col, int32_t b1, const sdp_buckets *out, uint64_t *d_stats,
                              void *stream) {
    if (col == nullptr || out == nullptr || b1 < 0 || b1 > 10) return set_error(SDP_EINVAL, "part_rows_bytes: args");
    if (col->length >= (int64_t)RMASK) return set_error(SDP_EINVAL, "part_rows_bytes: more than 2^40 rows");
    const int grid = gridcap((col->length + GT - 1) / GT, 2048);
    hipLaunchKernelGGL(part_rows_bytes_kernel, dim3(grid), dim3(GB), 0, (hipStream_t)stream, *col, to_b(out), b1,
                       d_stats);
    return check_launch("part_rows_bytes_kernel");
}

int sdp_group_part_recs(const sdp_buckets *in, int32_t nb1, const sdp_buckets *out, int32_t b1, int32_t b2,
                        const sdp_bytes_column *bytes_col, int32_t with_counts, uint64_t *d_stats, void *stream) {
    if (in == nullptr || out == nullptr || b2 < 1 || b2 > 10 || b1 + b2 > 40)
        return set_error(SDP_EINVAL, "part_recs: args");
    const int64_t chunks = (in->capacity + GT - 1) / GT;
    const int grid = gridcap((int64_t)nb1 * chunks, 65535 * 8);
    sdp_bytes_column bc;
    memset(&bc, 0, sizeof(bc));
    hipStream_t s = (hipStream_t)stream;
    if (bytes_col) {
        bc = *bytes_col;
        hipLaunchKernelGGL((part_recs_kernel<true, true>), dim3(grid), dim3(GB), 0, s, to_b(in), nb1, to_b(out), b1, b2,
                           bc, chunks, d_stats);
    } else if (with_counts) {
        hipLaunchKernelGGL((part_recs_kernel<false, true>), dim3(grid), dim3(GB), 0, s, to_b(in), nb1, to_b(out), b1,
                           b2, bc, chunks, d_stats);
    } else {
        hipLaunchKernelGGL((part_recs_kernel<false, false>), dim3(grid), dim3(GB), 0, s, to_b(in), nb1, to_b(out), b1,
                           b2, bc, chunks, d_stats);
    }
    return check_launch("part_recs_kernel");
}

int sdp_group_dedup(const sdp_buckets *in, int64_t nbuckets, const sdp_bytes_column *bytes_col, int32_t with_counts,
                    uint32_t *d_ngroups, uint64_t *d_stats, void *stream) {
    if (in == nullptr || nbuckets < 1) return set_error(SDP_EINVAL, "dedup: args");
    const int grid = gridcap(nbuckets, 65535 * 8);
    sdp_bytes_column bc;
    memset(&bc, 0, sizeof(bc));
    hipStream_t s = (hipStream_t)stream;
    if (bytes_col) {
        bc = *bytes_col;
        hipLaunchKernelGGL((dedup_kernel<true, true>), dim3(grid), dim3(GB), 0, s, to_b(in), nbuckets, bc, d_ngroups,
                           d_stats);
    } else if (with_counts) {
        hipLaunchKernelGGL((dedup_kernel<false, true>), dim3(grid), dim3(GB), 0, s, to_b(in), nbuckets, bc, d_ngroups,
                           d_stats);
    } else {
        hipLaunchKernelGGL((dedup_kernel<false, false>), dim3(grid), dim3(GB), 0, s, to_b(in), nbuckets, bc,
                           d_ngroups, d_stats);
    }
    return check_launch("dedup_kernel");
}

}  // extern "C"
