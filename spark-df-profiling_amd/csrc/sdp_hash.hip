// sdp_hash.hip -- exact distinct counts and value counts on gfx950.
//
// Replaces `countDistinct(col)` (describe.py:143) for every column and the
// `groupBy(col).agg(count(col)).orderBy(count desc)` + top-50 / others jobs of
// describe_categorical_1d (describe.py:250-271).
//
// Tables are open-addressing, linear probing, power-of-two capacity in HBM.
// Each block first de-duplicates a tile of rows in an LDS table (so hot keys of
// skewed columns cost one global atomic per tile, not per row), then flushes the
// tile's groups into the global table with 64-bit CAS.
//   u64 tables:   slot = the key itself, EMPTY = UINT64_MAX (the one key equal to
//                 EMPTY is counted on the side).
//   byte tables:  slot = (24-bit hash tag << 40) | (row + 1), EMPTY = 0; equal
//                 tags are confirmed by comparing the bytes, so counts are exact.
#include "sdp_common.h"

namespace sdp {

constexpr int H_BLOCK = 256;
constexpr int H_TILE = 2048;              // rows per block per LDS round
constexpr int H_LSLOTS = 4096;            // LDS table slots (load <= 0.5)
constexpr uint64_t ROW_MASK = (1ull << 40) - 1ull;

// ---- element -> key ---------------------------------------------------------
__device__ __forceinline__ bool fetch_key(const sdp_column &c, int64_t i, uint64_t &key) {
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

// ---- byte strings -------------------------------------------------------------
struct BytesRef {
    const uint8_t *p;
    int64_t len;
};

__device__ __forceinline__ BytesRef bytes_at(const sdp_bytes_column &c, int64_t row) {
    BytesRef r;
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

// 8 bytes starting at p (any alignment), zero beyond `avail` bytes.
__device__ __forceinline__ uint64_t load8(const uint8_t *p, int64_t avail) {
    const uint32_t a = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *w = (const uint32_t *)(p - a);   // pointer arithmetic keeps it a global load
    const int sh = (int)(a & 3) * 8;
    const uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    uint64_t v = lo >> sh;
    if (sh) v |= (uint64_t)w[2] << (64 - sh);
    if (avail < 8) v = avail <= 0 ? 0 : (v & ((1ull << (8 * avail)) - 1ull));
    return v;
}

__device__ __forceinline__ uint64_t hash_bytes(BytesRef s) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)s.len * 0xFF51AFD7ED558CCDull);
    int64_t i = 0;
    for (; i + 8 <= s.len; i += 8) h = mix64(h ^ load8(s.p + i, 8)) + 0x632BE59BD9B4E019ull;
    if (i < s.len) h = mix64(h ^ load8(s.p + i, s.len - i) ^ 0xA0761D6478BD642Full);
    return mix64(h);
}

__device__ __forceinline__ bool bytes_equal(BytesRef a, BytesRef b) {
    if (a.len != b.len) return false;
    for (int64_t i = 0; i < a.len; i += 8)
        if (load8(a.p + i, a.len - i) != load8(b.p + i, b.len - i)) return false;
    return true;
}

// big-endian (memcmp-order) 8-byte prefix at `off`, zero padded
__device__ __forceinline__ uint64_t be_prefix(BytesRef s, int64_t off) {
    const uint64_t v = load8(s.p + off, s.len - off);
    return __builtin_bswap64(v);
}

// -1, 0, 1 in unsigned bytewise order, shorter prefix first (Python str/bytes order)
__device__ __forceinline__ int bytes_cmp(BytesRef a, BytesRef b) {
    const int64_t n = a.len < b.len ? a.len : b.len;
    for (int64_t i = 0; i < n; i += 8) {
        const int64_t k = n - i < 8 ? n - i : 8;
        const uint64_t x = __builtin_bswap64(load8(a.p + i, k));
        const uint64_t y = __builtin_bswap64(load8(b.p + i, k));
        if (x != y) return x < y ? -1 : 1;
    }
    return a.len < b.len ? -1 : (a.len > b.len ? 1 : 0);
}

// ---- global insert ------------------------------------------------------------
__device__ __forceinline__ uint32_t insert_u64(uint64_t *slots, uint64_t *counts, uint64_t mask,
                                               uint64_t key, uint64_t c) {
    uint64_t pos = mix64(key) & mask;
    while (true) {
        uint64_t cur = slots[pos];
        if (cur == EMPTY64) {
            const uint64_t old = atomicCAS((unsigned long long *)&slots[pos], (unsigned long long)EMPTY64,
                                           (unsigned long long)key);
            if (old == EMPTY64) {
                if (counts) atomicAdd((unsigned long long *)&counts[pos], (unsigned long long)c);
                return 1;
            }
            cur = old;
        }
        if (cur == key) {
            if (counts) atomicAdd((unsigned long long *)&counts[pos], (unsigned long long)c);
            return 0;
        }
        pos = (pos + 1) & mask;
    }
}

__device__ __forceinline__ uint32_t insert_bytes(const sdp_bytes_column &col, uint64_t *slots, uint64_t *counts,
                                                 uint64_t mask, uint64_t h, int64_t row, uint64_t c) {
    const uint64_t tag = h >> 40;
    const uint64_t mine = (tag << 40) | (uint64_t)(row + 1);
    const BytesRef me = bytes_at(col, row);
    uint64_t pos = h & mask;
    while (true) {
        uint64_t cur = slots[pos];
        if (cur == 0) {
            const uint64_t old = atomicCAS((unsigned long long *)&slots[pos], 0ull, (unsigned long long)mine);
            if (old == 0) {
                atomicAdd((unsigned long long *)&counts[pos], (unsigned long long)c);
                return 1;
            }
            cur = old;
        }
        if ((cur >> 40) == tag && bytes_equal(me, bytes_at(col, (int64_t)(cur & ROW_MASK) - 1))) {
            atomicAdd((unsigned long long *)&counts[pos], (unsigned long long)c);
            return 0;
        }
        pos = (pos + 1) & mask;
    }
}

// ---- kernels --------------------------------------------------------------------
__global__ void table_clear_kernel(uint64_t *slots, uint64_t *counts, int64_t cap, uint64_t empty) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
        slots[i] = empty;
        if (counts) counts[i] = 0;
    }
}

__global__ void __launch_bounds__(H_BLOCK) hash_u64_kernel(sdp_column col, const uint64_t *row_counts,
                                                           uint64_t *slots, uint64_t *counts,
                                                           uint64_t mask, uint64_t *stats) {
    __shared__ uint64_t l_key[H_LSLOTS];
    __shared__ uint64_t l_cnt[H_LSLOTS];
    __shared__ uint64_t s_red[H_BLOCK / WAVE][3];
    const int64_t n = col.length;
    const int64_t ntiles = (n + H_TILE - 1) / H_TILE;
    uint64_t n_new = 0, n_rows = 0, n_max = 0;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (int i = threadIdx.x; i < H_LSLOTS; i += H_BLOCK) { l_key[i] = EMPTY64; l_cnt[i] = 0; }
        __syncthreads();
        const int64_t base = tile * H_TILE;
        for (int k = threadIdx.x; k < H_TILE; k += H_BLOCK) {
            const int64_t i = base + k;
            if (i >= n) break;
            uint64_t key;
            if (!fetch_key(col, i, key)) continue;
            const uint64_t rc = row_counts ? row_counts[i] : 1ull;
            n_rows += rc;
            if (key == EMPTY64) { n_max += rc; continue; }
            uint32_t pos = (uint32_t)(mix64(key) & (H_LSLOTS - 1));
            while (true) {
                const uint64_t old = atomicCAS((unsigned long long *)&l_key[pos], (unsigned long long)EMPTY64,
                                               (unsigned long long)key);
                if (old == EMPTY64 || old == key) {
                    atomicAdd((unsigned long long *)&l_cnt[pos], (unsigned long long)rc);
                    break;
                }
                pos = (pos + 1) & (H_LSLOTS - 1);
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < H_LSLOTS; i += H_BLOCK) {
            const uint64_t key = l_key[i];
            if (key != EMPTY64) n_new += insert_u64(slots, counts, mask, key, l_cnt[i]);
        }
        __syncthreads();
    }
    const int wid = threadIdx.x / WAVE;
    const uint64_t a = wave_sum_u64(n_new), b = wave_sum_u64(n_rows), c = wave_sum_u64(n_max);
    if (lane_id() == 0) { s_red[wid][0] = a; s_red[wid][1] = b; s_red[wid][2] = c; }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint64_t t = 0;
        for (int w = 0; w < H_BLOCK / WAVE; ++w) t += s_red[w][threadIdx.x];
        if (t) atomicAdd((unsigned long long *)&stats[threadIdx.x], (unsigned long long)t);
    }
}

__global__ void __launch_bounds__(H_BLOCK) hash_bytes_kernel(sdp_bytes_column col, const uint64_t *row_counts,
                                                             uint64_t *slots, uint64_t *counts, uint64_t mask,
                                                             uint64_t *stats) {
    __shared__ uint64_t l_slot[H_LSLOTS];     // (tag << 40) | (row + 1), 0 = empty
    __shared__ uint64_t l_hash[H_LSLOTS];
    __shared__ uint64_t l_cnt[H_LSLOTS];
    __shared__ uint64_t s_red[H_BLOCK / WAVE][2];
    const int64_t n = col.length;
    const int64_t ntiles = (n + H_TILE - 1) / H_TILE;
    uint64_t n_new = 0, n_rows = 0;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (int i = threadIdx.x; i < H_LSLOTS; i += H_BLOCK) { l_slot[i] = 0; l_cnt[i] = 0; }
        __syncthreads();
        const int64_t base = tile * H_TILE;
        for (int k = threadIdx.x; k < H_TILE; k += H_BLOCK) {
            const int64_t row = base + k;
            if (row >= n) break;
            if (!valid_bit(col.d_validity, col.validity_bit_offset, row)) continue;
            const uint64_t rc = row_counts ? row_counts[row] : 1ull;
            n_rows += rc;
            const BytesRef me = bytes_at(col, row);
            const uint64_t h = hash_bytes(me);
            const uint64_t tag = h >> 40;
            const uint64_t mine = (tag << 40) | (uint64_t)(row + 1);
            uint32_t pos = (uint32_t)(h & (H_LSLOTS - 1));
            while (true) {
                uint64_t cur = l_slot[pos];
                if (cur == 0) {
                    const uint64_t old = atomicCAS((unsigned long long *)&l_slot[pos], 0ull, (unsigned long long)mine);
                    if (old == 0) {
                        l_hash[pos] = h;
                        atomicAdd((unsigned long long *)&l_cnt[pos], (unsigned long long)rc);
                        break;
                    }
                    cur = old;
                }
                if ((cur >> 40) == tag && bytes_equal(me, bytes_at(col, (int64_t)(cur & ROW_MASK) - 1))) {
                    atomicAdd((unsigned long long *)&l_cnt[pos], (unsigned long long)rc);
                    break;
                }
                pos = (pos + 1) & (H_LSLOTS - 1);
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < H_LSLOTS; i += H_BLOCK) {
            const uint64_t s = l_slot[i];
            if (s != 0) n_new += insert_bytes(col, slots, counts, mask, l_hash[i], (int64_t)(s & ROW_MASK) - 1, l_cnt[i]);
        }
        __syncthreads();
    }
    const int wid = threadIdx.x / WAVE;
    const uint64_t a = wave_sum_u64(n_new), b = wave_sum_u64(n_rows);
    if (lane_id() == 0) { s_red[wid][0] = a; s_red[wid][1] = b; }
    __syncthreads();
    if (threadIdx.x < 2) {
        uint64_t t = 0;
        for (int w = 0; w < H_BLOCK / WAVE; ++w) t += s_red[w][threadIdx.x];
        if (t) atomicAdd((unsigned long long *)&stats[threadIdx.x], (unsigned long long)t);
    }
}

// flags: bit0 = byte keys (EMPTY = 0), bit1 = dense group arrays (every slot a group)
__device__ __forceinline__ bool occupied(const uint64_t *slots, int64_t i, int flags) {
    if (flags & 2) return true;
    return (flags & 1) ? (slots[i] != 0) : (slots[i] != EMPTY64);
}

__global__ void count_log2_hist_kernel(const uint64_t *slots, const uint64_t *counts, int64_t cap, int bytes_keys,
                                       uint64_t *hist) {
    __shared__ uint32_t h[64];
    if (threadIdx.x < 64) h[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
        if (occupied(slots, i, bytes_keys)) {
            const uint64_t c = counts[i];
            if (c) atomicAdd(&h[63 - __clzll((long long)c)], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < 64 && h[threadIdx.x])
        atomicAdd((unsigned long long *)&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

__global__ void count_hist_kernel(const uint64_t *slots, const uint64_t *counts, int64_t cap, int bytes_keys,
                                  uint64_t lo, uint64_t step, uint64_t *hist) {
    __shared__ uint32_t h[2048];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
        if (occupied(slots, i, bytes_keys)) {
            const uint64_t c = counts[i];
            if (c >= lo) {
                const uint64_t b = (c - lo) / step;
                if (b < 2048) atomicAdd(&h[b], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += blockDim.x)
        if (h[i]) atomicAdd((unsigned long long *)&hist[i], (unsigned long long)h[i]);
}

__global__ void table_select_kernel(const uint64_t *slots, const uint64_t *counts, int64_t cap, int bytes_keys,
                                    uint64_t cmin, uint64_t cmax, uint64_t *out, uint64_t *out_n, uint64_t out_cap) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t iters = (cap + stride - 1) / stride;
    for (int64_t it = 0; it < iters; ++it) {
        const int64_t i = it * stride + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        bool keep = false;
        if (i < cap && occupied(slots, i, bytes_keys)) {
            const uint64_t c = counts ? counts[i] : 1ull;   // distinct-only tables carry no counts
            keep = c >= cmin && c <= cmax;
        }
        const uint64_t m = __ballot(keep);
        if (m) {
            const int leader = __ffsll((long long)m) - 1;
            unsigned long long base = 0;
            if (lane_id() == leader) base = atomicAdd((unsigned long long *)out_n, (unsigned long long)__popcll(m));
            base = __shfl(base, leader, WAVE);
            const uint64_t pos = base + lane_rank(m);
            if (keep && pos < out_cap) out[pos] = (uint64_t)i;
        }
    }
}

// (count desc, key asc): true if group a sorts before group b
__device__ __forceinline__ bool group_before(uint64_t ca, uint64_t sa, uint64_t cb, uint64_t sb,
                                             const uint64_t *slots, const sdp_bytes_column *bc) {
    if (ca != cb) return ca > cb;
    if (bc == nullptr) return slots[sa] < slots[sb];
    const int c = bytes_cmp(bytes_at(*bc, (int64_t)(slots[sa] & ROW_MASK) - 1),
                            bytes_at(*bc, (int64_t)(slots[sb] & ROW_MASK) - 1));
    return c < 0;
}

constexpr int GSORT_MAX = 8192;

__global__ void __launch_bounds__(1024) sort_groups_kernel(uint64_t *sel, const uint64_t *n_ptr, const uint64_t *slots,
                                                           const uint64_t *counts, sdp_bytes_column bc, int has_bytes) {
    __shared__ uint64_t s_c[GSORT_MAX];
    __shared__ uint32_t s_s[GSORT_MAX];
    const int n = (int)min((uint64_t)GSORT_MAX, *n_ptr);
    const sdp_bytes_column *bcp = has_bytes ? &bc : nullptr;
    int P = 2;
    while (P < n) P <<= 1;
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
        if (i < n) { s_s[i] = (uint32_t)i; s_c[i] = counts[sel[i]]; }
        else { s_s[i] = 0xFFFFFFFFu; s_c[i] = 0; }
    }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t ia = s_s[i], ib = s_s[ixj];
                    bool a_first;   // padding (0xFFFFFFFF) sorts last
                    if (ia == 0xFFFFFFFFu) a_first = false;
                    else if (ib == 0xFFFFFFFFu) a_first = true;
                    else a_first = group_before(s_c[i], sel[ia], s_c[ixj], sel[ib], slots, bcp);
                    const bool asc = (i & k) == 0;
                    if (a_first != asc) {
                        s_s[i] = ib; s_s[ixj] = ia;
                        const uint64_t t = s_c[i]; s_c[i] = s_c[ixj]; s_c[ixj] = t;
                    }
                }
            }
            __syncthreads();
        }
    }
    // permute sel through s_s (copy out, then write back)
    uint64_t tmp[GSORT_MAX / 1024];
    for (int r = 0; r < GSORT_MAX / 1024; ++r) {
        const int i = threadIdx.x + r * 1024;
        tmp[r] = (i < n) ? sel[s_s[i]] : 0;
    }
    __syncthreads();
    for (int r = 0; r < GSORT_MAX / 1024; ++r) {
        const int i = threadIdx.x + r * 1024;
        if (i < n) sel[i] = tmp[r];
    }
}

__global__ void group_prefix_kernel(const uint64_t *sel, const uint64_t *n_ptr, const uint64_t *slots,
                                    sdp_bytes_column bc, int offset, uint64_t *out) {
    const uint64_t n = *n_ptr;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const BytesRef s = bytes_at(bc, (int64_t)(slots[sel[i]] & ROW_MASK) - 1);
        out[i] = be_prefix(s, offset);
    }
}

// keep entries of `sel` whose parallel key lies in [lo, hi]
__global__ void select_by_value_kernel(const uint64_t *sel, const uint64_t *vals, const uint64_t *n_ptr,
                                       uint64_t lo, uint64_t hi, uint64_t *out, uint64_t *out_vals, uint64_t *out_n) {
    const uint64_t n = *n_ptr;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t iters = (n + stride - 1) / stride;
    for (uint64_t it = 0; it < iters; ++it) {
        const uint64_t i = it * stride + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        bool keep = false;
        uint64_t v = 0;
        if (i < n) { v = vals[i]; keep = v >= lo && v <= hi; }
        const uint64_t m = __ballot(keep);
        if (m) {
            const int leader = __ffsll((long long)m) - 1;
            unsigned long long base = 0;
            if (lane_id() == leader) base = atomicAdd((unsigned long long *)out_n, (unsigned long long)__popcll(m));
            base = __shfl(base, leader, WAVE);
            if (keep) { out[base + lane_rank(m)] = sel[i]; if (out_vals) out_vals[base + lane_rank(m)] = v; }
        }
    }
}

// first k rows surviving na.drop (null; NaN for floats), in row order.  One
// workgroup scans forward chunk by chunk and stops once k rows are found.
__global__ void __launch_bounds__(1024) first_valid_kernel(sdp_column col, int k, int64_t *idx, int64_t *found) {
    __shared__ uint32_t s_cnt[1024 / WAVE];
    __shared__ int64_t s_total;
    if (threadIdx.x == 0) s_total = 0;
    __syncthreads();
    const int64_t n = col.length;
    const int wid = threadIdx.x / WAVE;
    for (int64_t base = 0; base < n; base += 1024) {
        const int64_t i = base + threadIdx.x;
        bool ok = false;
        if (i < n) {
            uint64_t key;
            ok = fetch_key(col, i, key);
            if (ok && (col.dtype == SDP_F32 || col.dtype == SDP_F64)) ok = key != KEY_NAN;
        }
        const uint64_t m = __ballot(ok);
        if (lane_id() == 0) s_cnt[wid] = (uint32_t)__popcll(m);
        __syncthreads();
        int64_t before = s_total;
        for (int w = 0; w < wid; ++w) before += s_cnt[w];
        const int64_t pos = before + lane_rank(m);
        if (ok && pos < k) idx[pos] = i;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t t = s_total;
            for (int w = 0; w < 1024 / WAVE; ++w) t += s_cnt[w];
            s_total = t;
        }
        __syncthreads();
        if (s_total >= k) break;
    }
    if (threadIdx.x == 0) *found = s_total < k ? s_total : k;
}

}  // namespace sdp

using namespace sdp;

static int grid_for(int64_t n, int per_block, int maxg) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    return (int)(g < maxg ? g : maxg);
}

static bool pow2(int64_t c) { return c > 0 && (c & (c - 1)) == 0; }

extern "C" int sdp_table_clear(uint64_t *d_slots, uint64_t *d_counts, int64_t capacity, int32_t bytes_keys,
                               void *stream) {
    if (!pow2(capacity)) return set_error(SDP_EINVAL, "sdp_table_clear: capacity %lld not a power of two",
                                          (long long)capacity);
    hipLaunchKernelGGL(table_clear_kernel, dim3(grid_for(capacity, 256 * 8, 4096)), dim3(256), 0,
                       (hipStream_t)stream, d_slots, d_counts, capacity, bytes_keys ? 0ull : EMPTY64);
    return check_launch("table_clear_kernel");
}

extern "C" int sdp_hash_u64(const sdp_column *col, const uint64_t *d_row_counts, uint64_t *d_slots,
                            uint64_t *d_counts, int64_t capacity, int32_t with_counts, uint64_t *d_stats,
                            void *stream) {
    if (col == nullptr || col->length < 0) return set_error(SDP_EINVAL, "sdp_hash_u64: column");
    if (!pow2(capacity)) return set_error(SDP_EINVAL, "sdp_hash_u64: capacity");
    if (col->dtype < SDP_I8 || col->dtype > SDP_BOOL) return set_error(SDP_EINVAL, "sdp_hash_u64: dtype %d", col->dtype);
    hipLaunchKernelGGL(hash_u64_kernel, dim3(grid_for(col->length, H_TILE, 2048)), dim3(H_BLOCK), 0,
                       (hipStream_t)stream, *col, d_row_counts, d_slots, with_counts ? d_counts : nullptr,
                       (uint64_t)(capacity - 1), d_stats);
    return check_launch("hash_u64_kernel");
}

extern "C" int sdp_hash_bytes(const sdp_bytes_column *col, const uint64_t *d_row_counts, uint64_t *d_slots,
                              uint64_t *d_counts, int64_t capacity, uint64_t *d_stats, void *stream) {
    if (col == nullptr || col->length < 0) return set_error(SDP_EINVAL, "sdp_hash_bytes: column");
    if (col->length >= (int64_t)ROW_MASK) return set_error(SDP_EINVAL, "sdp_hash_bytes: more than 2^40 rows");
    if (!pow2(capacity)) return set_error(SDP_EINVAL, "sdp_hash_bytes: capacity");
    if (col->fixed_width <= 0 && col->offset_width != 4 && col->offset_width != 8)
        return set_error(SDP_EINVAL, "sdp_hash_bytes: offset_width %d", col->offset_width);
    hipLaunchKernelGGL(hash_bytes_kernel, dim3(grid_for(col->length, H_TILE, 2048)), dim3(H_BLOCK), 0,
                       (hipStream_t)stream, *col, d_row_counts, d_slots, d_counts, (uint64_t)(capacity - 1),
                       d_stats);
    return check_launch("hash_bytes_kernel");
}

extern "C" int sdp_table_count_log2_hist(const uint64_t *d_slots, const uint64_t *d_counts, int64_t capacity,
                                         int32_t bytes_keys, uint64_t *d_hist, void *stream) {
    if (d_slots == nullptr || d_counts == nullptr || d_hist == nullptr)
        return set_error(SDP_EINVAL, "sdp_table_count_log2_hist: null pointer");
    hipLaunchKernelGGL(count_log2_hist_kernel, dim3(grid_for(capacity, 256 * 16, 2048)), dim3(256), 0,
                       (hipStream_t)stream, d_slots, d_counts, capacity, bytes_keys, d_hist);
    return check_launch("count_log2_hist_kernel");
}

extern "C" int sdp_table_count_hist(const uint64_t *d_slots, const uint64_t *d_counts, int64_t capacity,
                                    int32_t bytes_keys, uint64_t lo, uint64_t step, uint64_t *d_hist, void *stream) {
    if (step == 0) return set_error(SDP_EINVAL, "sdp_table_count_hist: step 0");
    if (d_slots == nullptr || d_counts == nullptr || d_hist == nullptr)
        return set_error(SDP_EINVAL, "sdp_table_count_hist: null pointer");
    hipLaunchKernelGGL(count_hist_kernel, dim3(grid_for(capacity, 256 * 16, 2048)), dim3(256), 0,
                       (hipStream_t)stream, d_slots, d_counts, capacity, bytes_keys, lo, step, d_hist);
    return check_launch("count_hist_kernel");
}

extern "C" int sdp_table_select(const uint64_t *d_slots, const uint64_t *d_counts, int64_t capacity,
                                int32_t bytes_keys, uint64_t min_count, uint64_t max_count, uint64_t *d_out,
                                uint64_t *d_out_n, uint64_t out_capacity, void *stream) {
    if (d_slots == nullptr || d_out == nullptr || d_out_n == nullptr)
        return set_error(SDP_EINVAL, "sdp_table_select: null pointer");
    hipLaunchKernelGGL(table_select_kernel, dim3(grid_for(capacity, 256 * 16, 2048)), dim3(256), 0,
                       (hipStream_t)stream, d_slots, d_counts, capacity, bytes_keys, min_count, max_count, d_out,
                       d_out_n, out_capacity);
    return check_launch("table_select_kernel");
}

extern "C" int sdp_sort_groups(uint64_t *d_sel, const uint64_t *d_n, const uint64_t *d_slots,
                               const uint64_t *d_counts, const sdp_bytes_column *bytes_col, void *stream) {
    if (d_sel == nullptr || d_n == nullptr || d_slots == nullptr || d_counts == nullptr)
        return set_error(SDP_EINVAL, "sdp_sort_groups: null pointer");
    sdp_bytes_column bc;
    memset(&bc, 0, sizeof(bc));
    if (bytes_col) bc = *bytes_col;
    hipLaunchKernelGGL(sort_groups_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_sel, d_n, d_slots, d_counts,
                       bc, bytes_col ? 1 : 0);
    return check_launch("sort_groups_kernel");
}

extern "C" int sdp_group_prefix(const uint64_t *d_sel, const uint64_t *d_n, const uint64_t *d_slots,
                                const sdp_bytes_column *col, int32_t offset, uint64_t *d_out, void *stream) {
    if (col == nullptr || offset < 0) return set_error(SDP_EINVAL, "sdp_group_prefix: args");
    hipLaunchKernelGGL(group_prefix_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, d_sel, d_n, d_slots, *col,
                       offset, d_out);
    return check_launch("group_prefix_kernel");
}

extern "C" int sdp_select_by_value(const uint64_t *d_sel, const uint64_t *d_vals, const uint64_t *d_n, uint64_t lo,
                                   uint64_t hi, uint64_t *d_out, uint64_t *d_out_vals, uint64_t *d_out_n,
                                   void *stream) {
    hipLaunchKernelGGL(select_by_value_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, d_sel, d_vals, d_n, lo,
                       hi, d_out, d_out_vals, d_out_n);
    return check_launch("select_by_value_kernel");
}

extern "C" int sdp_first_valid(const sdp_column *col, int32_t k, int64_t *d_idx, int64_t *d_found, void *stream) {
    if (col == nullptr || k < 0) return set_error(SDP_EINVAL, "sdp_first_valid: args");
    hipLaunchKernelGGL(first_valid_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, *col, k, d_idx, d_found);
    return check_launch("first_valid_kernel");
}

// Packs the key bytes of n groups (bytes [starts[i], starts[i] + lens[i]) of
// `data`) back to back at out + offs[i]: the payload of the sharded string
// exchange (distributed.exchange_bytes_groups).  One thread per group; keys are
// short, so a byte loop beats any per-byte index array (which would cost 8 B of
// index per key byte).
__global__ void gather_bytes_kernel(const uint8_t *data, const int64_t *starts, const int64_t *lens,
                                    const int64_t *offs, int64_t n, uint8_t *out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t *src = data + starts[i];
        uint8_t *dst = out + offs[i];
        const int64_t len = lens[i];
        for (int64_t b = 0; b < len; ++b) dst[b] = src[b];
    }
}

// validity of byte columns for first_valid: expose the count of valid rows too
__global__ void count_valid_kernel(const uint8_t *bm, int64_t off, int64_t n, uint64_t *out) {
    uint64_t c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        c += valid_bit(bm, off, i);
    c = wave_sum_u64(c);
    if (lane_id() == 0 && c) atomicAdd((unsigned long long *)out, (unsigned long long)c);
}

extern "C" int sdp_count_valid(const uint8_t *d_validity, int64_t bit_offset, int64_t length, uint64_t *d_out,
                               void *stream) {
    hipLaunchKernelGGL(count_valid_kernel, dim3(grid_for(length, 256 * 32, 2048)), dim3(256), 0, (hipStream_t)stream,
                       d_validity, bit_offset, length, d_out);
    return check_launch("count_valid_kernel");
}

extern "C" int sdp_gather_bytes(const uint8_t *d_data, const int64_t *d_starts, const int64_t *d_lens,
                                const int64_t *d_offs, int64_t n, uint8_t *d_out, void *stream) {
    if (n < 0) return set_error(SDP_EINVAL, "sdp_gather_bytes: n %lld", (long long)n);
    if (n == 0) return 0;
    int64_t grid = (n + 255) / 256;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(gather_bytes_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, d_data, d_starts,
                       d_lens, d_offs, n, d_out);
    return check_launch("gather_bytes_kernel");
}

// ---- owner order of the sharded exchange (distributed.py) --------------------
// Every rank sends each of its groups to the key's owner rank.  The groups go
// owner-major and, within an owner, in their table order (a stable counting
// sort by owner): per 2048-group chunk an owner histogram, one exclusive scan
// of the owner-major [owner][chunk] counts, then a scatter that ranks each
// group among the same-owner groups before it in its chunk.  Byte groups also
// get their key's (start, length) in the column, the (length, count) pair the
// owner re-aggregates with, and (a second scan) the byte offset of the key in
// the owner-major payload that sdp_gather_bytes packs.  Replaces a torch sort +
// searchsorted + prefix sum + gathers (round 5's exchange).
constexpr int OWN_T = 256;
constexpr int OWN_W = OWN_T / WAVE;
constexpr int OWN_PER = 8;
constexpr int OWN_CH = OWN_T * OWN_PER;       // groups per chunk
constexpr int OWN_MAX_WORLD = 2048;      // scatter LDS 5 x 4 B per owner: <= 40 KB

struct OwnerSrc {
    const uint64_t *keys;       // u64 keys, or byte-table slots (24-bit tag << 40 | row + 1)
    const uint64_t *sel;        // group i is entry sel[i] (NULL: entry i)
    const int64_t *counts;      // per entry, or NULL
    sdp_bytes_column col;       // byte groups: the column the rows index
    int64_t n;
    int32_t world;
    int32_t is_bytes;
};

struct OwnerOut {
    uint64_t *keys;             // fixed keys
    int64_t *counts;            // fixed keys' counts (NULL: none)
    int64_t *starts, *lens;     // byte groups
    int64_t *meta;              // byte groups: (length, count) pairs
    uint32_t *lens32;           // byte groups: lengths for the offsets scan
};

__device__ __forceinline__ uint32_t owner_of(const OwnerSrc &s, uint64_t k) {
    // distributed._owner_u64 (fixed keys: multiplicative hash) / the byte slot's tag
    const uint64_t h = s.is_bytes ? k : k * 0x9E3779B97F4A7C15ull;
    return (uint32_t)((h >> 40) & 0xFFFFFFull) % (uint32_t)s.world;
}

// lanes of this wave with the same owner: rank among the lower such lanes and
// their number (one round per distinct owner in the wave)
__device__ __forceinline__ void wave_owner_match(uint32_t o, bool act, uint32_t &rank, uint32_t &size) {
    uint64_t rem = __ballot(act);
    rank = 0;
    size = 0;
    while (rem) {
        const int l = __ffsll((unsigned long long)rem) - 1;
        const uint32_t lo = (uint32_t)__shfl((int)o, l, WAVE);
        const uint64_t m = __ballot(act && o == lo);
        if (act && o == lo) {
            rank = (uint32_t)lane_rank(m);
            size = (uint32_t)__popcll(m);
        }
        rem &= ~m;
    }
}

__global__ void __launch_bounds__(OWN_T) owner_hist_kernel(OwnerSrc s, int64_t nchunks, uint32_t *hist) {
    extern __shared__ uint32_t s_own[];       // [world]
    for (int o = threadIdx.x; o < s.world; o += OWN_T) s_own[o] = 0;
    __syncthreads();
    const int64_t c = blockIdx.x;
    for (int k = 0; k < OWN_PER; ++k) {
        const int64_t i = c * OWN_CH + (int64_t)k * OWN_T + threadIdx.x;
        const bool act = i < s.n;
        uint32_t o = 0;
        if (act) o = owner_of(s, s.keys[s.sel ? (int64_t)s.sel[i] : i]);
        uint32_t rank, size;
        wave_owner_match(o, act, rank, size);
        if (act && rank == 0) atomicAdd(&s_own[o], size);
    }
    __syncthreads();
    for (int o = threadIdx.x; o < s.world; o += OWN_T) hist[(int64_t)o * nchunks + c] = s_own[o];
}

__global__ void __launch_bounds__(OWN_T) owner_scatter_kernel(OwnerSrc s, int64_t nchunks, const uint64_t *hoffs,
                                                              OwnerOut out) {
    extern __shared__ uint32_t s_own[];       // run[world] | per-wave counts [OWN_W][world]
    uint32_t *s_run = s_own, *s_wc = s_own + s.world;
    for (int o = threadIdx.x; o < s.world * (1 + OWN_W); o += OWN_T) s_own[o] = 0;
    __syncthreads();
    const int w = threadIdx.x / WAVE;
    const int64_t c = blockIdx.x;
    for (int k = 0; k < OWN_PER; ++k) {
        const int64_t i = c * OWN_CH + (int64_t)k * OWN_T + threadIdx.x;
        const bool act = i < s.n;
        int64_t e = 0;
        uint64_t key = 0;
        uint32_t o = 0;
        if (act) {
            e = s.sel ? (int64_t)s.sel[i] : i;
            key = s.keys[e];
            o = owner_of(s, key);
        }
        uint32_t rank, size;
        wave_owner_match(o, act, rank, size);
        if (act && rank == 0) s_wc[w * s.world + o] = size;
        lds_barrier();
        uint64_t p = 0;
        if (act) {
            uint32_t before = s_run[o];
            for (int v = 0; v < w; ++v) before += s_wc[v * s.world + o];
            p = hoffs[(int64_t)o * nchunks + c] + before + rank;
        }
        lds_barrier();
        for (int t = threadIdx.x; t < s.world; t += OWN_T) {
            uint32_t a = 0;
            for (int v = 0; v < OWN_W; ++v) {
                a += s_wc[v * s.world + t];
                s_wc[v * s.world + t] = 0;
            }
            s_run[t] += a;
        }
        lds_barrier();
        if (!act) continue;
        const int64_t cnt = s.counts ? s.counts[e] : 0;
        if (!s.is_bytes) {
            out.keys[p] = key;
            if (out.counts) out.counts[p] = cnt;
            continue;
        }
        const int64_t row = (int64_t)(key & ROW_MASK) - 1;
        int64_t st, len;
        if (s.col.fixed_width > 0) {
            st = row * s.col.fixed_width;
            len = s.col.fixed_width;
        } else if (s.col.offset_width == 4) {
            const int32_t *off = (const int32_t *)s.col.d_offsets;
            st = off[row];
            len = (int64_t)off[row + 1] - st;
        } else {
            const int64_t *off = (const int64_t *)s.col.d_offsets;
            st = off[row];
            len = off[row + 1] - st;
        }
        out.starts[p] = st;
        out.lens[p] = len;
        out.meta[2 * p] = len;
        out.meta[2 * p + 1] = cnt;
        out.lens32[p] = (uint32_t)len;
    }
}

__global__ void __launch_bounds__(OWN_T) owner_totals_kernel(const uint64_t *hoffs, int64_t nchunks, int world,
                                                             const uint64_t *boffs, int64_t *per) {
    for (int o = threadIdx.x; o < world; o += OWN_T) {
        const uint64_t g0 = hoffs[(int64_t)o * nchunks], g1 = hoffs[(int64_t)(o + 1) * nchunks];
        per[o] = (int64_t)(g1 - g0);
        per[world + o] = boffs ? (int64_t)(boffs[g1] - boffs[g0]) : 0;
    }
}

static int64_t align16(int64_t b) { return (b + 15) & ~(int64_t)15; }

extern "C" int64_t sdp_owner_order_workspace_bytes(int64_t n, int32_t world) {
    if (n < 0 || world < 1) return 0;
    const int64_t nchunks = (n + OWN_CH - 1) / OWN_CH;
    const int64_t nh = (int64_t)world * nchunks;
    int64_t scan = sdp_scan_workspace_bytes(nh > 0 ? nh : 1);
    const int64_t scan_n = sdp_scan_workspace_bytes(n > 0 ? n : 1);
    if (scan_n > scan) scan = scan_n;
    return align16(nh * 4) + align16((nh + 1) * 8) + align16(n * 4) + align16(scan);
}

extern "C" int sdp_owner_order(const uint64_t *d_keys, const uint64_t *d_sel, const int64_t *d_counts, int64_t n,
                               int32_t world, const sdp_bytes_column *bcol, uint64_t *d_out_keys,
                               int64_t *d_out_counts, int64_t *d_starts, int64_t *d_lens, int64_t *d_meta,
                               uint64_t *d_offs, int64_t *d_per, void *d_work, int64_t work_bytes, void *stream) {
    if (n < 0 || world < 1 || world > OWN_MAX_WORLD || d_per == nullptr)
        return set_error(SDP_EINVAL, "sdp_owner_order: n %lld world %d", (long long)n, (int)world);
    const bool isb = bcol != nullptr;
    if (isb ? (d_starts == nullptr || d_lens == nullptr || d_meta == nullptr || d_offs == nullptr ||
               (bcol->fixed_width <= 0 && (bcol->d_offsets == nullptr ||
                                           (bcol->offset_width != 4 && bcol->offset_width != 8))))
            : d_out_keys == nullptr)
        return set_error(SDP_EINVAL, "sdp_owner_order: outputs");
    if (d_out_counts != nullptr && d_counts == nullptr)
        return set_error(SDP_EINVAL, "sdp_owner_order: counts out without counts in");
    if (isb && d_counts == nullptr) return set_error(SDP_EINVAL, "sdp_owner_order: byte groups need counts");
    if (work_bytes < sdp_owner_order_workspace_bytes(n, world))
        return set_error(SDP_ECAP, "sdp_owner_order: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        if (hipMemsetAsync(d_per, 0, (size_t)world * 2 * sizeof(int64_t), s) != hipSuccess ||
            (isb && hipMemsetAsync(d_offs, 0, sizeof(uint64_t), s) != hipSuccess))
            return set_error(SDP_EHIP, "sdp_owner_order: memset");
        return 0;
    }
    const int64_t nchunks = (n + OWN_CH - 1) / OWN_CH;
    if (nchunks > 0x7FFFFFFF) return set_error(SDP_EINVAL, "sdp_owner_order: too many groups");
    const int64_t nh = (int64_t)world * nchunks;
    uint8_t *wp = (uint8_t *)d_work;
    uint32_t *hist = (uint32_t *)wp;
    wp += align16(nh * 4);
    uint64_t *hoffs = (uint64_t *)wp;
    wp += align16((nh + 1) * 8);
    uint32_t *lens32 = (uint32_t *)wp;
    wp += align16(n * 4);
    void *scan = wp;
    const int64_t scan_bytes = work_bytes - (wp - (uint8_t *)d_work);
    OwnerSrc src;
    src.keys = d_keys;
    src.sel = d_sel;
    src.counts = d_counts;
    src.col = isb ? *bcol : sdp_bytes_column{};
    src.n = n;
    src.world = world;
    src.is_bytes = isb ? 1 : 0;
    OwnerOut out{d_out_keys, d_out_counts, d_starts, d_lens, d_meta, lens32};
    hipLaunchKernelGGL(owner_hist_kernel, dim3((unsigned)nchunks), dim3(OWN_T), (size_t)world * 4, s, src, nchunks,
                       hist);
    int rc = check_launch("owner_hist_kernel");
    if (rc) return rc;
    if ((rc = sdp_scan_u32(hist, nh, hoffs, scan, scan_bytes, stream))) return rc;
    hipLaunchKernelGGL(owner_scatter_kernel, dim3((unsigned)nchunks), dim3(OWN_T), (size_t)world * 4 * (1 + OWN_W),
                       s, src, nchunks, (const uint64_t *)hoffs, out);
    if ((rc = check_launch("owner_scatter_kernel"))) return rc;
    if (isb && (rc = sdp_scan_u32(lens32, n, d_offs, scan, scan_bytes, stream))) return rc;
    hipLaunchKernelGGL(owner_totals_kernel, dim3(1), dim3(OWN_T), 0, s, (const uint64_t *)hoffs, nchunks, (int)world,
                       isb ? (const uint64_t *)d_offs : nullptr, d_per);
    return check_launch("owner_totals_kernel");
}
