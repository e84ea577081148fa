// sdp_part.hip -- exact distinct counts and value counts by two-level hash
// partitioning with exact offsets (gfx950).
//
// Replaces countDistinct (describe.py:143) and the groupBy(c).count() of
// describe_categorical_1d (describe.py:251) for columns of any cardinality.
//
// Every valid row becomes one record.  Fixed-width keys: the record is
// h = mix64(key) (a bijection, so distinct h == distinct keys and the key is
// recovered by inv_mix64).  Byte keys: (k0, k1, meta) with k0/k1 the first 16
// bytes (zero padded) and meta = len << 40 | row + 1; strings longer than 16
// bytes carry their 64-bit hash in k0 and are compared byte for byte against
// the column.  Pipeline (each step a kernel, every probe in LDS):
//
//   rows  phase 0  per-block histogram of the top b1 hash bits -> H1[b][block]
//   scan           exclusive scan of H1 (bucket-major) -> exact record offsets
//   rows  phase 1  re-read; per 4096-row tile an LDS counting sort by bucket,
//                  then each bucket's run is written contiguously at its offset
//   recs  phase 0  per L1 chunk histogram of the next b2 bits -> H2
//   scan           -> exact offsets of every (L1 bucket, sub-bucket, chunk)
//   recs  phase 1  LDS counting sort + contiguous runs, as above
//   dedup          one workgroup per final bucket (~2-8 K records) groups its
//                  records in an LDS hash table; distinct counts, or groups +
//                  counts written in place and compacted
//
// Keys seen >= 3 times in a 16 K-row sample ("heavy" keys, at most 256) are
// counted per block in LDS during phase 0 and never become records, so skewed
// columns do not pile up in one bucket.  Offsets come from the scans, so the
// output is packed exactly and nothing can overflow; every stage except the
// LDS atomics inside a tile is deterministic.
#include <type_traits>
#include "sdp_heavy.h"

namespace sdp {

// SDP_DEBUG_BOUNDS builds (tools/debug_bounds.sh, never the shipped library):
// block-layout indices are checked against the record / block capacities of
// the last sdp_part_l2_blocks call, and an index outside them raises a flag
// bit (read by sdp_debug_bounds) and is replaced by 0 instead of faulting
#ifdef SDP_DEBUG_BOUNDS
__device__ unsigned long long dbg_flags, dbg_cap_rec, dbg_cap_blk;
__device__ __forceinline__ int64_t dbg_chk(int64_t i, unsigned long long cap, int code) {
    if ((unsigned long long)i >= cap) {
        atomicOr(&dbg_flags, 1ull << code);
        return 0;
    }
    return i;
}
#define DBG_REC(i, code) dbg_chk((int64_t)(i), dbg_cap_rec, (code))
#define DBG_BLK(i, code) dbg_chk((int64_t)(i), dbg_cap_blk, (code))
#else
#define DBG_REC(i, code) (i)
#define DBG_BLK(i, code) (i)
#endif

constexpr int PT = 256;                 // threads of the small helper kernels
constexpr uint64_t RMASK40 = (1ull << 40) - 1ull;
constexpr uint64_t LEN_MAX = (1ull << 24) - 1ull;

// ---- hashing ------------------------------------------------------------------
__device__ __forceinline__ uint64_t bh_init(uint64_t len) {
    return 0x9E3779B97F4A7C15ull ^ (len * 0xFF51AFD7ED558CCDull);
}
__device__ __forceinline__ uint64_t bh_step(uint64_t h, uint64_t w) {
    h = (h ^ w) * 0x87C37B91114253D5ull;
    return (h << 31) | (h >> 33);
}
// hash of a string of <= 16 bytes given as zero-padded little-endian words:
// the second word through one odd multiply, the length through a multiply of
// a value below 2^5 (24-bit multiplies), folded into the first word, then the
// partition mixer -- two 64-bit multiplies per string instead of four; every
// byte-record pass recomputes it (round 5)
__device__ __forceinline__ uint64_t bh_short(uint64_t k0, uint64_t k1, uint64_t len) {
    const uint32_t l = (uint32_t)len & 31u;
    const uint64_t lt = ((uint64_t)(l * 0x9E3779u) << 32) | (uint64_t)(l * 0xB97F4Bu);
    const uint64_t m = k1 * 0x9E3779B97F4A7C15ull;
    return mix64(k0 ^ ((m << 29) | (m >> 35)) ^ lt);
}
// hash of a byte record (short: recomputed from the bytes; long: carried in k0)
__device__ __forceinline__ uint64_t rec_hash(uint64_t k0, uint64_t k1, uint64_t meta) {
    const uint64_t len = meta >> 40;
    return len <= SHORT_MAX ? bh_short(k0, k1, len) : k0;
}

// ---- string access --------------------------------------------------------------
__device__ __forceinline__ int64_t str_off(const sdp_bytes_column &c, int64_t row) {
    if (c.fixed_width > 0) return row * (int64_t)c.fixed_width;
    if (c.offset_width == 8) return ((const int64_t *)c.d_offsets)[row];
    return (int64_t)((const int32_t *)c.d_offsets)[row];
}
// 8 bytes at an arbitrary global address (reads aligned dwords; the data
// buffer is padded by 16 bytes), zero beyond `avail`
__device__ __forceinline__ uint64_t gload8(const uint8_t *p, int64_t avail) {
    if (avail <= 0) return 0ull;
    const uint32_t a = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *w = (const uint32_t *)(p - a);   // pointer arithmetic keeps it a global load
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) |
                       ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    return avail >= 8 ? v : (v & ((1ull << (8 * avail)) - 1ull));
}
// 8 bytes at LDS byte offset `off` of a dword-staged buffer
__device__ __forceinline__ uint64_t lload8(const uint32_t *s, int64_t off, int64_t avail) {
    if (avail <= 0) return 0ull;
    const int64_t w = off >> 2;
    const uint32_t sh = (uint32_t)(off & 3);
    const uint32_t w0 = s[w], w1 = s[w + 1], w2 = s[w + 2];
    const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) |
                       ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    return avail >= 8 ? v : (v & ((1ull << (8 * avail)) - 1ull));
}
__device__ uint64_t hash_long_global(const uint8_t *p, int64_t len) {
    uint64_t h = bh_init((uint64_t)len);
    for (int64_t i = 0; i < len; i += 8) h = bh_step(h, gload8(p + i, len - i));
    return mix64(h);
}
__device__ uint64_t hash_long_lds(const uint32_t *s, int64_t off, int64_t len) {
    uint64_t h = bh_init((uint64_t)len);
    for (int64_t i = 0; i < len; i += 8) h = bh_step(h, lload8(s, off + i, len - i));
    return mix64(h);
}
__device__ bool rows_equal_global(const sdp_bytes_column &c, int64_t ra, int64_t rb) {
    // row indices come from record metas: records that are not what the
    // kernels were told (e.g. a layout mismatch between library and caller)
    // must not turn into reads outside the column -- unequal, so the caller
    // flags a collision and recounts on the exact path
    if (ra < 0 || rb < 0 || ra >= c.length || rb >= c.length) return false;
    const int64_t a0 = str_off(c, ra), a1 = str_off(c, ra + 1);
    const int64_t b0 = str_off(c, rb), b1 = str_off(c, rb + 1);
    const int64_t len = a1 - a0;
    if (len != b1 - b0) return false;
    for (int64_t i = 0; i < len; i += 8)
        if (gload8(c.d_data + a0 + i, len - i) != gload8(c.d_data + b0 + i, len - i)) return false;
    return true;
}

// ---- block scan of nb <= MAXB LDS counters (exclusive), NT threads -----------
template <int NT>
__device__ void block_excl_scan(const uint32_t *in, uint32_t *out, int nb, uint32_t *s_wsum) {
    constexpr int PER = (MAXB + NT - 1) / NT;
    const int t = threadIdx.x;
    uint32_t v[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = t * PER + k;
        v[k] = i < nb ? in[i] : 0u;
        sum += v[k];
    }
    // inclusive scan of `sum` across the wave
    uint32_t x = sum;
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, WAVE);
        if (lane >= o) x += y;
    }
    const int w = t / WAVE;
    if (lane == WAVE - 1) s_wsum[w] = x;
    lds_barrier();
    uint32_t wb = 0;
    for (int k = 0; k < w; ++k) wb += s_wsum[k];
    uint32_t run = wb + x - sum;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = t * PER + k;
        if (i < nb) out[i] = run;
        run += v[k];
    }
    lds_barrier();
}

// ---- fixed-width row loading ----------------------------------------------------
__device__ __forceinline__ uint64_t fetch_key(const sdp_column &c, int64_t i, bool &valid) {
    valid = valid_bit(c.d_validity, c.validity_bit_offset, i);
    switch (c.dtype) {
    case SDP_I8: return Elem<int8_t>::key(((const int8_t *)c.d_values)[i]);
    case SDP_I16: return Elem<int16_t>::key(((const int16_t *)c.d_values)[i]);
    case SDP_I32: return Elem<int32_t>::key(((const int32_t *)c.d_values)[i]);
    case SDP_I64: return Elem<int64_t>::key(((const int64_t *)c.d_values)[i]);
    case SDP_U8: return ((const uint8_t *)c.d_values)[i];
    case SDP_U16: return ((const uint16_t *)c.d_values)[i];
    case SDP_U32: return ((const uint32_t *)c.d_values)[i];
    case SDP_U64: return ((const uint64_t *)c.d_values)[i];
    case SDP_F32: return Elem<float>::key(((const float *)c.d_values)[i]);
    case SDP_F64: return Elem<double>::key(((const double *)c.d_values)[i]);
    case SDP_BOOL: {
        const int64_t b = c.validity_bit_offset + i;
        return (((const uint8_t *)c.d_values)[b >> 3] >> (b & 7)) & 1u;
    }
    default: valid = false; return 0;
    }
}

// One tile of NT * RPT rows held in registers.  Full tiles of a vectorisable
// dtype are fetched with 16-byte loads by load() (issued early, so the next
// tile's loads overlap this tile's LDS work); slot q of thread t is row
// base + ((q / VPT) * NT + t) * VPT + q % VPT.  Other tiles are read row by row
// in hash() (slot q = row base + q * NT + t).
template <typename T, int NT, int RPT>
struct RowTile {
    static constexpr bool VEC = !std::is_same<T, bool>::value;
    using VT = typename std::conditional<VEC, T, uint8_t>::type;
    static constexpr int VPT = VEC ? Vec16<T>::N : 1;
    static constexpr int NV = VEC ? (RPT / VPT > 0 ? RPT / VPT : 1) : 1;
    VecIn<VT> v[NV];            // values + raw validity words, decoded in hash()
    bool full;

    __device__ __forceinline__ void load(const sdp_column &c, const VBits &vbm, int64_t base, int64_t end) {
        full = VEC && (RPT % VPT == 0) && base + (int64_t)NT * RPT <= end && (base % VPT) == 0;
        if (!full) return;
        const Vec16<VT> *vals = (const Vec16<VT> *)c.d_values;
#pragma unroll
        for (int u = 0; u < NV; ++u) v[u].load(vals, vbm, base / VPT + (int64_t)u * NT + threadIdx.x, INT64_MAX);
    }
    __device__ __forceinline__ void hash(const sdp_column &c, const VBits &vbm, int64_t base, int64_t end,
                                         uint64_t (&h)[RPT], uint32_t &vmask) const {
        vmask = 0;
        if constexpr (VEC) {
            if (full) {
#pragma unroll
                for (int u = 0; u < NV; ++u) {
                    const uint32_t vb = v[u].bits(vbm);
#pragma unroll
                    for (int e = 0; e < VPT; ++e) {
                        const int q = u * VPT + e;
                        h[q] = mix64(key_of<T>(v[u].v.v[e]));
                        vmask |= ((vb >> e) & 1u) << q;
                    }
                }
                return;
            }
        }
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int64_t i = base + (int64_t)q * NT + threadIdx.x;
            h[q] = 0;
            if (i < end) {
                bool ok;
                const uint64_t k = fetch_key(c, i, ok);
                h[q] = mix64(k);
                vmask |= (uint32_t)ok << q;
            }
        }
    }
};

// ---- rows -> L1 buckets (fixed width) ------------------------------------------
// Phase 0 (count): small LDS, many waves per CU; phase 1 (scatter): 1024
// threads, an 8 K-row tile counting-sorted by bucket in LDS so every bucket's
// run leaves as one contiguous write.  Both phases see the same rows per block.
constexpr int CT = 256;                 // count-phase threads
constexpr int C_RPT = 16;
constexpr int ST = 1024;                // scatter-phase threads
constexpr int S_RPT = 16;
constexpr int S_TILE = ST * S_RPT;      // 16 K rows / records per scatter tile (128 KB stage)
constexpr int ROWS_ALIGN = S_TILE;      // rows per block are a multiple of this

struct CountLds {
    HeavyLdsT<false> heavy;
    uint32_t hist[MAXB];
};

template <typename T>
__global__ void __launch_bounds__(CT) part_count_rows_u64_kernel(sdp_column col, HeavyArg heavy, int b1,
                                                                 int64_t rows_per_block, uint32_t *hist,
                                                                 uint64_t *heavy_counts, uint64_t *stats) {
    __shared__ CountLds s;
    const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
    const int nb = 1 << b1;
    const int shift = 64 - b1;
    const int64_t r0 = (int64_t)g * rows_per_block;
    const int64_t r1 = min(col.length, r0 + rows_per_block);
    heavy_build<false>(s.heavy, heavy);
    for (int b = t; b < nb; b += CT) s.hist[b] = 0;
    lds_barrier();
    uint64_t rows = 0, special = 0;
    const bool any_heavy = heavy.n > 0;
    RowTile<T, CT, C_RPT> tile;
    const VBits vbm = vbits_init(col.d_validity, col.validity_bit_offset, col.d_values);
    for (int64_t base = r0; base < r1; base += CT * C_RPT) {
        uint64_t h[C_RPT];
        uint32_t vmask;
        tile.load(col, vbm, base, r1);
        tile.hash(col, vbm, base, r1, h, vmask);
#pragma unroll
        for (int q = 0; q < C_RPT; ++q) {
            if ((vmask >> q) & 1u) {
                ++rows;
                const int hv = any_heavy ? heavy_find_u64(s.heavy, heavy.n, h[q]) : -1;
                if (hv >= 0) atomicAdd(&s.heavy.cnt[hv], 1u);
                else if (h[q] == EMPTY64) ++special;       // the key whose hash is the empty marker
                else atomicAdd(&s.hist[b1 ? (int)(h[q] >> shift) : 0], 1u);
            }
        }
    }
    lds_barrier();
    for (int b = t; b < nb; b += CT) hist[(int64_t)b * G + g] = s.hist[b];
    heavy_flush(s.heavy, heavy.n, heavy_counts);
    block_add_u64(rows, &stats[0]);
    block_add_u64(special, &stats[1]);
}

// ---- write-combined bucket output ------------------------------------------------
// A scatter appends each bucket's records at that bucket's cursor.  Written
// straight from a tile sorted in LDS, a bucket's run per 16 K-record tile (~16
// records) starts and ends inside 128-byte lines, and the two half-filled lines
// of every run reach HBM separately: 6.1 ms per 1e9 records against 3.8 ms when
// every write is one whole aligned line (1024 streams per workgroup, 256
// workgroups; tools/ubench/scatter_bench.hip, profiles/r04sb_scatter_bench.txt).
// So each bucket's current line is assembled in LDS and leaves whole once it
// fills; lines a tile fills entirely go out directly (their records are written
// together, the L2 merges them), and only a segment's first and last lines are
// written in part.  Used by the record scatters: fixed keys (f64_norm 1e9
// records: 4.1-5.1 -> 3.1 ms) and byte keys' level-1 / level-2 (64-byte lines;
// C3 step 11.5 -> 9.4 and 9.2 -> 7.1 ms) and, since round 5, the row scatter
// (scatter_rows_u64_wc_body: its time had moved with where its records land).
// (WcLdsT<NA, L, NBM>: NA parallel record arrays (1 for fixed keys, 3 for the
// k0 / k1 / meta of byte keys), lines of L records, at most NBM buckets.)
template <int NA, int L, int NBM>
struct WcLdsT {
    uint64_t line[NA][NBM][L];                  // bucket b's current line (slots lo[b] .. cur[b] % L filled)
    uint64_t cur[NBM];                          // bucket b's next output position
    uint32_t cnt[NBM];                          // this tile's records of bucket b
    uint16_t list[NBM];                         // buckets whose current line this tile completes
    uint8_t lo[NBM];                            // first slot of the current line that is this segment's
    uint32_t nlist;
};
using WcLds = WcLdsT<1, 16, MAXB>;              // fixed keys: 128-byte lines, 1024 buckets (146 KB)
template <int NA> struct WcOut { uint64_t *a[NA]; };
// (owner thread of bucket b) the records of the current line not yet written
template <int NA, int L, int NBM>
__device__ __forceinline__ void wc_flush_partial(WcLdsT<NA, L, NBM> &s, int b, const WcOut<NA> &out) {
    const uint64_t c = s.cur[b];
    const uint64_t base = c & ~(uint64_t)(L - 1);
    const int e = (int)(c & (L - 1));
    for (int j = s.lo[b]; j < e; ++j)
#pragma unroll
        for (int a = 0; a < NA; ++a) out.a[a][base + j] = s.line[a][b][j];
}
template <int NA, int L, int NBM>
__device__ __forceinline__ void wc_start(WcLdsT<NA, L, NBM> &s, int b, uint64_t pos) {
    s.cur[b] = pos;
    s.lo[b] = (uint8_t)(pos & (L - 1));
    s.cnt[b] = 0;
}
// (owner) continue bucket b at pos: a jump flushes the partial line first
template <int NA, int L, int NBM>
__device__ __forceinline__ void wc_seek(WcLdsT<NA, L, NBM> &s, int b, uint64_t pos, const WcOut<NA> &out) {
    if (pos != s.cur[b]) {
        wc_flush_partial(s, b, out);
        wc_start(s, b, pos);
    }
}
// One tile: record q of this thread (bit q of `have`; values v[.][q]) goes to
// bucket bk(q).  Every thread of the workgroup calls it.
template <int NT, int RPT, int NA, int L, int NBM, typename BK>
__device__ __forceinline__ void wc_tile(WcLdsT<NA, L, NBM> &s, const uint64_t (&v)[NA][RPT], uint32_t have, int nb,
                                        const WcOut<NA> &out, BK &&bk) {
    static_assert(L <= 16 && (L & (L - 1)) == 0, "lines of 2^k <= 16 records");
    const int t = threadIdx.x;
    static_assert(NT * RPT <= 65536, "ranks are packed 16 bits per record");
    uint32_t r[(RPT + 1) / 2] = {};             // rank of record q in its bucket: 16 bits each
#pragma unroll
    for (int q = 0; q < RPT; ++q)
        if ((have >> q) & 1u) r[q / 2] |= atomicAdd(&s.cnt[bk(q)], 1u) << (16 * (q & 1));
    lds_barrier();
    // records of the current line into LDS, of lines this tile fills entirely
    // straight out, of the new partial line held until the current one is out
    static_assert(RPT <= 16, "pending slots are packed 4 bits per record");
    uint32_t pend = 0;
    uint64_t slots = 0;                         // slot of pending record q: bits 4q .. 4q+3
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        if ((have >> q) & 1u) {
            const int b = bk(q);
            const uint64_t c = s.cur[b];
            const uint64_t p = c + ((r[q / 2] >> (16 * (q & 1))) & 0xFFFFu), e = c + s.cnt[b];
            if (p / L == c / L) {
#pragma unroll
                for (int a = 0; a < NA; ++a) s.line[a][b][p & (L - 1)] = v[a][q];
            } else if (p / L != e / L) {
#pragma unroll
                for (int a = 0; a < NA; ++a) out.a[a][p] = v[a][q];
            } else {
                pend |= 1u << q;
                slots |= (p & (L - 1)) << (4 * q);
            }
        }
    }
    for (int b = t; b < nb; b += NT) {
        const uint64_t c = s.cur[b];
        if ((c + s.cnt[b]) / L != c / L) s.list[atomicAdd(&s.nlist, 1u)] = (uint16_t)b;
    }
    lds_barrier();
    // completed lines: L lanes per line, one aligned write per array
    const uint32_t nl = s.nlist;
    for (uint32_t i = t / L; i < nl; i += NT / L) {
        const int b = s.list[i], l = t & (L - 1);
        if (l >= s.lo[b]) {
            const uint64_t o = (s.cur[b] & ~(uint64_t)(L - 1)) + l;
#pragma unroll
            for (int a = 0; a < NA; ++a) out.a[a][o] = s.line[a][b][l];
        }
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < RPT; ++q)
        if ((pend >> q) & 1u) {
            const int b = bk(q), sl = (int)((slots >> (4 * q)) & 15);
#pragma unroll
            for (int a = 0; a < NA; ++a) s.line[a][b][sl] = v[a][q];
        }
    for (int b = t; b < nb; b += NT) {
        const uint64_t c = s.cur[b], e = c + s.cnt[b];
        if (e / L != c / L) s.lo[b] = 0;
        s.cur[b] = e;
        s.cnt[b] = 0;
    }
    if (t == 0) s.nlist = 0;
    lds_barrier();
}

constexpr int WC_RPT = 8;                       // records per thread per tile (16 spills registers, no faster)
// block bx of a G-block grid (the batched launch runs several columns' grids
// side by side, blockIdx.y = column)
// The row scatter (write-combined since round 5): the records of a
// tile go to their buckets through wc_tile -- each bucket's current 128-byte
// line assembled in LDS and written whole -- instead of leaving the sorted
// tile as runs that start and end inside lines.  The row scatter's time moves
// 20 % and more with where its records land (DRAM write back-pressure,
// profiles/r05sp_*), while the write-combined level-2 scatter, which never
// writes a partial line, holds within 3 % across the round's boxes.  Under
// the probe's allocator states (profiles/r05af_rows_scatter_wc_probe_ab.log):
// 4.23-5.36 vs 4.44-5.59 ms per 1e9-row f64 column, the arena state 4.2-4.7
// vs 5.5-5.6.  (Round 4 measured a write-combined row scatter on one box as
// no gain, 4.7-5.1 vs 4.5-5.0 ms.)
struct ScatterWcLds {
    HeavyLdsT<false> heavy;
    WcLds wc;
};
template <typename T>
__device__ __forceinline__ void scatter_rows_u64_wc_body(const sdp_column &col, const HeavyArg &heavy, int b1,
                                                         int64_t rows_per_block, const uint64_t *offs,
                                                         uint64_t *out_h, int xcd_map, const int G, const int bx) {
    __shared__ ScatterWcLds s;
    const int t = threadIdx.x;
    const int g = (xcd_map && G % 8 == 0) ? (int)((bx % 8) * (G / 8) + bx / 8) : bx;
    const int nb = 1 << b1;
    const int shift = 64 - b1;
    const int64_t r0 = (int64_t)g * rows_per_block;
    const int64_t r1 = min(col.length, r0 + rows_per_block);
    heavy_build<false>(s.heavy, heavy);
    for (int b = t; b < nb; b += ST) wc_start(s.wc, b, offs[(int64_t)b * G + g]);
    if (t == 0) s.wc.nlist = 0;
    lds_barrier();
    const bool any_heavy = heavy.n > 0;
    constexpr int64_t TILE = (int64_t)ST * WC_RPT;
    RowTile<T, ST, WC_RPT> tile;
    const VBits vbm = vbits_init(col.d_validity, col.validity_bit_offset, col.d_values);
    WcOut<1> out;
    out.a[0] = out_h;
    if (r0 < r1) tile.load(col, vbm, r0, r1);
    for (int64_t base = r0; base < r1; base += TILE) {
        uint64_t x[1][WC_RPT];
        uint32_t vmask;
        tile.hash(col, vbm, base, r1, x[0], vmask);
        if (base + TILE < r1) tile.load(col, vbm, base + TILE, r1);      // next tile in flight
        uint32_t have = 0;
#pragma unroll
        for (int q = 0; q < WC_RPT; ++q) {
            if ((vmask >> q) & 1u) {
                const int hv = any_heavy ? heavy_find_u64(s.heavy, heavy.n, x[0][q]) : -1;
                if (hv < 0 && x[0][q] != EMPTY64) have |= 1u << q;
            }
        }
        wc_tile<ST, WC_RPT>(s.wc, x, have, nb, out, [&](int q) { return b1 ? (int)(x[0][q] >> shift) : 0; });
    }
    for (int b = t; b < nb; b += ST) wc_flush_partial(s.wc, b, out);
}

template <typename T>
__global__ void __launch_bounds__(ST) part_scatter_rows_u64_kernel(sdp_column col, HeavyArg heavy, int b1,
                                                                   int64_t rows_per_block, const uint64_t *offs,
                                                                   uint64_t *out_h, int xcd_map) {
    scatter_rows_u64_wc_body<T>(col, heavy, b1, rows_per_block, offs, out_h, xcd_map, (int)gridDim.x, (int)blockIdx.x);
}
template <typename T>
__global__ void __launch_bounds__(ST) part_scatter_rows_u64_batch_kernel(const sdp_rows_task *tasks, int xcd_map) {
    const sdp_rows_task &tk = tasks[blockIdx.y];
    if ((int)blockIdx.x >= tk.grid) return;
    const HeavyArg hv{tk.heavy.d_h, nullptr, nullptr, nullptr, tk.heavy.n};
    // (the XCD map needs the column's grid to be the launch's x extent)
    scatter_rows_u64_wc_body<T>(tk.col, hv, tk.b1, tk.rows_per_block, tk.d_offsets, tk.d_out,
                                xcd_map && tk.grid == (int)gridDim.x, tk.grid, (int)blockIdx.x);
}

// ---- rows -> L1 buckets (byte keys) ---------------------------------------------
// Strings are read straight from the column (adjacent rows share cache lines);
// a row becomes (k0, k1, meta) in registers, and the scatter phase stages the
// records of a 4 K-row tile in LDS to write each bucket's run contiguously.
constexpr int B_CT = 256;
constexpr int B_C_RPT = 4;
constexpr int B_ST = 1024;
constexpr int B_S_RPT = 4;
constexpr int B_S_TILE = B_ST * B_S_RPT;   // 4096

__device__ __forceinline__ void bytes_record(const sdp_bytes_column &col, int64_t row, uint64_t &k0, uint64_t &k1,
                                             uint64_t &meta, uint64_t &h) {
    const int64_t o0 = str_off(col, row), o1 = str_off(col, row + 1);
    const int64_t len = o1 - o0;
    if (len <= SHORT_MAX) {
        k0 = gload8(col.d_data + o0, len);
        k1 = gload8(col.d_data + o0 + 8, len - 8);
        h = bh_short(k0, k1, (uint64_t)len);
    } else {
        h = hash_long_global(col.d_data + o0, len);
        k0 = h;
        k1 = 0;
    }
    meta = ((uint64_t)min((int64_t)LEN_MAX, len) << 40) | (uint64_t)(row + 1);
}

__device__ __forceinline__ uint64_t mask_bytes(uint64_t v, int64_t avail) {
    return avail <= 0 ? 0ull : (avail >= 8 ? v : (v & ((1ull << (8 * avail)) - 1ull)));
}

// A tile of rows in stages: A1 issues the validity bytes and offsets, A2 turns
// them into a mask and lengths, B1 issues the key words (which depend on A), B2
// decodes and hashes.  The row kernels run A2(i) B1(i) A1(i+1) B2(i): the next
// tile's stage A is in flight while this tile is decoded and stored.  (A
// wave-cooperative B1 -- each wave's span of key bytes read as coalesced 16-byte
// chunks and handed to the lanes by ds_bpermute -- measured 12 % slower on the
// count pass: 8.8 -> 9.9 ms per 1e9 rows.)
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

template <int RPT>
struct BytesOffs {
    int64_t o0[RPT];
    uint32_t ln[RPT];                   // string length (strings of >= 4 GiB are not supported)
    uint32_t vmask;
};
// OW: the offsets layout -- 8 or 4 (Arrow offsets of that width) or 0 (fixed
// width) -- a template argument, so no layout test sits between the loads.
// the OW a column's layout selects (-1: neither)
static inline int bytes_ow(const sdp_bytes_column &col) {
    if (col.fixed_width > 0) return 0;
    return (col.offset_width == 8 || col.offset_width == 4) ? col.offset_width : -1;
}
template <int RPT>
struct BytesRaw {                       // stage A as loaded: not yet waited on
    int64_t o0[RPT], o1[RPT];
    uint32_t vb[RPT];                   // the validity byte holding the row's bit
};
// stage A1: issue every load of the tile and use none of them.  Rows past the
// end are clamped to the last row and offsets are read whether or not the row
// is valid (an Arrow offsets buffer always holds length + 1 entries), so there
// is no control flow between the loads; the layout is a template argument.
// Testing validity right after the loads waits them out in place -- one memory
// latency per row (the records kernel measured 71 % of its wave cycles waiting).
template <int NT, int RPT, int OW>
__device__ __forceinline__ void bytes_tile_issue(const sdp_bytes_column &col, int64_t base, int64_t end,
                                                 BytesRaw<RPT> &raw, int t) {
    // without a validity bitmap the byte comes from a buffer that is at least
    // length / 8 bytes long and stage A2 forces it to all-valid (a load either
    // way, so no branch splits the tile's loads)
    const bool has_valid = col.d_validity != nullptr;
    const uint8_t *vp = has_valid ? col.d_validity : (OW == 0 ? col.d_data : (const uint8_t *)col.d_offsets);
    const int64_t vo = has_valid ? col.validity_bit_offset : 0;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const int64_t r = min(base + (int64_t)q * NT + t, end - 1);
        raw.vb[q] = vp[(vo + r) >> 3];
        if constexpr (OW == 0) {
            raw.o0[q] = r * (int64_t)col.fixed_width;
            raw.o1[q] = raw.o0[q] + col.fixed_width;
        } else if constexpr (OW == 8) {
            raw.o0[q] = ((const int64_t *)col.d_offsets)[r];
            raw.o1[q] = ((const int64_t *)col.d_offsets)[r + 1];
        } else {
            raw.o0[q] = ((const int32_t *)col.d_offsets)[r];
            raw.o1[q] = ((const int32_t *)col.d_offsets)[r + 1];
        }
    }
}
// The row kernels issue the next tile's stage A unconditionally -- past the
// last tile it re-reads the last row -- so the count of loads in flight is the
// same on every path and the wait for this tile's key words leaves them flying.
// stage A2: validity mask and lengths (register work only; the first use of
// the loads, so it belongs where the tile is about to be worked on)
template <int NT, int RPT>
__device__ __forceinline__ void bytes_tile_ready(const sdp_bytes_column &col, int64_t base, int64_t end,
                                                 const BytesRaw<RPT> &raw, BytesOffs<RPT> &a, int t) {
    const uint32_t vfill = col.d_validity ? 0u : 0xFFu;
    a.vmask = 0;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const int64_t row = base + (int64_t)q * NT + t;
        const uint32_t ok =
            (uint32_t)(row < end) & ((raw.vb[q] | vfill) >> ((col.validity_bit_offset + row) & 7)) & 1u;
        a.vmask |= ok << q;
        a.o0[q] = ok ? raw.o0[q] : 0;
        // (the clamp reads o1's high word: a loaded register left dead is
        // reused for temporaries while its load is still in flight, and every
        // such reuse waits for all outstanding loads)
        a.ln[q] = ok ? (uint32_t)min(raw.o1[q] - raw.o0[q], (int64_t)UINT32_MAX) : 0u;
    }
}

// stage B1: the key words of a tile (issue only)
template <int RPT>
__device__ __forceinline__ void bytes_tile_words(const sdp_bytes_column &col, const BytesOffs<RPT> &a,
                                                 uint32_t (&w)[RPT][5]) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const int64_t len = a.ln[q];
        const uint8_t *pb = col.d_data + a.o0[q];
        const uint32_t ad = (uint32_t)((uintptr_t)pb & 3u);
        const uint32_t *p = (const uint32_t *)(pb - ad);
        const int64_t need = len <= SHORT_MAX ? (int64_t)(ad + len + 3) >> 2 : 0;
        // words 0-3 as ONE 16-byte load (dword-aligned: unaligned-access mode;
        // the data buffer's 16 padding bytes cover it), word 4 only when the
        // string reaches it -- two load instructions per row instead of five
        const bool ok = ((a.vmask >> q) & 1u) && need > 0;
        const u32x4a4 v = ok ? *(const u32x4a4 *)p : u32x4a4{0u, 0u, 0u, 0u};
        w[q][0] = v.x; w[q][1] = v.y; w[q][2] = v.z; w[q][3] = v.w;
        w[q][4] = (ok && need > 4) ? p[4] : 0u;
    }
}
// (round 5) every lane forms the short-string record, selects zero for an
// invalid row, and only a wave holding a string of more than 16 bytes takes
// the long-hash branch: the per-row valid / short / long branches had cost
// ~160 scalar instructions per 64 rows in exec-mask bookkeeping
template <int NT, int RPT>
__device__ __forceinline__ void bytes_tile_decode(const sdp_bytes_column &col, int64_t base, const BytesOffs<RPT> &a,
                                                  const uint32_t (&w)[RPT][5], uint64_t (&k0)[RPT],
                                                  uint64_t (&k1)[RPT], uint64_t (&meta)[RPT], uint64_t (&h)[RPT],
                                                  int t) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const bool ok = (a.vmask >> q) & 1u;
        const int64_t row = base + (int64_t)q * NT + t;
        const int64_t len = a.ln[q];                   // 0 for an invalid row
        const uint32_t sh = (uint32_t)((uintptr_t)(col.d_data + a.o0[q]) & 3);
        const uint64_t v0 = (uint64_t)__builtin_amdgcn_alignbyte(w[q][1], w[q][0], sh) |
                            ((uint64_t)__builtin_amdgcn_alignbyte(w[q][2], w[q][1], sh) << 32);
        const uint64_t v1 = (uint64_t)__builtin_amdgcn_alignbyte(w[q][3], w[q][2], sh) |
                            ((uint64_t)__builtin_amdgcn_alignbyte(w[q][4], w[q][3], sh) << 32);
        const uint64_t a0 = mask_bytes(v0, len), a1 = mask_bytes(v1, len - 8);
        uint64_t hh = bh_short(a0, a1, (uint64_t)len);
        uint64_t b0 = a0, b1 = a1;
        const bool lng = ok && len > SHORT_MAX;
        if (__ballot(lng)) {                           // wave-uniform, rare
            if (lng) {
                hh = hash_long_global(col.d_data + a.o0[q], len);
                b0 = hh;
                b1 = 0;
            }
        }
        k0[q] = ok ? b0 : 0;
        k1[q] = ok ? b1 : 0;
        h[q] = ok ? hh : 0;
        meta[q] = ok ? (((uint64_t)min((int64_t)LEN_MAX, len) << 40) | (uint64_t)(row + 1)) : 0;
    }
}

struct BCountLds {
    HeavyLdsT<true> heavy;
    uint32_t hist[MAXB];
};
struct BScatterLds {
    HeavyLdsT<true> heavy;
    uint32_t hist[MAXB];
    uint32_t off[MAXB];
    uint64_t cur[MAXB];
    uint64_t k0[B_S_TILE];
    uint64_t k1[B_S_TILE];
    uint64_t meta[B_S_TILE];
    uint16_t bkt[B_S_TILE];
    uint32_t wsum[B_ST / WAVE];
};

template <int OW>
__global__ void __launch_bounds__(B_CT) part_count_rows_bytes_kernel(sdp_bytes_column col, HeavyArg heavy, int b1,
                                                                     int64_t rows_per_block, uint32_t *hist,
                                                                     uint64_t *heavy_counts, uint64_t *stats) {
    __shared__ BCountLds s;
    const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
    const int nb = 1 << b1;
    const int shift = 64 - b1;
    const int64_t r0 = (int64_t)g * rows_per_block;
    const int64_t r1 = min(col.length, r0 + rows_per_block);
    heavy_build<true>(s.heavy, heavy);
    for (int b = t; b < nb; b += B_CT) s.hist[b] = 0;
    lds_barrier();
    uint64_t rows = 0;
    constexpr int64_t STEP = (int64_t)B_CT * B_C_RPT;
    BytesRaw<B_C_RPT> raw;
    if (r0 < r1) bytes_tile_issue<B_CT, B_C_RPT, OW>(col, r0, r1, raw, t);
    for (int64_t base = r0; base < r1; base += STEP) {
        uint64_t k0[B_C_RPT], k1[B_C_RPT], meta[B_C_RPT], h[B_C_RPT];
        uint32_t wd[B_C_RPT][5];
        BytesOffs<B_C_RPT> oc;
        bytes_tile_ready<B_CT, B_C_RPT>(col, base, r1, raw, oc, t);
        bytes_tile_words<B_C_RPT>(col, oc, wd);
        bytes_tile_issue<B_CT, B_C_RPT, OW>(col, base + STEP, r1, raw, t);   // next tile in flight (see below)
        bytes_tile_decode<B_CT, B_C_RPT>(col, base, oc, wd, k0, k1, meta, h, t);
        const uint32_t vmask = oc.vmask;
#pragma unroll
        for (int q = 0; q < B_C_RPT; ++q) {
            if ((vmask >> q) & 1u) {
                ++rows;
                const int hv = heavy_find_bytes(s.heavy, heavy.n, h[q], k0[q], k1[q], (uint32_t)(meta[q] >> 40));
                if (hv >= 0) atomicAdd(&s.heavy.cnt[hv], 1u);
                else atomicAdd(&s.hist[b1 ? (int)(h[q] >> shift) : 0], 1u);
            }
        }
    }
    lds_barrier();
    for (int b = t; b < nb; b += B_CT) hist[(int64_t)b * G + g] = s.hist[b];
    heavy_flush(s.heavy, heavy.n, heavy_counts);
    block_add_u64(rows, &stats[0]);
}

template <int OW>
__global__ void __launch_bounds__(B_ST) part_scatter_rows_bytes_kernel(sdp_bytes_column col, HeavyArg heavy, int b1,
                                                                       int64_t rows_per_block, const uint64_t *offs,
                                                                       uint64_t *out_k0, uint64_t *out_k1,
                                                                       uint64_t *out_meta) {
    __shared__ BScatterLds s;
    const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
    const int nb = 1 << b1;
    const int shift = 64 - b1;
    const int64_t r0 = (int64_t)g * rows_per_block;
    const int64_t r1 = min(col.length, r0 + rows_per_block);
    heavy_build<true>(s.heavy, heavy);
    for (int b = t; b < nb; b += B_ST) {
        s.hist[b] = 0;
        s.cur[b] = offs[(int64_t)b * G + g];
    }
    lds_barrier();
    BytesRaw<B_S_RPT> raw;
    if (r0 < r1) bytes_tile_issue<B_ST, B_S_RPT, OW>(col, r0, r1, raw, t);
    for (int64_t base = r0; base < r1; base += B_S_TILE) {
        uint64_t k0[B_S_RPT], k1[B_S_RPT], meta[B_S_RPT], h[B_S_RPT];
        uint32_t rank[B_S_RPT];
        int bk[B_S_RPT];
        uint32_t keep = 0;
        uint32_t wd[B_S_RPT][5];
        BytesOffs<B_S_RPT> oc;
        bytes_tile_ready<B_ST, B_S_RPT>(col, base, r1, raw, oc, t);
        bytes_tile_words<B_S_RPT>(col, oc, wd);
        // the next tile's stage A flies during this tile's LDS phases
        bytes_tile_issue<B_ST, B_S_RPT, OW>(col, base + B_S_TILE, r1, raw, t);
        bytes_tile_decode<B_ST, B_S_RPT>(col, base, oc, wd, k0, k1, meta, h, t);
        const uint32_t vmask = oc.vmask;
#pragma unroll
        for (int q = 0; q < B_S_RPT; ++q) {
            if ((vmask >> q) & 1u) {
                const int hv = heavy_find_bytes(s.heavy, heavy.n, h[q], k0[q], k1[q], (uint32_t)(meta[q] >> 40));
                if (hv < 0) {
                    keep |= 1u << q;
                    bk[q] = b1 ? (int)(h[q] >> shift) : 0;
                    rank[q] = atomicAdd(&s.hist[bk[q]], 1u);
                }
            }
        }
        lds_barrier();
        block_excl_scan<B_ST>(s.hist, s.off, nb, s.wsum);
#pragma unroll
        for (int q = 0; q < B_S_RPT; ++q) {
            if ((keep >> q) & 1u) {
                const uint32_t p = s.off[bk[q]] + rank[q];
                s.k0[p] = k0[q];
                s.k1[p] = k1[q];
                s.meta[p] = meta[q];
                s.bkt[p] = (uint16_t)bk[q];
            }
        }
        lds_barrier();
        const uint32_t total = s.off[nb - 1] + s.hist[nb - 1];
        for (uint32_t j = t; j < total; j += B_ST) {
            const int b = s.bkt[j];
            const uint64_t o = s.cur[b] + (j - s.off[b]);
            out_k0[o] = s.k0[j];
            out_k1[o] = s.k1[j];
            out_meta[o] = s.meta[j];
        }
        lds_barrier();
        for (int b = t; b < nb; b += B_ST) {
            s.cur[b] += s.hist[b];
            s.hist[b] = 0;
        }
        lds_barrier();
    }
}

// ---- L1 records -> L2 buckets ----------------------------------------------------
// Chunk c = records [start, end) of one L1 bucket; its histogram entry for
// sub-bucket s lives at hbase + s * hstride (so the flat exclusive scan orders
// records by (L1 bucket, sub-bucket, chunk)).
struct Chunk {
    int64_t start, end, hbase, hstride;
};

// ---- byte rows -> compacted records (one read of the strings) ----------------------
// The string bytes are the expensive read of a byte column (offsets, then
// unaligned key words, then the hash).  Counting level-1 buckets in one pass and
// scattering in a second would read them twice; instead every wave turns its
// own strip of rows into records written contiguously from the strip's first
// row position (ballot + mbcnt compaction, no atomics), counts their level-1
// buckets in a wave-private LDS histogram, and publishes its strip as a Chunk.
// part_scatter_recs_kernel<true> (b1 = 0, b2 = level-1 bits) then moves the
// records -- 24 B each, sequential reads -- into their buckets.  Heavy keys are
// counted in LDS and never become records, as in the other row kernels.
constexpr int BR_T = 1024;                  // 16 waves, one strip each, one workgroup per CU
                                            // (<= 128 VGPRs; the 256-block grid is resident in
                                            // one round) -- the LDS holds 1024 heavy keys
constexpr int BR_W = BR_T / WAVE;
constexpr int BR_RPT = 4;                   // rows per lane per tile

struct BRecLds {
    HeavyRecT<HEAVY_MAX_REC> heavy;
    uint32_t hist[BR_W][MAXB];
};
static_assert(sizeof(BRecLds) <= 150 * 1024, "records kernel LDS");

constexpr int BR_MINB = 1;
template <int OW>
__global__ void __launch_bounds__(BR_T, BR_MINB) part_records_rows_bytes_kernel(sdp_bytes_column col, HeavyArg heavy, int b1,
                                                                       int64_t rows_per_block, uint32_t *hist,
                                                                       Chunk *chunks, uint64_t *out_k0,
                                                                       uint64_t *out_k1, uint64_t *out_meta,
                                                                       uint64_t *heavy_counts, uint64_t *stats) {
    __shared__ BRecLds s;
    const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
    const int lane = lane_id(), w = t / WAVE;
    const int nb = 1 << b1;
    const int shift = 64 - b1;
    const int64_t rpw = rows_per_block / BR_W;                     // a multiple of WAVE * BR_RPT
    const int64_t s0 = min(col.length, (int64_t)g * rows_per_block + (int64_t)w * rpw);
    const int64_t s1 = min(col.length, s0 + rpw);
    heavy_rec_build(s.heavy, heavy);
    for (int b = lane; b < nb; b += WAVE) s.hist[w][b] = 0;
    lds_barrier();
    uint64_t rows = 0;
    int64_t cur = s0;                                               // next record slot of this strip
    constexpr int64_t STEP = (int64_t)WAVE * BR_RPT;
    BytesRaw<BR_RPT> raw;
    if (s0 < s1) bytes_tile_issue<WAVE, BR_RPT, OW>(col, s0, s1, raw, lane);
    for (int64_t base = s0; base < s1; base += STEP) {
        uint64_t k0[BR_RPT], k1[BR_RPT], meta[BR_RPT], h[BR_RPT];
        uint32_t wd[BR_RPT][5];
        BytesOffs<BR_RPT> oc;
        bytes_tile_ready<WAVE, BR_RPT>(col, base, s1, raw, oc, lane);
        bytes_tile_words<BR_RPT>(col, oc, wd);                  // this tile's key words, then
        bytes_tile_issue<WAVE, BR_RPT, OW>(col, base + STEP, s1, raw, lane);   // the next tile's stage A
        bytes_tile_decode<WAVE, BR_RPT>(col, base, oc, wd, k0, k1, meta, h, lane);
        const uint32_t vmask = oc.vmask;
        int hv[BR_RPT];
        heavy_rec_find(s.heavy, heavy.n, h, k0, k1, meta, vmask, hv);
#pragma unroll
        for (int q = 0; q < BR_RPT; ++q) {
            bool keep = false;
            if ((vmask >> q) & 1u) {
                ++rows;
                if (hv[q] >= 0) atomicAdd(&s.heavy.cnt[hv[q]], 1u);
                else keep = true;
            }
            const uint64_t m = __ballot(keep);
            if (keep) {
                const int64_t o = cur + lane_rank(m);
                out_k0[o] = k0[q];
                out_k1[o] = k1[q];
                out_meta[o] = meta[q];
                atomicAdd(&s.hist[w][b1 ? (int)(h[q] >> shift) : 0], 1u);
            }
            cur += __popcll(m);
        }
    }
    const int64_t C = (int64_t)G * BR_W, c = (int64_t)g * BR_W + w;
    lds_barrier();
    for (int b = lane; b < nb; b += WAVE) hist[(int64_t)b * C + c] = s.hist[w][b];
    if (lane == 0) chunks[c] = Chunk{s0, cur, c, C};
    heavy_rec_flush(s.heavy, heavy.n, heavy_counts);
    block_add_u64(rows, &stats[0]);
}

// fixed keys: 16-byte loads of record pairs (an even record index; the pairs
// that straddle a chunk edge are read element by element), then one LDS atomic
// per record
__global__ void __launch_bounds__(CT) part_count_recs_u64_kernel(const uint64_t *in_k0, const Chunk *chunks,
                                                                 int64_t nchunks, int b1, int b2, uint32_t *hist) {
    constexpr int PP = 8;                       // record pairs per thread per step
    __shared__ uint32_t s_hist[MAXB];
    const int t = threadIdx.x;
    const int nb = 1 << b2;
    const int shift = 64 - b1 - b2;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const Chunk ch = chunks[c];
        for (int b = t; b < nb; b += CT) s_hist[b] = 0;
        lds_barrier();
        const int64_t a0 = ch.start & ~(int64_t)1;
        for (int64_t base = a0; base < ch.end; base += (int64_t)CT * PP * 2) {
            uint64_t x[PP][2];
            int64_t rr[PP];
#pragma unroll
            for (int q = 0; q < PP; ++q) {
                const int64_t r = base + 2 * ((int64_t)q * CT + t);
                rr[q] = r;
                if (r >= ch.start && r + 1 < ch.end) {
                    const ulonglong2 v = *(const ulonglong2 *)(in_k0 + r);
                    x[q][0] = v.x; x[q][1] = v.y;
                } else {
                    x[q][0] = (r >= ch.start && r < ch.end) ? in_k0[r] : 0ull;
                    x[q][1] = (r + 1 >= ch.start && r + 1 < ch.end) ? in_k0[r + 1] : 0ull;
                }
            }
#pragma unroll
            for (int q = 0; q < PP; ++q)
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int64_t r = rr[q] + e;
                    if (r >= ch.start && r < ch.end)
                        atomicAdd(&s_hist[(int)((x[q][e] >> shift) & (uint64_t)(nb - 1))], 1u);
                }
        }
        lds_barrier();
        for (int b = t; b < nb; b += CT) hist[ch.hbase + (int64_t)b * ch.hstride] = s_hist[b];
        lds_barrier();
    }
}

template <bool BYTES>
__global__ void __launch_bounds__(CT) part_count_recs_kernel(const uint64_t *in_k0, const uint64_t *in_k1,
                                                             const uint64_t *in_meta, const Chunk *chunks,
                                                             int64_t nchunks, int b1, int b2, uint32_t *hist) {
    constexpr int RPT = BYTES ? 8 : 16;
    __shared__ uint32_t s_hist[MAXB];
    const int t = threadIdx.x;
    const int nb = 1 << b2;
    const int shift = 64 - b1 - b2;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const Chunk ch = chunks[c];
        for (int b = t; b < nb; b += CT) s_hist[b] = 0;
        lds_barrier();
        for (int64_t base = ch.start; base < ch.end; base += CT * RPT) {
            uint64_t k0[RPT], k1[RPT], meta[RPT];
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const int64_t r = base + (int64_t)q * CT + t;
                if (r < ch.end) {
                    k0[q] = in_k0[r];
                    if (BYTES) { k1[q] = in_k1[r]; meta[q] = in_meta[r]; }
                }
            }
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const int64_t r = base + (int64_t)q * CT + t;
                if (r < ch.end) {
                    const uint64_t h = BYTES ? rec_hash(k0[q], k1[q], meta[q]) : k0[q];
                    atomicAdd(&s_hist[(int)((h >> shift) & (uint64_t)(nb - 1))], 1u);
                }
            }
        }
        lds_barrier();
        for (int b = t; b < nb; b += CT) hist[ch.hbase + (int64_t)b * ch.hstride] = s_hist[b];
        lds_barrier();
    }
}

template <bool BYTES>
struct RecsLds {
    uint32_t hist[MAXB];
    uint32_t off[MAXB];
    uint64_t cur[MAXB];
    uint64_t k0[BYTES ? B_S_TILE : S_TILE];
    uint64_t k1[BYTES ? B_S_TILE : 1];
    uint64_t meta[BYTES ? B_S_TILE : 1];
    uint16_t bkt[BYTES ? B_S_TILE : 1];     // fixed keys: the bucket is recomputed from the key
    uint32_t wsum[ST / WAVE];
};

template <bool BYTES>
__global__ void __launch_bounds__(ST) part_scatter_recs_kernel(const uint64_t *in_k0, const uint64_t *in_k1,
                                                               const uint64_t *in_meta, const Chunk *chunks,
                                                               int64_t nchunks, int b1, int b2, const uint64_t *offs,
                                                               uint64_t *out_k0, uint64_t *out_k1,
                                                               uint64_t *out_meta, int xcd_map) {
    constexpr int RPT = BYTES ? B_S_RPT : S_RPT;
    constexpr int TILE = ST * RPT;
    __shared__ RecsLds<BYTES> s;
    const int t = threadIdx.x;
    const int nb = 1 << b2;
    const int shift = 64 - b1 - b2;
    // XCD-aware (as in the row scatter): each XCD takes one contiguous range of
    // chunks, so the chunks it runs at once are neighbours in every sub-bucket
    const bool xm = xcd_map && gridDim.x % 8 == 0;
    const int64_t per = xm ? (nchunks + 7) / 8 : nchunks;
    const int64_t c0 = xm ? (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8 : (int64_t)blockIdx.x;
    const int64_t c1 = xm ? min(nchunks, (int64_t)(blockIdx.x % 8 + 1) * per) : nchunks;
    const int64_t cstep = xm ? gridDim.x / 8 : gridDim.x;
    // A chunk's bucket offsets and first tile are loaded while the previous
    // chunk's last tile is sorted (nb <= ST: thread t owns sub-bucket t), so a
    // chunk no longer starts with three dependent memory latencies (header,
    // offsets, first tile) in front of an otherwise idle workgroup.
    auto load_tile = [&](int64_t base, int64_t end, uint64_t (&a0)[RPT], uint64_t (&a1)[RPT],
                         uint64_t (&am)[RPT]) {
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int64_t r = base + (int64_t)q * ST + t;
            if (r < end) {
                a0[q] = in_k0[r];
                if (BYTES) { a1[q] = in_k1[r]; am[q] = in_meta[r]; }
            }
        }
    };
    // chunk headers are wave-uniform: kept in scalar registers
    auto uniform_chunk = [](const Chunk &x) {
        auto u = [](int64_t v) {
            const uint32_t lo = uniform_u32((uint32_t)v);
            const uint32_t hi = uniform_u32((uint32_t)((uint64_t)v >> 32));
            return (int64_t)(((uint64_t)hi << 32) | lo);
        };
        return Chunk{u(x.start), u(x.end), u(x.hbase), u(x.hstride)};
    };
    uint64_t k0[RPT], k1[RPT], meta[RPT];
    Chunk ch{0, 0, 0, 0};
    uint64_t cur_next = 0;
    if (c0 < c1) {
        ch = uniform_chunk(chunks[c0]);
        if (t < nb) cur_next = offs[ch.hbase + (int64_t)t * ch.hstride];
        load_tile(ch.start, ch.end, k0, k1, meta);
    }
    for (int64_t c = c0; c < c1; c += cstep) {
        if (t < nb) {
            s.hist[t] = 0;
            s.cur[t] = cur_next;
        }
        const int64_t cn = c + cstep;
        const Chunk chn = cn < c1 ? uniform_chunk(chunks[cn]) : Chunk{0, 0, 0, 0};
        lds_barrier();
        for (int64_t base = ch.start; base < ch.end; base += TILE) {
            uint32_t rank[RPT];
            int bk[RPT];
            uint64_t x0[RPT], x1[RPT], xm[RPT];
            uint32_t have = 0;
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                const int64_t r = base + (int64_t)q * ST + t;
                x0[q] = k0[q];
                if (BYTES) { x1[q] = k1[q]; xm[q] = meta[q]; }
                if (r < ch.end) {
                    have |= 1u << q;
                    const uint64_t h = BYTES ? rec_hash(x0[q], x1[q], xm[q]) : x0[q];
                    bk[q] = (int)((h >> shift) & (uint64_t)(nb - 1));
                    rank[q] = atomicAdd(&s.hist[bk[q]], 1u);
                }
            }
            // the next tile (of this chunk, or the next chunk's first with its
            // bucket offsets) in flight during the LDS work
            const int64_t nbase = base + TILE;
            const bool last = nbase >= ch.end;                 // wave-uniform
            if (last && cn < c1 && t < nb) cur_next = offs[chn.hbase + (int64_t)t * chn.hstride];
            load_tile(last ? chn.start : nbase, last ? chn.end : ch.end, k0, k1, meta);
            lds_barrier();
            block_excl_scan<ST>(s.hist, s.off, nb, s.wsum);
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                if ((have >> q) & 1u) {
                    const uint32_t p = s.off[bk[q]] + rank[q];
                    s.k0[p] = x0[q];
                    if (BYTES) { s.k1[p] = x1[q]; s.meta[p] = xm[q]; s.bkt[p] = (uint16_t)bk[q]; }
                }
            }
            lds_barrier();
            const uint32_t total = s.off[nb - 1] + s.hist[nb - 1];
            for (uint32_t j = t; j < total; j += ST) {
                const uint64_t x = s.k0[j];
                const int b = BYTES ? (int)s.bkt[j] : (int)((x >> shift) & (uint64_t)(nb - 1));
                const uint64_t o = s.cur[b] + (j - s.off[b]);
                out_k0[o] = x;
                if (BYTES) { out_k1[o] = s.k1[j]; out_meta[o] = s.meta[j]; }
            }
            lds_barrier();
            for (int b = t; b < nb; b += ST) {
                s.cur[b] += s.hist[b];
                s.hist[b] = 0;
            }
            lds_barrier();
        }
        if (ch.start >= ch.end && cn < c1) {               // (an empty chunk prefetched nothing)
            if (t < nb) cur_next = offs[chn.hbase + (int64_t)t * chn.hstride];
            load_tile(chn.start, chn.end, k0, k1, meta);
        }
        ch = chn;
    }
}

// Write-combined scatter of partition records (WcLdsT): workgroup g takes one
// contiguous range of chunks, so consecutive chunks of one level-1 bucket
// continue every sub-bucket's cursor (the chunk-major order of the level-2
// offsets), and a sub-bucket's partial line is flushed only where the next
// chunk's offset jumps.  Fixed keys: 128-byte lines of 1024 sub-buckets.  Byte
// keys (k0 / k1 / meta, three arrays): 64-byte lines of <= 512 buckets, so the
// three line buffers fit in 96 KB.
template <bool BYTES> struct WcRecs {
    static constexpr int NA = BYTES ? 3 : 1;
    static constexpr int L = BYTES ? 8 : 16;
    static constexpr int NBM = BYTES ? 512 : MAXB;
    static constexpr int RPT = BYTES ? 4 : WC_RPT;
    using Lds = WcLdsT<NA, L, NBM>;
};
template <bool BYTES>
__global__ void __launch_bounds__(ST) part_scatter_recs_wc_kernel(const uint64_t *in_k0, const uint64_t *in_k1,
                                                                  const uint64_t *in_meta, const Chunk *chunks,
                                                                  int64_t nchunks, int b1, int b2,
                                                                  const uint64_t *offs, uint64_t *out_k0,
                                                                  uint64_t *out_k1, uint64_t *out_meta, int xcd_map) {
    using W = WcRecs<BYTES>;
    constexpr int RPT = W::RPT, NA = W::NA;
    constexpr int TILE = ST * RPT;
    __shared__ typename W::Lds s;
    const int t = threadIdx.x;
    const int nb = 1 << b2;
    const int shift = 64 - b1 - b2;
    const uint64_t mask = (uint64_t)(nb - 1);
    const int G = gridDim.x, bx = blockIdx.x;
    const int g = (xcd_map && G % 8 == 0) ? (int)((bx % 8) * (G / 8) + bx / 8) : bx;
    const int64_t c0 = nchunks * g / G, c1 = nchunks * (g + 1) / G;
    auto load_tile = [&](int64_t base, int64_t end, uint64_t (&a)[NA][RPT]) {
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int64_t r = base + (int64_t)q * ST + t;
            if (r < end) {
                a[0][q] = in_k0[r];
                if constexpr (BYTES) { a[1][q] = in_k1[r]; a[2][q] = in_meta[r]; }
            }
        }
    };
    auto uniform_chunk = [](const Chunk &x) {
        auto u = [](int64_t v) {
            const uint32_t lo = uniform_u32((uint32_t)v);
            const uint32_t hi = uniform_u32((uint32_t)((uint64_t)v >> 32));
            return (int64_t)(((uint64_t)hi << 32) | lo);
        };
        return Chunk{u(x.start), u(x.end), u(x.hbase), u(x.hstride)};
    };
    if (c0 >= c1) return;                       // (workgroup-uniform: no barrier is skipped by a part)
    uint64_t k[NA][RPT];
    Chunk ch = uniform_chunk(chunks[c0]);
    uint64_t pos = t < nb ? offs[ch.hbase + (int64_t)t * ch.hstride] : 0;
    load_tile(ch.start, ch.end, k);
    WcOut<NA> out;
    out.a[0] = out_k0;
    if constexpr (BYTES) { out.a[1] = out_k1; out.a[2] = out_meta; }
    if (t < nb) wc_start(s, t, pos);
    if (t == 0) s.nlist = 0;
    for (int64_t c = c0; c < c1; ++c) {
        if (c > c0 && t < nb) wc_seek(s, t, pos, out);
        const int64_t cn = c + 1;
        const Chunk chn = cn < c1 ? uniform_chunk(chunks[cn]) : Chunk{0, 0, 0, 0};
        lds_barrier();
        for (int64_t base = ch.start; base < ch.end; base += TILE) {
            uint64_t x[NA][RPT];
            uint32_t have = 0;
            uint32_t bkp[(RPT + 1) / 2] = {};              // byte keys: bucket of record q, 16 bits each
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
#pragma unroll
                for (int a = 0; a < NA; ++a) x[a][q] = k[a][q];
                if (base + (int64_t)q * ST + t < ch.end) {
                    have |= 1u << q;
                    if constexpr (BYTES)
                        bkp[q / 2] |= (uint32_t)((rec_hash(x[0][q], x[1][q], x[2][q]) >> shift) & mask)
                                      << (16 * (q & 1));
                }
            }
            const int64_t nbase = base + TILE;
            const bool last = nbase >= ch.end;                 // wave-uniform
            // the next tile (of this chunk, or the next chunk's first with its
            // offsets) in flight; issued before the placement: 3.10 vs 3.21-3.38 ms
            // per 1e9 fixed-key records after it
            if (last && cn < c1 && t < nb) pos = offs[chn.hbase + (int64_t)t * chn.hstride];
            load_tile(last ? chn.start : nbase, last ? chn.end : ch.end, k);
            wc_tile<ST, RPT>(s, x, have, nb, out, [&](int q) {
                if constexpr (BYTES) return (int)((bkp[q / 2] >> (16 * (q & 1))) & 0xFFFFu);
                else return (int)((x[0][q] >> shift) & mask);
            });
        }
        if (ch.start >= ch.end && cn < c1) {                   // (an empty chunk prefetched nothing)
            if (t < nb) pos = offs[chn.hbase + (int64_t)t * chn.hstride];
            load_tile(chn.start, chn.end, k);
        }
        ch = chn;
    }
    if (t < nb) wc_flush_partial(s, t, out);
}

// ---- level 2 into runs + blocks, no count pass (round 6) ----------------------------
// The exact-offset level 2 above needs a count pass over every record first
// (part_count_recs_*: 7.6 GB read per 1e9-row f64 column) because several
// workgroups fill one level-1 bucket's sub-buckets.  Here ONE workgroup owns a
// whole level-1 bucket, so the cursors of its sub-buckets are its own and no
// prior count is needed.  Sub-bucket j's records fill a contiguous run of R
// blocks (L2B records each) at a fixed place of the bucket's region -- R is
// sized from the bucket's record count S as mean + 4 sigma of a sub-bucket's
// share, so near-unique keys practically never leave their run -- and the
// records past the run go to overflow blocks the workgroup hands out in LDS
// (one LDS atomic per sub-bucket per tile that crosses a block edge).  Every
// sub-bucket's current line is assembled in LDS and written whole (as wc_tile).
// The region holds nb2 * R run blocks and ceil(S / L2B) + 8 overflow blocks,
// so nothing can overflow.  At the end of the bucket the workgroup writes
// every final bucket f = bucket * nb2 + j as a descriptor {records n, first
// entry of its overflow list, run block, run records} and fills the overflow
// lists: record r of f lies in the run
// (r < run records) or at overflow block list[l + (r - run) / L2B].  The
// de-duplication and compaction kernels read that layout (BLK template
// parameter); on the common path it is the contiguous layout of before.
constexpr int L2B = 64;                          // records per block: one wave-wide load
constexpr int DESC_W = 4;                        // u32 words per final-bucket descriptor
template <bool BYTES> struct L2BCfg {
    static constexpr int NA = BYTES ? 3 : 1;
    static constexpr int L = BYTES ? 8 : 16;     // records per line: 64 B (three arrays) / 128 B
    static constexpr int NBM = BYTES ? 512 : MAXB;
    static constexpr int RPT = BYTES ? 4 : WC_RPT;
};
template <int NA, int L, int NBM>
struct L2BLds {
    uint64_t line[NA][NBM][L];                   // sub-bucket j's current line
    uint32_t cur[NBM];                           // records of j so far (bucket-local positions)
    uint32_t cnt[NBM];                           // this tile's records of j
    int32_t nbase[NBM];                          // overflow block k of j allocated in this tile: nbase[j] + k
    uint32_t cb[NBM];                            // overflow block holding position cur[j] (past the run, % L2B != 0)
    uint16_t list[NBM];                          // sub-buckets whose current line this tile completes
    uint32_t nlist, next;
    uint32_t wsum[ST / WAVE];
};
static_assert(sizeof(L2BLds<1, 16, MAXB>) <= 160 * 1024, "level-2 block scatter LDS (fixed keys)");
static_assert(sizeof(L2BLds<3, 8, 512>) <= 160 * 1024, "level-2 block scatter LDS (byte keys)");

// The record index of position p of sub-bucket j (p >= cur[j], within this
// tile's span): in the run (RL records from block RB + j * R) or an overflow
// block (from block OB).
struct L2Geo {
    uint64_t RB, OB;                             // region's first run block, first overflow block
    uint32_t R, RL;                              // run blocks, run records
};
template <int NA, int L, int NBM>
__device__ __forceinline__ uint64_t l2b_rec(const L2BLds<NA, L, NBM> &s, const L2Geo &g, int j, uint32_t p) {
    if (p < g.RL) return (g.RB + (uint64_t)j * g.R) * L2B + p;
    const uint32_t c = s.cur[j], oc = c > g.RL ? c - g.RL : 0u, o = p - g.RL, k = o / L2B;
    const uint32_t b = (k == oc / L2B && (oc % L2B) != 0) ? s.cb[j] : (uint32_t)(s.nbase[j] + (int32_t)k);
    return (g.OB + b) * L2B + o % L2B;
}

// Workgroup g walks the segments segs[soff[g] .. soff[g+1]) (host-built, so
// the buckets are dealt to workgroups by size): segment = records [start, end)
// of bucket `hbase`; hstride = the region's first block (bits 0-31) | bit 32:
// the bucket's first segment | bit 33: its last | run blocks R (bits 40-63).
// A bucket's segments are consecutive (one per bucket on a single rank, one
// per source rank on a sharded owner).  The next segment's first tile is
// loaded while the last tile of the current one is placed, across buckets
// too, so a bucket change costs no exposed memory latency.  bmeta: scratch,
// one u64 per block (sub-bucket << 32 | overflow block index in it); regions
// start at multiples of 8 blocks (no 64-byte line of bmeta is shared by two
// buckets' regions).
template <bool BYTES>
__global__ void __launch_bounds__(ST) part_l2_blocks_kernel(const uint64_t *in_k0, const uint64_t *in_k1,
                                                            const uint64_t *in_meta, const Chunk *segs,
                                                            const int64_t *soff, int b1, int b2, uint64_t *out_k0,
                                                            uint64_t *out_k1, uint64_t *out_meta, uint64_t *bmeta,
                                                            uint32_t *blist, uint32_t *desc) {
    using C = L2BCfg<BYTES>;
    constexpr int NA = C::NA, L = C::L, RPT = C::RPT;
    constexpr int TILE = ST * RPT;
    __shared__ L2BLds<NA, L, C::NBM> s;
    const int t = threadIdx.x;
    const int nb = 1 << b2;
    const int shift = 64 - b1 - b2;
    const uint64_t mask = (uint64_t)(nb - 1);
    const int64_t s0 = soff[blockIdx.x], s1 = soff[blockIdx.x + 1];
    if (s0 >= s1) return;                       // (workgroup-uniform)
    uint64_t *out[NA];
    out[0] = out_k0;
    if constexpr (BYTES) { out[1] = out_k1; out[2] = out_meta; }
    auto load_tile = [&](int64_t base, int64_t end, uint64_t (&a)[NA][RPT]) {
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int64_t r = base + (int64_t)q * ST + t;
            if (r < end) {
                a[0][q] = in_k0[r];
                if constexpr (BYTES) { a[1][q] = in_k1[r]; a[2][q] = in_meta[r]; }
            }
        }
    };
    auto uniform_seg = [](const Chunk &x) {
        auto u = [](int64_t v) {
            const uint32_t lo = uniform_u32((uint32_t)v);
            const uint32_t hi = uniform_u32((uint32_t)((uint64_t)v >> 32));
            return (int64_t)(((uint64_t)hi << 32) | lo);
        };
        return Chunk{u(x.start), u(x.end), u(x.hbase), u(x.hstride)};
    };
    uint64_t k[NA][RPT];
    Chunk sg = uniform_seg(segs[s0]);
    load_tile(sg.start, sg.end, k);
    L2Geo g{0, 0, 1, L2B};
    for (int64_t si = s0; si < s1; ++si) {
        const Chunk sn = si + 1 < s1 ? uniform_seg(segs[si + 1]) : Chunk{0, 0, 0, 0};
        if ((sg.hstride >> 32) & 1) {                          // a bucket's first segment
            g.RB = (uint32_t)sg.hstride;
            g.R = (uint32_t)((uint64_t)sg.hstride >> 40);
            g.RL = g.R * L2B;
            g.OB = g.RB + (uint64_t)nb * g.R;
            for (int j = t; j < nb; j += ST) { s.cur[j] = 0; s.cnt[j] = 0; }
            if (t == 0) { s.nlist = 0; s.next = 0; }
            lds_barrier();
        }
        const int64_t lo = sg.start, hi = sg.end;
        for (int64_t base = lo; base < hi; base += TILE) {
            uint64_t x[NA][RPT];
            uint32_t have = 0;
            uint32_t bkp[(RPT + 1) / 2] = {};            // sub-bucket of record q, 16 bits each
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
#pragma unroll
                for (int a = 0; a < NA; ++a) x[a][q] = k[a][q];
                if (base + (int64_t)q * ST + t < hi) {
                    have |= 1u << q;
                    uint64_t h;
                    if constexpr (BYTES) h = rec_hash(x[0][q], x[1][q], x[2][q]);
                    else h = x[0][q];
                    bkp[q / 2] |= (uint32_t)((h >> shift) & mask) << (16 * (q & 1));
                }
            }
            // the next tile: of this segment, or the next segment's first
            const bool last = base + TILE >= hi;                // wave-uniform
            load_tile(last ? sn.start : base + TILE, last ? sn.end : hi, k);
            auto bk = [&](int q) { return (int)((bkp[q / 2] >> (16 * (q & 1))) & 0xFFFFu); };
            // ranks within this tile's records of each sub-bucket
            uint32_t r[(RPT + 1) / 2] = {};
#pragma unroll
            for (int q = 0; q < RPT; ++q)
                if ((have >> q) & 1u) r[q / 2] |= atomicAdd(&s.cnt[bk(q)], 1u) << (16 * (q & 1));
            lds_barrier();
            // owners: overflow blocks this tile starts (consecutive ids), lines it completes
            for (int j = t; j < nb; j += ST) {
                const uint32_t cc = s.cur[j], e = cc + s.cnt[j];
                if (e > g.RL && e > cc) {
                    const uint32_t oc = cc > g.RL ? cc - g.RL : 0u, oe = e - g.RL;
                    const uint32_t kf = (oc % L2B) ? oc / L2B + 1 : oc / L2B, kl = (oe - 1) / L2B;
                    if (kl >= kf) {
                        const uint32_t nn = kl - kf + 1;
                        const uint32_t b0 = atomicAdd(&s.next, nn);
                        s.nbase[j] = (int32_t)b0 - (int32_t)kf;
                        for (uint32_t u = 0; u < nn; ++u)
                            bmeta[DBG_BLK(g.OB + b0 + u, 9)] = ((uint64_t)j << 32) | (uint64_t)(kf + u);
                    }
                }
                if (e / L != cc / L) s.list[atomicAdd(&s.nlist, 1u)] = (uint16_t)j;
            }
            lds_barrier();
            // records of the current line into LDS, of lines this tile fills
            // entirely straight out, of the new partial line held back
            uint32_t pend = 0;
            uint64_t slots = 0;
#pragma unroll
            for (int q = 0; q < RPT; ++q) {
                if ((have >> q) & 1u) {
                    const int j = bk(q);
                    const uint32_t cc = s.cur[j];
                    const uint32_t p = cc + ((r[q / 2] >> (16 * (q & 1))) & 0xFFFFu), e = cc + s.cnt[j];
                    if (p / L == cc / L) {
#pragma unroll
                        for (int a = 0; a < NA; ++a) s.line[a][j][p % L] = x[a][q];
                    } else if (p / L != e / L) {
                        const uint64_t o = DBG_REC(l2b_rec(s, g, j, p), 8);
#pragma unroll
                        for (int a = 0; a < NA; ++a) out[a][o] = x[a][q];
                    } else {
                        pend |= 1u << q;
                        slots |= (uint64_t)(p % L) << (4 * q);
                    }
                }
            }
            lds_barrier();
            // completed current lines: L lanes per line, one aligned write per array
            const uint32_t nl = s.nlist;
            for (uint32_t i = t / L; i < nl; i += ST / L) {
                const int j = s.list[i], l = t & (L - 1);
                const uint64_t o = DBG_REC(l2b_rec(s, g, j, (s.cur[j] / L) * L + l), 11);
#pragma unroll
                for (int a = 0; a < NA; ++a) out[a][o] = s.line[a][j][l];
            }
            lds_barrier();
#pragma unroll
            for (int q = 0; q < RPT; ++q)
                if ((pend >> q) & 1u) {
                    const int j = bk(q), sl = (int)((slots >> (4 * q)) & 15);
#pragma unroll
                    for (int a = 0; a < NA; ++a) s.line[a][j][sl] = x[a][q];
                }
            for (int j = t; j < nb; j += ST) {
                const uint32_t e = s.cur[j] + s.cnt[j];
                if (e > g.RL && ((e - g.RL) % L2B) != 0) {
                    const uint64_t rec = l2b_rec(s, g, j, e);
                    s.cb[j] = (uint32_t)(rec / L2B - g.OB);
                }
                s.cur[j] = e;
                s.cnt[j] = 0;
            }
            if (t == 0) s.nlist = 0;
            lds_barrier();
        }
        if (lo >= hi) load_tile(sn.start, sn.end, k);        // (an empty segment prefetched nothing)
        if ((sg.hstride >> 33) & 1) {                          // the bucket's last segment: finish it
            const uint32_t bi = (uint32_t)sg.hbase;
            // partial lines: positions below cur (in the run, or the block cb)
            for (int j = t; j < nb; j += ST) {
                const uint32_t cc = s.cur[j];
                for (uint32_t pp = (cc / L) * L; pp < cc; ++pp) {
                    const uint64_t o = DBG_REC(pp < g.RL ? (g.RB + (uint64_t)j * g.R) * L2B + pp
                                                         : (g.OB + s.cb[j]) * L2B + (pp - g.RL) % L2B, 12);
#pragma unroll
                    for (int a = 0; a < NA; ++a) out[a][o] = s.line[a][j][pp % L];
                }
                s.cnt[j] = cc > g.RL ? (cc - g.RL + L2B - 1) / L2B : 0u;       // overflow blocks of j
            }
            lds_barrier();
            block_excl_scan<ST>(s.cnt, (uint32_t *)s.nbase, nb, s.wsum);
            const uint64_t f0 = (uint64_t)bi << b2;
            for (int j = t; j < nb; j += ST) {
                uint32_t *d = desc + (f0 + j) * DESC_W;
                d[0] = s.cur[j];
                d[1] = (uint32_t)g.OB + (uint32_t)s.nbase[j];
                d[2] = (uint32_t)(g.RB + (uint64_t)j * g.R);
                d[3] = g.RL;
            }
            // the overflow lists, in block order within each sub-bucket: bmeta
            // was written by the waves of this workgroup (their stores complete
            // before the barrier) and no line of this region was read before,
            // so the loads miss the L1 and read L2
            __syncthreads();
            const uint32_t nblk = s.next;
            for (uint32_t u = t; u < nblk; u += ST) {
                const uint64_t m = bmeta[DBG_BLK(g.OB + u, 13)];
                const int j = (int)(m >> 32);
                const uint32_t kk = (uint32_t)m;
                blist[DBG_BLK((uint32_t)g.OB + (uint32_t)s.nbase[j] + kk, 10)] = (uint32_t)g.OB + u;
            }
            lds_barrier();                                     // (LDS reused by the next bucket)
        }
        sg = sn;
    }
}

// ---- final buckets: LDS grouping -------------------------------------------------
// Records of a final bucket: contiguous [starts[f], starts[f+1]) (BLK false),
// or laid out by part_l2_blocks_kernel (BLK true): descriptor desc[f] =
// DESC_W u32 words {records n, first overflow-list entry, run block, run
// records}: record i < run records lies in the run, the others in the
// overflow blocks of the list.  Bucket-local index i (lo = 0 for
// blocks).  A kernel loads a bucket's descriptor one bucket ahead, so its
// records cost one memory latency, as with the contiguous layout.
struct BlkArg {
    const uint32_t *desc, *blist;
};
// scalar (constant address space) loads of data no kernel writes while it runs
typedef __attribute__((address_space(4))) const uint32_t cu32;
__device__ __forceinline__ uint32_t sload(const uint32_t *p, uint32_t i) { return ((cu32 *)p)[i]; }

template <bool BLK>
struct Bkt {
    int64_t lo = 0, hi = 0;                      // contiguous: [lo, hi)
    const uint32_t *blist = nullptr;             // blocks: the overflow lists,
    uint4 d = {0, 0, 0, 0};                      //   the descriptor {n, first list entry, run block, run records}
    // the bucket-local range (contiguous: lo, hi; blocks: 0, n)
    __device__ __forceinline__ void range(int64_t &a, int64_t &b) const {
        if constexpr (BLK) {
            a = 0;
            b = (int64_t)d.x;
        } else {
            a = lo;
            b = hi;
        }
    }
    __device__ __forceinline__ uint64_t r0() const { return (uint64_t)d.z * L2B; }
    // record i (i / L2B wave-uniform; no branch: the overflow list entry is
    // read either way, of block 0 for a record in the run)
    __device__ __forceinline__ int64_t at(int64_t i) const {
        if constexpr (BLK) {
            const bool inrun = (uint64_t)i < d.w;
            const uint32_t ob = uniform_u32(inrun ? 0u : (uint32_t)((i - d.w) / L2B));
            const uint32_t b = sload(blist, DBG_BLK(d.y + ob, 5));
            return DBG_REC(inrun ? (int64_t)(r0() + (uint64_t)i) : (int64_t)b * L2B + (i % L2B), 1);
        } else {
            return i;
        }
    }
    // record i, any i per lane
    __device__ __forceinline__ int64_t at_lane(int64_t i) const {
        if constexpr (BLK) {
            if ((uint64_t)i < d.w) return DBG_REC((int64_t)(r0() + (uint64_t)i), 2);
            return DBG_REC((int64_t)blist[DBG_BLK(d.y + (uint32_t)((i - d.w) / L2B), 6)] * L2B + (i % L2B), 2);
        } else {
            return i;
        }
    }
    // the records of a batch of Q wave-wide loads from rb (below hi) lie in
    // the run (the common case: a bucket within its run)
    __device__ __forceinline__ bool inline_batch(int64_t rb, int Q, int64_t hi_) const {
        if constexpr (BLK) return min(hi_, rb + (int64_t)Q * WAVE) <= (int64_t)d.w;
        else return true;
    }
    // (inline_batch) records rb + q * WAVE + lane start here.  Blocks: the
    // pointer is made a scalar value, so the load takes it as its scalar base
    // with the lane offset in one VGPR (left to itself the compiler hoists 16
    // per-q 64-bit lane offsets out of the bucket loop and spills them)
    __device__ __forceinline__ const uint64_t *wave_base_inl(const uint64_t *p, int64_t rb, int q) const {
        if constexpr (BLK) {
            const uint64_t a = (uint64_t)(p + DBG_REC(r0() + rb + (int64_t)q * WAVE, 4));
            return (const uint64_t *)uniform_u64(a);
        } else {
            return p + rb + (int64_t)q * WAVE;
        }
    }
    // records rb + q * WAVE + lane start here (rb a multiple of WAVE and q
    // wave-uniform)
    __device__ __forceinline__ const uint64_t *wave_base(const uint64_t *p, int64_t rb, int q) const {
        if constexpr (BLK) {
            static_assert(L2B == WAVE, "one block per wave-wide load");
            const int64_t i = rb + (int64_t)q * WAVE;
            const bool inrun = (uint64_t)i < d.w;
            const uint32_t ob = inrun ? 0u : (uint32_t)((i - d.w) / L2B);
            const uint32_t b = sload(blist, DBG_BLK(d.y + ob, 7));
            return p + DBG_REC(inrun ? r0() + i : (uint64_t)b * L2B, 3);
        } else {
            return p + rb + (int64_t)q * WAVE;
        }
    }
};
// bucket f's range / descriptor (f wave-uniform: scalar loads, waited for at use)
template <bool BLK>
__device__ __forceinline__ Bkt<BLK> bucket_load(const uint64_t *starts, const BlkArg &ba, int64_t f) {
    Bkt<BLK> k;
    if constexpr (BLK) {
        k.blist = ba.blist;
        const uint32_t o = (uint32_t)f * DESC_W;
        k.d = make_uint4(sload(ba.desc, o), sload(ba.desc, o + 1), sload(ba.desc, o + 2), sload(ba.desc, o + 3));
    } else {
        k.lo = starts[f];
        k.hi = starts[f + 1];
    }
    return k;
}

constexpr int DT = 1024;                // dedup threads per workgroup
constexpr int D_U64 = 8192;             // table slots, fixed keys, distinct only (64 KB: 2 workgroups/CU)
constexpr int D_U64C = 8192;            // fixed keys with counts (96 KB)
constexpr int D_B = 4096;               // byte keys (144 KB)
constexpr int DTU = 512;                // fixed-key dedup threads (2 workgroups of 64 KB per CU)
constexpr int DU_BATCH = 8;             // records per thread loaded before probing

// stats: [1] records whose h == UINT64_MAX (fixed keys; kept outside the table),
// [2] hash collision between different byte strings, [3] table full,
// [4 + (f & 63)] groups.
// Each round loads DU_BATCH records per thread (all loads in flight at once),
// then inserts them: a bucket of <= 8 K records costs one memory latency (the next bucket batch is already in flight).
template <bool COUNTS, bool BLK>
__global__ void __launch_bounds__(DTU) part_dedup_u64_kernel(const uint64_t *in_h, const uint64_t *starts,
                                                            BlkArg ba, int64_t nbuckets, uint64_t *out_key,
                                                            uint64_t *out_cnt, uint32_t *ngroups,
                                                            uint64_t *stats) {
    constexpr int S = COUNTS ? D_U64C : D_U64;
    __shared__ uint64_t s_key[S];
    __shared__ uint32_t s_cnt[COUNTS ? S : 1];
    __shared__ uint32_t s_n, s_special, s_full;
    const int t = threadIdx.x;
    // the first batch of the next bucket is loaded while this one is probed
    int64_t f = blockIdx.x;
    int64_t lo = 0, hi = 0;
    Bkt<BLK> ra, ra_n, ra_n2;                  // buckets f, f + G (records prefetched), f + 2G (range only)
    uint64_t hb[DU_BATCH];
    // per-block totals, flushed once (one global atomic per bucket would serialise
    // hundreds of thousands of device-scope atomics on a few addresses)
    uint64_t acc_groups = 0, acc_special = 0;
    bool acc_full = false;
    auto load_batch = [&](const Bkt<BLK> &rr, int64_t from, int64_t to, uint64_t (&dst)[DU_BATCH]) {
#pragma unroll
        for (int q = 0; q < DU_BATCH; ++q) {
            const int64_t r = from + (int64_t)q * DTU + t;
            dst[q] = r < to ? in_h[rr.at(r)] : EMPTY64;
        }
    };
    if (f < nbuckets) {
        ra = bucket_load<BLK>(starts, ba, f);
        ra.range(lo, hi);
        load_batch(ra, lo, hi, hb);
    }
    if (f + gridDim.x < nbuckets) ra_n2 = bucket_load<BLK>(starts, ba, f + gridDim.x);
    for (; f < nbuckets; f += gridDim.x) {
        const int64_t fn = f + gridDim.x;
        int64_t lo_n = 0, hi_n = 0;
        uint64_t hn[DU_BATCH];
        ra_n = ra_n2;
        if (fn < nbuckets) {
            ra_n.range(lo_n, hi_n);
            load_batch(ra_n, lo_n, hi_n, hn);
        }
        if (fn + gridDim.x < nbuckets) ra_n2 = bucket_load<BLK>(starts, ba, fn + gridDim.x);
        if (lo == hi) {
            if (COUNTS && t == 0) ngroups[f] = 0;
        } else {
            for (int i = t; i < S; i += DTU) {
                s_key[i] = EMPTY64;
                if (COUNTS) s_cnt[i] = 0;
            }
            if (t == 0) { s_n = 0; s_special = 0; s_full = 0; }
            lds_barrier();
            uint32_t fresh = 0, special = 0;
            bool full = false;
            for (int64_t rb = lo; rb < hi; rb += (int64_t)DTU * DU_BATCH) {
                if (rb != lo) load_batch(ra, rb, hi, hb);      // buckets beyond one batch
                // Lane-local queue: each lane walks its own records, so a long probe
                // sequence delays only that lane's later records, not the whole wave.
                const int64_t rem = hi - rb - t;
                int left = rem <= 0 ? 0 : (int)min((int64_t)DU_BATCH, (rem + DTU - 1) / DTU);
                uint64_t h = 0;
                uint32_t pos = 0;
                int probes = 0;
                bool have = false;
                while (true) {
                    if (!have) {
                        if (left == 0) break;
                        h = hb[0];
#pragma unroll
                        for (int k = 0; k < DU_BATCH - 1; ++k) hb[k] = hb[k + 1];
                        --left;
                        if (h == EMPTY64) { ++special; continue; }
                        pos = (uint32_t)h & (S - 1);
                        probes = 0;
                        have = true;
                    }
                    uint64_t cur = s_key[pos];
                    if (cur == EMPTY64) {
                        cur = atomicCAS((unsigned long long *)&s_key[pos], (unsigned long long)EMPTY64,
                                        (unsigned long long)h);
                        if (cur == EMPTY64) ++fresh;
                    }
                    if (cur == EMPTY64 || cur == h) {
                        if (COUNTS) atomicAdd(&s_cnt[pos], 1u);
                        have = false;
                        continue;
                    }
                    pos = (pos + 1) & (S - 1);
                    if (++probes >= S) { full = true; have = false; }
                }
            }
            if (special) atomicAdd(&s_special, special);
            if (full) s_full = 1;
            if (!COUNTS) {
                fresh = (uint32_t)wave_sum_u64(fresh);
                if (lane_id() == 0 && fresh) atomicAdd(&s_n, fresh);
            }
            lds_barrier();
            if constexpr (COUNTS) {
                for (int i = t; i < S; i += DTU) {
                    const uint64_t h = s_key[i];
                    if (h != EMPTY64) {
                        const uint32_t p = atomicAdd(&s_n, 1u);
                        const int64_t o = ra.at_lane(lo + p);
                        out_key[o] = inv_mix64(h);
                        out_cnt[o] = s_cnt[i];
                    }
                }
                lds_barrier();
            }
            if (t == 0) {
                if (COUNTS) ngroups[f] = s_n;
                acc_groups += s_n;
                acc_special += s_special;
                acc_full |= s_full != 0;
            }
            lds_barrier();
        }
        lo = lo_n;
        hi = hi_n;
        ra = ra_n;
#pragma unroll
        for (int q = 0; q < DU_BATCH; ++q) hb[q] = hn[q];
    }
    if (t == 0) {
        if (acc_groups) atomicAdd((unsigned long long *)&stats[4 + (blockIdx.x & 63)], (unsigned long long)acc_groups);
        if (acc_special) atomicAdd((unsigned long long *)&stats[1], (unsigned long long)acc_special);
        if (acc_full) atomicOr((unsigned long long *)&stats[3], 1ull);
    }
}

// Distinct-only fixed keys: one WAVE per final bucket (~1 K records), a
// wave-private 2048-slot LDS table, no workgroup barriers.  DIRECT (near-unique
// columns, chosen from the heavy-key sample): every probe is one CAS -- a new
// key is claimed in one LDS round trip instead of a read and a CAS (f64 N(0,1)
// at 1e9 rows: 4.91 -> 4.37 ms); with repeated keys the read-first form wins
// (zipf int64: 3.51 vs 4.18 ms), as same-slot CASes of a wave serialise where
// reads broadcast.  More than WV_SLOTS/2 distinct keys in one bucket raises
// stats[3] (the caller recounts on the global-table path).  The key whose hash
// is UINT64_MAX never reaches here (the row kernels count it in stats[1]).
constexpr int WV_W = 4;                 // waves per workgroup
constexpr int WV_SLOTS = 2048;          // table slots per wave (16 KB)
constexpr int WV_Q = 20;                // records per lane per batch
constexpr int WV_BATCH = WV_Q * WAVE;   // 1280
template <bool BLK>
__device__ __forceinline__ void wave_load_batch(uint64_t (&hq)[WV_Q], const uint64_t *in_h, const Bkt<BLK> &ra,
                                                int64_t rb, int64_t hi, int lane) {
    // (validity as q * WAVE < rem: a compare with a constant per q, where
    // rb + q * WAVE + lane < hi makes the compiler hoist 64-bit q * WAVE + lane
    // values out of the bucket loop)
    const int64_t rem = hi - rb - lane;
    if (ra.inline_batch(rb, WV_Q, hi)) {
        const uint64_t *base = ra.wave_base_inl(in_h, rb, 0);      // (one scalar base: wave_load_batch16)
#pragma unroll
        for (int q = 0; q < WV_Q; ++q) hq[q] = (int64_t)q * WAVE < rem ? base[q * WAVE + lane] : EMPTY64;
        return;
    }
    const uint64_t *pr = in_h + (BLK ? ra.r0() : 0);               // (as wave_load_batch16)
#pragma unroll
    for (int q = 0; q < WV_Q; ++q) {
        if (!BLK || (uint64_t)(rb + (int64_t)q * WAVE) < (uint64_t)ra.d.w)
            hq[q] = (int64_t)q * WAVE < rem ? pr[rb + (int64_t)q * WAVE + lane] : EMPTY64;
        else
            hq[q] = (int64_t)q * WAVE < rem ? ra.wave_base(in_h, rb, q)[lane] : EMPTY64;
    }
}
// Two-phase wave dedup (round 3).  The round-2 register-queue loop (each lane
// walking its own queue of records, deleted in round 5) paid a dependent LDS round trip plus a shift of
// its 20-record queue (40 VGPR moves) for every probe: PMC showed ~1300 VALU and
// ~700 SALU instructions per ~1 K-record bucket against ~80 LDS instructions
// (profiles/r03h_pmc_group_f64_norm.csv).
//   Phase A: every record of the batch tries its home slot once.  A lane's
//   WV_Q home CASes (reads, then CASes of the empty ones, for repeated keys)
//   do not depend on each other, so they issue back to back and the LDS
//   pipelines them.  A record whose home holds a different key is appended to
//   a wave-private LDS list (ballot + mbcnt; about a quarter of the records at
//   the final load of one half).
//   Phase B: lane l takes list entries l, l + 64, ... and probes linearly from
//   home + 1 (the next entry is read while the current one probes).
// Correctness: a slot is written once, so a deferred key's home still holds the
// other key in phase B and every copy of a key walks the same probe sequence;
// the table is the same linear-probing table as above, filled in another order.
// A batch with more collisions than the list holds re-reads the extra records
// from global memory (L2) in phase B (never seen on the bench columns).
constexpr int WV2_OVF = 448;                    // list entries per wave (3.5 KB; 2 workgroups per CU)
// MODE 0: read, then CAS an empty slot (repeated keys: reads broadcast);
// MODE 1: CAS at once (near-unique keys).  (An atomic-free form -- the table is
// wave-private and lanes run in lockstep, so read / store-if-empty / read-back
// settles same-instruction conflicts, groups = occupied slots at the end -- was
// measured slower: f64 4.51 -> 5.23, f32 2.31 -> 2.69 ms per 1e9 records,
// profiles/r03n_dedup_modes_ab.log.)
template <int MODE, bool LIMIT>
__device__ __forceinline__ uint32_t wave2_probe(uint64_t *T, uint64_t x, bool &full) {
    uint32_t pos = ((uint32_t)x + 1u) & (WV_SLOTS - 1);
    for (int probes = 1;; ++probes) {
        uint64_t cur;
        if (MODE == 1) {
            cur = atomicCAS((unsigned long long *)&T[pos], (unsigned long long)EMPTY64, (unsigned long long)x);
        } else {
            cur = T[pos];
            if (cur == EMPTY64)
                cur = atomicCAS((unsigned long long *)&T[pos], (unsigned long long)EMPTY64, (unsigned long long)x);
        }
        if (cur == EMPTY64) return 1u;
        if (cur == x) return 0u;
        pos = (pos + 1) & (WV_SLOTS - 1);
        if (LIMIT && probes >= WV_SLOTS / 2) { full = true; return 0u; }
    }
}
// one batch (records rb + q * 64 + lane, q < WV_Q, below hi) -> new groups of this lane
template <int MODE, bool LIMIT, bool BLK>
__device__ __forceinline__ uint32_t wave2_insert(uint64_t *T, uint64_t *O, const uint64_t (&hq)[WV_Q],
                                                 const uint64_t *in_h, const Bkt<BLK> &ra, int64_t rb, int64_t hi,
                                                 int lane, bool &full) {
    const int64_t rem = hi - rb - lane;
    const int left = rem <= 0 ? 0 : (int)min((int64_t)WV_Q, (rem + WAVE - 1) / WAVE);
    uint64_t cur[WV_Q];
#pragma unroll
    for (int q = 0; q < WV_Q; ++q) {
        const uint64_t x = hq[q];
        uint64_t c = 0;
        if (q < left) {
            uint64_t *p = &T[(uint32_t)x & (WV_SLOTS - 1)];
            c = MODE == 1 ? (uint64_t)atomicCAS((unsigned long long *)p, (unsigned long long)EMPTY64,
                                                (unsigned long long)x)
                          : *p;
        }
        cur[q] = c;
    }
    if (MODE == 0) {
#pragma unroll
        for (int q = 0; q < WV_Q; ++q)
            if (q < left && cur[q] == EMPTY64)
                cur[q] = atomicCAS((unsigned long long *)&T[(uint32_t)hq[q] & (WV_SLOTS - 1)],
                                   (unsigned long long)EMPTY64, (unsigned long long)hq[q]);
    }
    uint32_t fresh = 0, late = 0, nov = 0;
#pragma unroll
    for (int q = 0; q < WV_Q; ++q) {
        const bool v = q < left;
        fresh += (v && cur[q] == EMPTY64) ? 1u : 0u;
        const bool coll = v && cur[q] != EMPTY64 && cur[q] != hq[q];
        const uint64_t m = __ballot(coll);
        if (m) {                                             // wave-uniform
            const uint32_t slot = nov + (uint32_t)lane_rank(m);
            if (coll) {
                if (slot < (uint32_t)WV2_OVF) O[slot] = hq[q];
                else late |= 1u << q;
            }
            nov += (uint32_t)__popcll(m);
        }
    }
    if (nov == 0) return fresh;
    nov = min(nov, (uint32_t)WV2_OVF);
    __builtin_amdgcn_wave_barrier();
    // phase B: lane-local walk of the list, the next entry read while probing
    uint32_t j = lane;
    uint64_t nx = j < nov ? O[j] : 0;
    while (j < nov) {
        const uint64_t x = nx;
        j += WAVE;
        nx = j < nov ? O[j] : 0;
        fresh += wave2_probe<MODE, LIMIT>(T, x, full);
    }
    while (late) {                                           // list overflow: re-read from L2
        const int q = __builtin_ctz(late);
        late &= late - 1;
        fresh += wave2_probe<MODE, LIMIT>(T, in_h[ra.at_lane(rb + (int64_t)q * WAVE + lane)], full);
    }
    __builtin_amdgcn_wave_barrier();
    return fresh;
}
// ngroups (optional): groups of every bucket (a batch of columns' buckets in
// one launch needs them per column)
template <int MODE, bool BLK>
__global__ void __launch_bounds__(WV_W * WAVE) part_dedup_u64_wave2_kernel(const uint64_t *in_h,
                                                                           const uint64_t *starts, BlkArg ba,
                                                                           int64_t nbuckets, uint32_t *ngroups,
                                                                           uint64_t *stats) {
    __shared__ uint64_t tab[WV_W][WV_SLOTS];
    __shared__ uint64_t lst[WV_W][WV2_OVF];
    const int lane = lane_id(), w = threadIdx.x / WAVE;
    uint64_t *T = tab[w];
    uint64_t *O = lst[w];
    uint64_t groups = 0;
    bool full = false;
    const int64_t stride = (int64_t)gridDim.x * WV_W;
    int64_t f = (int64_t)uniform_u32(blockIdx.x * WV_W + w);
    int64_t lo = 0, hi = 0;
    Bkt<BLK> ra, ra_n, ra_n2;                  // buckets f, f + stride (records prefetched), f + 2 stride
    uint64_t hq[WV_Q];
    if (f < nbuckets) {
        ra = bucket_load<BLK>(starts, ba, f);
        ra.range(lo, hi);
        wave_load_batch<BLK>(hq, in_h, ra, lo, hi, lane);
    }
    if (f + stride < nbuckets) ra_n2 = bucket_load<BLK>(starts, ba, f + stride);
    uint64_t hn[WV_Q];
    auto step = [&](uint64_t (&cur)[WV_Q], uint64_t (&nxt)[WV_Q]) {
        const int64_t fn = f + stride;
        int64_t lo_n = 0, hi_n = 0;
        ra_n = ra_n2;
        if (fn < nbuckets) {
            ra_n.range(lo_n, hi_n);
            wave_load_batch<BLK>(nxt, in_h, ra_n, lo_n, hi_n, lane);
        }
        if (fn + stride < nbuckets) ra_n2 = bucket_load<BLK>(starts, ba, fn + stride);
        if (lo != hi) {
            ulonglong2 *T2 = (ulonglong2 *)T;
#pragma unroll
            for (int k = 0; k < WV_SLOTS / (2 * WAVE); ++k) T2[k * WAVE + lane] = make_ulonglong2(EMPTY64, EMPTY64);
            __builtin_amdgcn_wave_barrier();
            uint32_t fresh = 0;
            if (hi - lo <= WV_BATCH) {
                fresh = wave2_insert<MODE, false, BLK>(T, O, cur, in_h, ra, lo, hi, lane, full);
            } else {
                for (int64_t rb = lo; rb < hi; rb += WV_BATCH) {
                    if (rb != lo) wave_load_batch<BLK>(cur, in_h, ra, rb, hi, lane);
                    fresh += wave2_insert<MODE, true, BLK>(T, O, cur, in_h, ra, rb, hi, lane, full);
                }
            }
            groups += fresh;
            if (ngroups != nullptr) {
                const uint32_t bucket = (uint32_t)wave_sum_u64(fresh);
                if (lane == 0) ngroups[f] = bucket;
            }
            __builtin_amdgcn_wave_barrier();
        } else if (ngroups != nullptr && lane == 0) {
            ngroups[f] = 0;
        }
        lo = lo_n;
        hi = hi_n;
        ra = ra_n;
        f = fn;
    };
    while (f < nbuckets) {
        step(hq, hn);
        if (f >= nbuckets) break;
        step(hn, hq);
    }
    groups = wave_sum_u64(groups);
    const bool any_full = __any(full);
    if (lane == 0) {
        if (groups) atomicAdd((unsigned long long *)&stats[4 + (blockIdx.x & 63)], (unsigned long long)groups);
        if (any_full) atomicOr((unsigned long long *)&stats[3], 1ull);
    }
}

// Half-space wave dedup (round 5).  The two-phase kernel above is latency
// bound at two waves per SIMD (its 16 KB table per wave caps a CU at 8 waves;
// SQ counters: wait 0.51 of wave cycles, VALU busy 0.15).  Here a wave takes
// its bucket's records once into registers and groups them in two passes,
// one per value of hash bit 10, each in a 1024-slot (8 KB) table indexed by
// bits 0..9: the same records, keys and linear probing (a key lives in exactly
// one half, so the halves' group counts add), but 4 KB of list and 8 KB of
// table per wave -- four 4-wave workgroups, 16 waves per CU.  Same-box A/B per
// 1e9-row column (profiles/r05f_dedup_half_ab.log): f64 N(0,1) (direct CAS)
// 4.59 -> 3.94 ms; repeated keys lose (i64 zipf 3.73 -> 4.94, f32 2.55 -> 2.71:
// the second pass's loop overhead outweighs the occupancy), so the read-first
// mode keeps the 2048-slot kernel.
constexpr int WH_SLOTS = 1024;
constexpr int WH_Q = 16;                        // records per lane per batch (1024 per wave)
constexpr int WH_BATCH = WH_Q * WAVE;
constexpr int WH_OVF = 256;                     // collision-list entries per wave (2 KB)
template <bool BLK>
__device__ __forceinline__ void wave_load_batch16(uint64_t (&hq)[WH_Q], const uint64_t *in_h, const Bkt<BLK> &ra,
                                                  int64_t rb, int64_t hi, int lane) {
    // (validity as q * WAVE < rem: a compare with a constant per q, where
    // rb + q * WAVE + lane < hi makes the compiler hoist 64-bit q * WAVE + lane
    // values out of the bucket loop)
    const int64_t rem = hi - rb - lane;
    if (ra.inline_batch(rb, WH_Q, hi)) {
        // the contiguous form's loads from the run's first record (scalar
        // per-q pointers, 16 of them held across the bucket, spilled the block
        // kernel: profiles/r06k_*, r06l_*)
        const uint64_t *p = in_h + (BLK ? ra.r0() : 0);
#pragma unroll
        for (int q = 0; q < WH_Q; ++q) hq[q] = (int64_t)q * WAVE < rem ? p[rb + (int64_t)q * WAVE + lane] : EMPTY64;
        return;
    }
    // a batch reaching past the run: the wave-wide loads still inside it in
    // the contiguous form, the list read only for those in overflow blocks
    // (a column of repeated keys overflows many runs: whole groups of copies
    // land in one sub-bucket)
    const uint64_t *pr = in_h + (BLK ? ra.r0() : 0);
#pragma unroll
    for (int q = 0; q < WH_Q; ++q) {
        if (!BLK || (uint64_t)(rb + (int64_t)q * WAVE) < (uint64_t)ra.d.w)         // (wave-uniform)
            hq[q] = (int64_t)q * WAVE < rem ? pr[rb + (int64_t)q * WAVE + lane] : EMPTY64;
        else
            hq[q] = (int64_t)q * WAVE < rem ? ra.wave_base(in_h, rb, q)[lane] : EMPTY64;
    }
}
template <int MODE, bool LIMIT>
__device__ __forceinline__ uint32_t wh_probe(uint64_t *T, uint64_t x, bool &full) {
    uint32_t pos = ((uint32_t)x + 1u) & (WH_SLOTS - 1);
    for (int probes = 1;; ++probes) {
        uint64_t cur;
        if (MODE == 1) {
            cur = atomicCAS((unsigned long long *)&T[pos], (unsigned long long)EMPTY64, (unsigned long long)x);
        } else {
            cur = T[pos];
            if (cur == EMPTY64)
                cur = atomicCAS((unsigned long long *)&T[pos], (unsigned long long)EMPTY64, (unsigned long long)x);
        }
        if (cur == EMPTY64) return 1u;
        if (cur == x) return 0u;
        pos = (pos + 1) & (WH_SLOTS - 1);
        if (LIMIT && probes >= WH_SLOTS / 2) { full = true; return 0u; }
    }
}
// the records of half `hb` (hash bit 10) among this lane's batch -> new groups
template <int MODE, bool LIMIT, bool BLK>
__device__ __forceinline__ uint32_t wh_insert(uint64_t *T, uint64_t *O, const uint64_t (&hq)[WH_Q],
                                              const uint64_t *in_h, const Bkt<BLK> &ra, int64_t rb, int64_t hi,
                                              int lane, uint32_t hb, bool &full) {
    const int64_t rem = hi - rb - lane;
    const int left = rem <= 0 ? 0 : (int)min((int64_t)WH_Q, (rem + WAVE - 1) / WAVE);
    uint64_t cur[WH_Q];
    uint32_t mine = 0;
#pragma unroll
    for (int q = 0; q < WH_Q; ++q) {
        const uint64_t x = hq[q];
        const bool v = q < left && (((uint32_t)(x >> 10)) & 1u) == hb;
        mine |= (v ? 1u : 0u) << q;
        uint64_t c = 0;
        if (v) {
            uint64_t *p = &T[(uint32_t)x & (WH_SLOTS - 1)];
            c = MODE == 1 ? (uint64_t)atomicCAS((unsigned long long *)p, (unsigned long long)EMPTY64,
                                                (unsigned long long)x)
                          : *p;
        }
        cur[q] = c;
    }
    if (MODE == 0) {
#pragma unroll
        for (int q = 0; q < WH_Q; ++q)
            if (((mine >> q) & 1u) && cur[q] == EMPTY64)
                cur[q] = atomicCAS((unsigned long long *)&T[(uint32_t)hq[q] & (WH_SLOTS - 1)],
                                   (unsigned long long)EMPTY64, (unsigned long long)hq[q]);
    }
    uint32_t fresh = 0, late = 0, nov = 0;
#pragma unroll
    for (int q = 0; q < WH_Q; ++q) {
        const bool v = (mine >> q) & 1u;
        fresh += (v && cur[q] == EMPTY64) ? 1u : 0u;
        const bool coll = v && cur[q] != EMPTY64 && cur[q] != hq[q];
        const uint64_t m = __ballot(coll);
        if (m) {
            const uint32_t slot = nov + (uint32_t)lane_rank(m);
            if (coll) {
                if (slot < (uint32_t)WH_OVF) O[slot] = hq[q];
                else late |= 1u << q;
            }
            nov += (uint32_t)__popcll(m);
        }
    }
    if (nov == 0) return fresh;
    nov = min(nov, (uint32_t)WH_OVF);
    __builtin_amdgcn_wave_barrier();
    uint32_t j = lane;
    uint64_t nx = j < nov ? O[j] : 0;
    while (j < nov) {
        const uint64_t x = nx;
        j += WAVE;
        nx = j < nov ? O[j] : 0;
        fresh += wh_probe<MODE, LIMIT>(T, x, full);
    }
    while (late) {
        const int q = __builtin_ctz(late);
        late &= late - 1;
        fresh += wh_probe<MODE, LIMIT>(T, in_h[ra.at_lane(rb + (int64_t)q * WAVE + lane)], full);
    }
    __builtin_amdgcn_wave_barrier();
    return fresh;
}
template <int MODE, bool BLK>
__global__ void __launch_bounds__(WV_W * WAVE, 4) part_dedup_u64_half_kernel(const uint64_t *in_h,
                                                                             const uint64_t *starts, BlkArg ba,
                                                                             int64_t nbuckets, uint32_t *ngroups,
                                                                             uint64_t *stats) {
    // (no next-bucket prefetch in registers: 16 waves per CU hide the loads)
    __shared__ uint64_t tab[WV_W][WH_SLOTS];
    __shared__ uint64_t lst[WV_W][WH_OVF];
    const int lane = lane_id(), w = threadIdx.x / WAVE;
    uint64_t *T = tab[w];
    uint64_t *O = lst[w];
    uint64_t groups = 0;
    bool full = false;
    const int64_t stride = (int64_t)gridDim.x * WV_W;
    Bkt<BLK> ra_n;                             // the next bucket's range / descriptor, one bucket ahead
    // (blocks: the bucket index in a scalar register, so are the descriptor addresses)
    const int64_t f0 = BLK ? (int64_t)uniform_u32(blockIdx.x * WV_W + w)
                           : (int64_t)blockIdx.x * WV_W + w;
    if (f0 < nbuckets) ra_n = bucket_load<BLK>(starts, ba, f0);
    for (int64_t f = f0; f < nbuckets; f += stride) {
        int64_t lo, hi;
        Bkt<BLK> ra = ra_n;
        ra.range(lo, hi);
        if (f + stride < nbuckets) ra_n = bucket_load<BLK>(starts, ba, f + stride);
        uint32_t fresh = 0;
        if (lo != hi) {
            uint64_t hq[WH_Q];
            wave_load_batch16<BLK>(hq, in_h, ra, lo, hi, lane);
            const bool one = hi - lo <= WH_BATCH;
#pragma unroll 1
            for (uint32_t hb = 0; hb < 2; ++hb) {
                ulonglong2 *T2 = (ulonglong2 *)T;
#pragma unroll
                for (int k = 0; k < WH_SLOTS / (2 * WAVE); ++k) T2[k * WAVE + lane] = make_ulonglong2(EMPTY64, EMPTY64);
                __builtin_amdgcn_wave_barrier();
                if (one) {
                    fresh += wh_insert<MODE, false, BLK>(T, O, hq, in_h, ra, lo, hi, lane, hb, full);
                } else {
                    // (a bucket beyond one batch: its batches are re-read from L2 per half)
#pragma unroll 1
                    for (int64_t rb = lo; rb < hi; rb += WH_BATCH) {
                        if (rb != lo || hb) wave_load_batch16<BLK>(hq, in_h, ra, rb, hi, lane);
                        fresh += wh_insert<MODE, true, BLK>(T, O, hq, in_h, ra, rb, hi, lane, hb, full);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        groups += fresh;
        if (ngroups != nullptr) {
            const uint32_t bucket = (uint32_t)wave_sum_u64(fresh);
            if (lane == 0) ngroups[f] = bucket;
        }
    }
    groups = wave_sum_u64(groups);
    const bool any_full = __any(full);
    if (lane == 0) {
        if (groups) atomicAdd((unsigned long long *)&stats[4 + (blockIdx.x & 63)], (unsigned long long)groups);
        if (any_full) atomicOr((unsigned long long *)&stats[3], 1ull);
    }
}

// Byte keys, in rounds of DT * 4 records held in registers:
//   1. claim a slot per distinct hash (CAS on h)        2. the claimant writes
//   its record into the slot    3. everyone compares bytes and counts.
// Different strings with equal 64-bit hashes raise stats[2] (the caller then
// recounts the column on the exact global-table path).
// One workgroup (144 KB of LDS) per CU: the first round of the workgroup's NEXT
// bucket is loaded before the current bucket is grouped, so the bucket's memory
// latency overlaps the LDS phases instead of idling the CU (the hash is
// recomputed at use, which keeps both rounds within the 128-VGPR budget of a
// 1024-thread workgroup); group slots are handed out one LDS atomic per wave.
constexpr int D_RPT = 4;
struct DRound {
    uint64_t k0[D_RPT], k1[D_RPT], meta[D_RPT];
};
template <bool BLK>
__device__ __forceinline__ void dedup_load_round(DRound &r, const uint64_t *in_k0, const uint64_t *in_k1,
                                                 const uint64_t *in_meta, const Bkt<BLK> &ra, int64_t rb,
                                                 int64_t hi) {
#pragma unroll
    for (int q = 0; q < D_RPT; ++q) {
        const int64_t i = rb + (int64_t)q * DT + threadIdx.x;
        const bool in = i < hi;
        const int64_t a = in ? ra.at(i) : 0;
        r.k0[q] = in ? in_k0[a] : 0ull;
        r.k1[q] = in ? in_k1[a] : 0ull;
        r.meta[q] = in ? in_meta[a] : 0ull;
    }
}
template <bool BLK>
__global__ void __launch_bounds__(DT) part_dedup_bytes_kernel(const uint64_t *in_k0, const uint64_t *in_k1,
                                                              const uint64_t *in_meta, const uint64_t *starts,
                                                              BlkArg ba, int64_t nbuckets, sdp_bytes_column col,
                                                              uint64_t *out_key, uint64_t *out_cnt,
                                                              uint32_t *ngroups, uint64_t *stats) {
    __shared__ uint64_t s_h[D_B];
    __shared__ uint64_t s_k0[D_B];
    __shared__ uint64_t s_k1[D_B];
    __shared__ uint64_t s_meta[D_B];
    __shared__ uint32_t s_cnt[D_B];
    // slots claimed in this bucket, in claim order: the output and the reset of
    // the table walk the bucket's groups only (a zipf bucket of ~2 K records
    // holds a few hundred groups, a mid-cardinality one often a handful), not
    // all D_B slots
    __shared__ uint16_t s_list[D_B];
    __shared__ uint32_t s_n, s_full, s_coll;
    const int t = threadIdx.x;
    uint64_t acc_groups = 0;
    bool acc_full = false, acc_coll = false;
    int64_t f = blockIdx.x, lo = 0, hi = 0;
    Bkt<BLK> ra, ra_n, ra_n2;                  // buckets f, f + G (first round prefetched), f + 2G
    DRound cur, nxt;
    for (int i = t; i < D_B; i += DT) {                 // once: buckets reset only their own slots
        s_h[i] = EMPTY64;
        s_cnt[i] = 0;
    }
    if (f < nbuckets) {
        ra = bucket_load<BLK>(starts, ba, f);
        ra.range(lo, hi);
        dedup_load_round<BLK>(cur, in_k0, in_k1, in_meta, ra, lo, hi);
    }
    if (f + gridDim.x < nbuckets) ra_n2 = bucket_load<BLK>(starts, ba, f + gridDim.x);
    for (; f < nbuckets; f += gridDim.x) {
        const int64_t fn = f + gridDim.x;
        int64_t lo_n = 0, hi_n = 0;
        ra_n = ra_n2;
        if (fn < nbuckets) {                                     // next bucket in flight
            ra_n.range(lo_n, hi_n);
            dedup_load_round<BLK>(nxt, in_k0, in_k1, in_meta, ra_n, lo_n, hi_n);
        }
        if (fn + gridDim.x < nbuckets) ra_n2 = bucket_load<BLK>(starts, ba, fn + gridDim.x);
        if (lo == hi) {
            if (t == 0) ngroups[f] = 0;
        } else {
            if (t == 0) { s_n = 0; s_full = 0; s_coll = 0; }
            lds_barrier();
            for (int64_t rb = lo; rb < hi; rb += (int64_t)DT * D_RPT) {
                if (rb != lo) dedup_load_round<BLK>(cur, in_k0, in_k1, in_meta, ra, rb, hi);   // buckets beyond one round
                int pos[D_RPT];
                uint32_t mine = 0;
#pragma unroll
                for (int q = 0; q < D_RPT; ++q) {
                    pos[q] = -1;
                    const int64_t r = rb + (int64_t)q * DT + t;
                    if (r >= hi) continue;
                    // EMPTY64 is the empty marker: remap that one hash value
                    const uint64_t h = rec_hash(cur.k0[q], cur.k1[q], cur.meta[q]);
                    const uint64_t hk = h == EMPTY64 ? 0xFFFFFFFFFFFFFFFEull : h;
                    uint32_t p = (uint32_t)hk & (D_B - 1);
                    for (int probe = 0; probe < D_B; ++probe) {
                        uint64_t c = s_h[p];
                        if (c == EMPTY64) {
                            c = atomicCAS((unsigned long long *)&s_h[p], (unsigned long long)EMPTY64,
                                          (unsigned long long)hk);
                            if (c == EMPTY64) {
                                pos[q] = (int)p;
                                mine |= 1u << q;
                                s_list[atomicAdd(&s_n, 1u)] = (uint16_t)p;
                                break;
                            }
                        }
                        if (c == hk) { pos[q] = (int)p; break; }
                        p = (p + 1) & (D_B - 1);
                    }
                    if (pos[q] < 0) s_full = 1;
                }
                lds_barrier();
#pragma unroll
                for (int q = 0; q < D_RPT; ++q)
                    if ((mine >> q) & 1u) {
                        s_k0[pos[q]] = cur.k0[q];
                        s_k1[pos[q]] = cur.k1[q];
                        s_meta[pos[q]] = cur.meta[q];
                    }
                lds_barrier();
#pragma unroll
                for (int q = 0; q < D_RPT; ++q) {
                    if (pos[q] < 0) continue;
                    const int p = pos[q];
                    // a meta whose row lies outside the column (records that are
                    // not what the caller described) is a collision: the caller
                    // recounts exactly, and no representative row leaves here
                    const int64_t row = (int64_t)(cur.meta[q] & RMASK40) - 1;
                    if (row < 0 || row >= col.length) s_coll = 1;
                    bool eq;
                    if ((mine >> q) & 1u) {
                        eq = true;
                    } else {
                        const uint64_t om = s_meta[p];
                        eq = (om >> 40) == (cur.meta[q] >> 40) && s_k0[p] == cur.k0[q] && s_k1[p] == cur.k1[q];
                        if (eq && (cur.meta[q] >> 40) > SHORT_MAX)
                            eq = rows_equal_global(col, (int64_t)(om & RMASK40) - 1,
                                                   (int64_t)(cur.meta[q] & RMASK40) - 1);
                    }
                    if (eq) atomicAdd(&s_cnt[p], 1u);
                    else s_coll = 1;
                }
                lds_barrier();
            }
            const uint32_t ng = s_n;
            for (uint32_t i = t; i < ng; i += DT) {                // the bucket's groups, claim order
                const int p = s_list[i];
                const uint64_t hk = s_h[p];
                const int64_t o = ra.at(lo + i);
                out_key[o] = ((hk >> 40) << 40) | (s_meta[p] & RMASK40);
                out_cnt[o] = s_cnt[p];
            }
            lds_barrier();
            for (uint32_t i = t; i < ng; i += DT) {                // reset the claimed slots
                const int p = s_list[i];
                s_h[p] = EMPTY64;
                s_cnt[p] = 0;
            }
            if (t == 0) {
                ngroups[f] = ng;
                acc_groups += ng;
                acc_full |= s_full != 0;
                acc_coll |= s_coll != 0;
            }
            lds_barrier();
        }
        lo = lo_n;
        hi = hi_n;
        ra = ra_n;
        cur = nxt;
    }
    if (t == 0) {
        if (acc_groups) atomicAdd((unsigned long long *)&stats[4 + (blockIdx.x & 63)], (unsigned long long)acc_groups);
        if (acc_full) atomicOr((unsigned long long *)&stats[3], 1ull);
        if (acc_coll) atomicOr((unsigned long long *)&stats[2], 1ull);
    }
}

// groups of bucket f: src[starts[f] .. +ngroups[f]) -> dst[out_off[f] ..)
template <bool BLK>
__global__ void __launch_bounds__(PT) part_compact_kernel(const uint64_t *src_a, const uint64_t *src_b,
                                                          const uint64_t *starts, BlkArg ba, const uint32_t *ngroups,
                                                          const uint64_t *out_off, int64_t nbuckets,
                                                          uint64_t *dst_a, uint64_t *dst_b) {
    for (int64_t f = blockIdx.x; f < nbuckets; f += gridDim.x) {
        int64_t lo, hi;
        Bkt<BLK> ra = bucket_load<BLK>(starts, ba, f);
        ra.range(lo, hi);
        const int64_t o = out_off[f];
        const uint32_t m = ngroups[f];
        for (uint32_t i = threadIdx.x; i < m; i += PT) {
            const int64_t a = ra.at(lo + i);
            dst_a[o + i] = src_a[a];
            if (src_b) dst_b[o + i] = src_b[a];
        }
    }
}

// ---- sample (heavy-key detection) ------------------------------------------------
__device__ __forceinline__ void part_sample_u64_one(const sdp_column &col, int32_t ns, uint64_t *out_h, int j) {
    if (j >= ns) return;
    const int64_t n = col.length;
    const int64_t i = (int64_t)(((double)j + 0.5) * (double)n / (double)ns);
    uint64_t h = EMPTY64;
    if (i < n) {
        bool ok;
        const uint64_t k = fetch_key(col, i, ok);
        if (ok) h = mix64(k);
    }
    out_h[j] = h;
}
__global__ void part_sample_u64_kernel(sdp_column col, int32_t ns, uint64_t *out_h) {
    part_sample_u64_one(col, ns, out_h, blockIdx.x * blockDim.x + threadIdx.x);
}
// every column's sample in one launch: blockIdx.y = column, out_h[c * ns ..)
__global__ void part_sample_u64_batch_kernel(const sdp_column *cols, int32_t ns, uint64_t *out_h) {
    part_sample_u64_one(cols[blockIdx.y], ns, out_h + (int64_t)blockIdx.y * ns, blockIdx.x * blockDim.x + threadIdx.x);
}
__global__ void part_sample_bytes_kernel(sdp_bytes_column col, int32_t ns, uint64_t *out_h, uint64_t *out_k0,
                                         uint64_t *out_k1, uint64_t *out_meta) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ns) return;
    const int64_t n = col.length;
    const int64_t i = (int64_t)(((double)j + 0.5) * (double)n / (double)ns);
    uint64_t h = EMPTY64, k0 = 0, k1 = 0, meta = 0;
    if (i < n && valid_bit(col.d_validity, col.validity_bit_offset, i)) {
        const int64_t o0 = str_off(col, i), len = str_off(col, i + 1) - o0;
        if (len <= SHORT_MAX) {
            k0 = gload8(col.d_data + o0, len);
            k1 = gload8(col.d_data + o0 + 8, len - 8);
            h = bh_short(k0, k1, (uint64_t)len);
        } else {
            h = hash_long_global(col.d_data + o0, len);
            k0 = h;
        }
        meta = ((uint64_t)min((int64_t)LEN_MAX, len) << 40) | (uint64_t)(i + 1);
    }
    out_h[j] = h;
    out_k0[j] = k0;
    out_k1[j] = k1;
    out_meta[j] = meta;
}

// ---- exclusive scan of u32 counts into u64 offsets (n + 1 entries) ---------------
constexpr int SCAN_T = 256;
constexpr int SCAN_PER = 16;
constexpr int SCAN_B = SCAN_T * SCAN_PER;   // 4096 entries per block

__device__ uint64_t block_scan_u64(uint64_t v, uint64_t *s_w, uint64_t &total) {
    // exclusive scan of one value per thread (SCAN_T threads)
    uint64_t x = v;
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, WAVE);
        if (lane >= o) x += y;
    }
    const int w = threadIdx.x / WAVE;
    if (lane == WAVE - 1) s_w[w] = x;
    lds_barrier();
    uint64_t wb = 0, tot = 0;
    for (int k = 0; k < SCAN_T / WAVE; ++k) {
        if (k < w) wb += s_w[k];
        tot += s_w[k];
    }
    lds_barrier();
    total = tot;
    return wb + x - v;
}

__global__ void __launch_bounds__(SCAN_T) scan_reduce_kernel(const uint32_t *in, int64_t n, uint64_t *part) {
    __shared__ uint64_t s_w[SCAN_T / WAVE];
    const int64_t b0 = (int64_t)blockIdx.x * SCAN_B;
    uint64_t sum = 0;
    for (int k = 0; k < SCAN_PER; ++k) {
        const int64_t i = b0 + (int64_t)k * SCAN_T + threadIdx.x;
        if (i < n) sum += in[i];
    }
    uint64_t total;
    block_scan_u64(sum, s_w, total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}
__global__ void __launch_bounds__(SCAN_T) scan_partials_kernel(uint64_t *part, int64_t nparts) {
    __shared__ uint64_t s_w[SCAN_T / WAVE];
    uint64_t carry = 0;
    for (int64_t c0 = 0; c0 < nparts; c0 += SCAN_T) {
        const int64_t i = c0 + threadIdx.x;
        const uint64_t v = i < nparts ? part[i] : 0;
        uint64_t total;
        const uint64_t ex = block_scan_u64(v, s_w, total);
        if (i < nparts) part[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) part[nparts] = carry;
}
__global__ void __launch_bounds__(SCAN_T) scan_apply_kernel(const uint32_t *in, int64_t n, const uint64_t *part,
                                                            uint64_t *out, int64_t nparts) {
    __shared__ uint64_t s_w[SCAN_T / WAVE];
    const int64_t b0 = (int64_t)blockIdx.x * SCAN_B;
    // thread t owns entries [b0 + t*SCAN_PER, +SCAN_PER) (contiguous)
    uint32_t v[SCAN_PER];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        const int64_t i = b0 + (int64_t)threadIdx.x * SCAN_PER + k;
        v[k] = i < n ? in[i] : 0u;
        sum += v[k];
    }
    uint64_t total;
    uint64_t run = part[blockIdx.x] + block_scan_u64(sum, s_w, total);
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        const int64_t i = b0 + (int64_t)threadIdx.x * SCAN_PER + k;
        if (i < n) out[i] = run;
        run += v[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = part[nparts];
}

static int grid_of(int64_t items, int64_t cap) {
    if (items < 1) return 1;
    return (int)(items < cap ? items : cap);
}

// SDP_XCD_MAP=0 turns the XCD-aware workgroup mapping of the scatters off (A/B runs)
static int xcd_map_enabled() {
    const char *e = getenv("SDP_XCD_MAP");
    return (e && e[0] == '0') ? 0 : 1;
}

template <typename T>
static void launch_rows_u64(int phase, int grid, hipStream_t s, const sdp_column &c, HeavyArg hv, int b1, int64_t rpb,
                            uint32_t *hist, const uint64_t *offs, uint64_t *out, uint64_t *hc, uint64_t *st) {
    if (phase == 0)
        hipLaunchKernelGGL((part_count_rows_u64_kernel<T>), dim3(grid), dim3(CT), 0, s, c, hv, b1, rpb, hist, hc, st);
    else
        hipLaunchKernelGGL((part_scatter_rows_u64_kernel<T>), dim3(grid), dim3(ST), 0, s, c, hv, b1, rpb, offs, out,
                           xcd_map_enabled());
}


// ---- 32-bit key spaces: partitions of 4-byte records + LDS bitmaps -------------
// countDistinct (describe.py:143) of a column whose keys fit 32 bits -- float32
// (its order-preserving 32-bit key, NaN one value, -0.0 == 0.0) or an integral
// column with imax - imin < 2^32 (key = v - imin).  h = mix32(key) is a
// bijection of [0, 2^32), so distinct h == distinct keys, and h needs no
// table: the top 6 bits pick one of 64 level-1 buckets, the next 6 one of 64
// level-2 buckets, and the low 20 bits index a 2^20-bit LDS bitmap of the final
// bucket.  Records are the 4-byte h (the 64-bit path moves 8-byte records
// through a count, two scatters and a hash-table de-duplication).  The level-1
// scatter also counts every (level-1 bucket, level-2 bucket) pair of its block
// (64 x 64 LDS counters), so the level-2 offsets need no count pass of their
// own; both scatters write runs of ~256 records per bucket per tile.
constexpr int D32_B2 = 6;
constexpr int D32_NB2 = 1 << D32_B2, D32_NF = D32_NB1 * D32_NB2;
constexpr int D32_BM_WORDS = 1 << (32 - D32_B1 - D32_B2 - 5);   // 2^20 bits -> 32 K words (128 KB)


// One tile of NT * RPT rows as 32-bit hashes (16-byte loads of full tiles)
template <typename T, int NT, int RPT>
struct RowTile32 {
    static constexpr int VPT = Vec16<T>::N;
    static constexpr int NV = RPT / VPT;
    VecIn<T> v[NV];
    bool full;
    __device__ __forceinline__ void load(const sdp_column &c, const VBits &vbm, int64_t base, int64_t end) {
        full = base + (int64_t)NT * RPT <= end && (base % VPT) == 0;
        if (!full) return;
        const Vec16<T> *vals = (const Vec16<T> *)c.d_values;
#pragma unroll
        for (int u = 0; u < NV; ++u) v[u].load(vals, vbm, base / VPT + (int64_t)u * NT + threadIdx.x, INT64_MAX);
    }
    __device__ __forceinline__ void hash(const sdp_column &c, const VBits &vbm, int64_t base, int64_t end, int64_t lo,
                                         uint32_t (&h)[RPT], uint32_t &vmask) const {
        vmask = 0;
        if (full) {
#pragma unroll
            for (int u = 0; u < NV; ++u) {
                const uint32_t vb = v[u].bits(vbm);
#pragma unroll
                for (int e = 0; e < VPT; ++e) {
                    const int q = u * VPT + e;
                    h[q] = mix32(key32_rel<T>(v[u].v.v[e], lo));
                    vmask |= ((vb >> e) & 1u) << q;
                }
            }
            return;
        }
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            // slot q of thread t: the same row as the vector layout above
            const int64_t i = base + ((int64_t)(q / VPT) * NT + threadIdx.x) * VPT + q % VPT;
            h[q] = 0;
            if (i < end) {
                const bool ok = valid_bit(c.d_validity, c.validity_bit_offset, i);
                h[q] = mix32(key32_rel<T>(((const T *)c.d_values)[i], lo));
                vmask |= (uint32_t)ok << q;
            }
        }
    }
};

constexpr int D32_CT = 256, D32_C_RPT = 16;
template <typename T>
__global__ void __launch_bounds__(D32_CT) d32_count_kernel(sdp_column col, int64_t lo, int64_t rows_per_block,
                                                            uint32_t *hist1, uint64_t *stats) {
    __shared__ uint32_t s_h[D32_CT / WAVE][D32_NB1];       // wave-private counters
    const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x, w = t / WAVE;
    for (int i = t; i < (D32_CT / WAVE) * D32_NB1; i += D32_CT) (&s_h[0][0])[i] = 0;
    lds_barrier();
    const int64_t r0 = (int64_t)g * rows_per_block, r1 = min(col.length, r0 + rows_per_block);
    RowTile32<T, D32_CT, D32_C_RPT> tile;
    const VBits vbm = vbits_init(col.d_validity, col.validity_bit_offset, col.d_values);
    uint64_t rows = 0;
    for (int64_t base = r0; base < r1; base += D32_CT * D32_C_RPT) {
        uint32_t h[D32_C_RPT], vmask;
        tile.load(col, vbm, base, r1);
        tile.hash(col, vbm, base, r1, lo, h, vmask);
        rows += __popc(vmask);
#pragma unroll
        for (int q = 0; q < D32_C_RPT; ++q)
            if ((vmask >> q) & 1u) atomicAdd(&s_h[w][h[q] >> (32 - D32_B1)], 1u);
    }
    lds_barrier();
    for (int b = t; b < D32_NB1; b += D32_CT) {
        uint32_t s = 0;
        for (int k = 0; k < D32_CT / WAVE; ++k) s += s_h[k][b];
        hist1[(int64_t)b * G + g] = s;
    }
    block_add_u64(rows, &stats[1]);
}

struct D32ScatterLds {
    uint32_t hist[D32_NB1];
    uint32_t off[D32_NB1];
    uint64_t cur[D32_NB1];
    uint32_t h2[D32_NF];
    uint32_t stage[S_TILE];
    uint32_t wsum[ST / WAVE];
};

// level 1: rows -> 64 buckets of 4-byte records, + the block's (b1, b2) counts
template <typename T>
__global__ void __launch_bounds__(ST) d32_scatter1_kernel(sdp_column col, int64_t lo, int64_t rows_per_block,
                                                           const uint64_t *offs1, uint32_t *out, uint32_t *h2) {
    __shared__ D32ScatterLds s;
    const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
    for (int b = t; b < D32_NB1; b += ST) {
        s.hist[b] = 0;
        s.cur[b] = offs1[(int64_t)b * G + g];
    }
    for (int f = t; f < D32_NF; f += ST) s.h2[f] = 0;
    lds_barrier();
    const int64_t r0 = (int64_t)g * rows_per_block, r1 = min(col.length, r0 + rows_per_block);
    RowTile32<T, ST, S_RPT> tile;
    const VBits vbm = vbits_init(col.d_validity, col.validity_bit_offset, col.d_values);
    if (r0 < r1) tile.load(col, vbm, r0, r1);
    for (int64_t base = r0; base < r1; base += S_TILE) {
        uint32_t h[S_RPT], vmask, rank[S_RPT / 2] = {};  // ranks 16 bits each (< S_TILE): no VGPR spills
        tile.hash(col, vbm, base, r1, lo, h, vmask);
        if (base + S_TILE < r1) tile.load(col, vbm, base + S_TILE, r1);      // next tile in flight
#pragma unroll
        for (int q = 0; q < S_RPT; ++q) {
            if ((vmask >> q) & 1u) {
                rank[q / 2] |= atomicAdd(&s.hist[h[q] >> (32 - D32_B1)], 1u) << (16 * (q & 1));
                atomicAdd(&s.h2[h[q] >> (32 - D32_B1 - D32_B2)], 1u);
            }
        }
        lds_barrier();
        block_excl_scan<ST>(s.hist, s.off, D32_NB1, s.wsum);
#pragma unroll
        for (int q = 0; q < S_RPT; ++q)
            if ((vmask >> q) & 1u)
                s.stage[s.off[h[q] >> (32 - D32_B1)] + ((rank[q / 2] >> (16 * (q & 1))) & 0xFFFFu)] = h[q];
        lds_barrier();
        const uint32_t total = s.off[D32_NB1 - 1] + s.hist[D32_NB1 - 1];
        for (uint32_t j = t; j < total; j += ST) {
            const uint32_t x = s.stage[j];
            const int b = (int)(x >> (32 - D32_B1));
            out[s.cur[b] + (j - s.off[b])] = x;
        }
        lds_barrier();
        for (int b = t; b < D32_NB1; b += ST) {
            s.cur[b] += s.hist[b];
            s.hist[b] = 0;
        }
        lds_barrier();
    }
    // (b1, b2) counts of this block's runs, laid out [b1][b2][block] for the scan
    for (int f = t; f < D32_NF; f += ST) h2[(int64_t)f * G + g] = s.h2[f];
}

// level 2: every level-1 run (bucket b1, block g) -> its 64 sub-buckets
// Workgroup (b1, j) of a GG-per-bucket grid takes the level-1 chunks g0 .. g1 - 1
// of bucket b1 as one record range: consecutive chunks of a bucket are
// adjacent in the input, and so are their runs of every sub-bucket in the
// output, so one cursor per sub-bucket runs across them (one workgroup per
// chunk -- ~1900 records each at 1.25e8 rows -- cost 0.96 ms per launch there
// in fixed per-workgroup work, against 0.27 ms of bytes).
__global__ void __launch_bounds__(ST) d32_scatter2_kernel(const uint32_t *in, const uint64_t *offs1,
                                                           const uint64_t *offs2, int G, int GG, uint32_t *out) {
    __shared__ D32ScatterLds s;
    const int t = threadIdx.x;
    const int b1 = (int)(blockIdx.x / GG), j = (int)(blockIdx.x % GG);
    const int g0 = (int)((int64_t)j * G / GG), g1 = (int)((int64_t)(j + 1) * G / GG);
    const uint64_t start = offs1[(int64_t)b1 * G + g0], end = offs1[(int64_t)b1 * G + g1];
    for (int b = t; b < D32_NB2; b += ST) {
        s.hist[b] = 0;
        s.cur[b] = offs2[((int64_t)b1 * D32_NB2 + b) * G + g0];
    }
    lds_barrier();
    for (uint64_t base = start; base < end; base += S_TILE) {
        uint32_t x[S_RPT], rank[S_RPT];
#pragma unroll
        for (int q = 0; q < S_RPT; ++q) {
            const uint64_t r = base + (uint64_t)q * ST + t;
            x[q] = r < end ? in[r] : 0u;
        }
#pragma unroll
        for (int q = 0; q < S_RPT; ++q)
            if (base + (uint64_t)q * ST + t < end) rank[q] = atomicAdd(&s.hist[(x[q] >> 20) & (D32_NB2 - 1)], 1u);
        lds_barrier();
        block_excl_scan<ST>(s.hist, s.off, D32_NB2, s.wsum);
#pragma unroll
        for (int q = 0; q < S_RPT; ++q)
            if (base + (uint64_t)q * ST + t < end) s.stage[s.off[(x[q] >> 20) & (D32_NB2 - 1)] + rank[q]] = x[q];
        lds_barrier();
        const uint32_t total = s.off[D32_NB2 - 1] + s.hist[D32_NB2 - 1];
        for (uint32_t j = t; j < total; j += ST) {
            const uint32_t y = s.stage[j];
            const int b = (int)((y >> 20) & (D32_NB2 - 1));
            out[s.cur[b] + (j - s.off[b])] = y;
        }
        lds_barrier();
        for (int b = t; b < D32_NB2; b += ST) {
            s.cur[b] += s.hist[b];
            s.hist[b] = 0;
        }
        lds_barrier();
    }
}

// one workgroup per final bucket: its records' low 20 bits into an LDS bitmap,
// then the set bits counted (distinct keys of the bucket)
__global__ void __launch_bounds__(1024) d32_bitmap_kernel(const uint32_t *in, const uint64_t *offs2, int G,
                                                           uint64_t *out) {
    __shared__ uint32_t bm[D32_BM_WORDS];
    const int t = threadIdx.x;
    const int64_t f = blockIdx.x;
    for (int i = t; i < D32_BM_WORDS; i += 1024) bm[i] = 0;
    lds_barrier();
    const uint64_t start = offs2[f * G], end = offs2[(f + 1) * G];
    constexpr int R = 8;                                   // records in flight per thread
    for (uint64_t base = start; base < end; base += (uint64_t)1024 * R) {
        uint32_t x[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const uint64_t r = base + (uint64_t)q * 1024 + t;
            x[q] = r < end ? in[r] : 0u;
        }
#pragma unroll
        for (int q = 0; q < R; ++q)
            if (base + (uint64_t)q * 1024 + t < end) atomicOr(&bm[(x[q] >> 5) & (D32_BM_WORDS - 1)], 1u << (x[q] & 31));
    }
    lds_barrier();
    uint64_t cnt = 0;
    for (int i = t; i < D32_BM_WORDS; i += 1024) cnt += (uint64_t)__popc(bm[i]);
    block_add_u64(cnt, &out[0]);
}

}  // namespace sdp

using namespace sdp;

template <bool BLK>
static int dedup_launch(const sdp_records *in, int32_t is_bytes, const sdp_bytes_column *bcol, const uint64_t *d_starts,
                        const BlkArg &ba, int64_t nbuckets, int32_t with_counts, uint64_t *d_out_key,
                        uint64_t *d_out_cnt, uint32_t *d_ngroups, uint64_t *d_stats, void *stream) {
    if (in == nullptr || nbuckets < 1 || d_stats == nullptr) return set_error(SDP_EINVAL, "part_dedup: args");
    if (((with_counts & 1) || is_bytes) && (d_out_key == nullptr || d_out_cnt == nullptr || d_ngroups == nullptr))
        return set_error(SDP_EINVAL, "part_dedup: group outputs");
    const int grid = grid_of(nbuckets, 256 * 8);
    hipStream_t s = (hipStream_t)stream;
    if (is_bytes) {
        if (bcol == nullptr) return set_error(SDP_EINVAL, "part_dedup: byte keys need the column");
        hipLaunchKernelGGL(part_dedup_bytes_kernel<BLK>, dim3(grid), dim3(DT), 0, s, in->d_k0, in->d_k1, in->d_meta,
                           d_starts, ba, nbuckets, *bcol, d_out_key, d_out_cnt, d_ngroups, d_stats);
    } else if (with_counts & 1) {
        hipLaunchKernelGGL((part_dedup_u64_kernel<true, BLK>), dim3(grid), dim3(DTU), 0, s, in->d_k0, d_starts, ba,
                           nbuckets, d_out_key, d_out_cnt, d_ngroups, d_stats);
    } else if (with_counts & 2) {       // buckets beyond the wave tables (> 2^30 rows per device)
        hipLaunchKernelGGL((part_dedup_u64_kernel<false, BLK>), dim3(grid), dim3(DTU), 0, s, in->d_k0, d_starts, ba,
                           nbuckets, nullptr, nullptr, nullptr, d_stats);
    } else {
        const int wgrid = grid_of((nbuckets + WV_W - 1) / WV_W, 256 * 16);
        if (with_counts & 4)            // near-unique keys: one CAS per probe, half-space tables
            hipLaunchKernelGGL((part_dedup_u64_half_kernel<1, BLK>), dim3(wgrid), dim3(WV_W * WAVE), 0, s, in->d_k0,
                               d_starts, ba, nbuckets, d_ngroups, d_stats);
        else                            // repeated keys: read-first probes, 2048-slot tables
            hipLaunchKernelGGL((part_dedup_u64_wave2_kernel<0, BLK>), dim3(wgrid), dim3(WV_W * WAVE), 0, s, in->d_k0,
                               d_starts, ba, nbuckets, d_ngroups, d_stats);
    }
    return check_launch("part_dedup");
}

extern "C" {

int64_t sdp_part_rows_per_block(int64_t length, int32_t is_bytes) {
    const int64_t tile = is_bytes ? B_S_TILE : ROWS_ALIGN;
    const int64_t tiles = (length + tile - 1) / tile;
    if (tiles < 1) return tile;         // an empty shard: one block of no rows (never a zero divisor)
    const int64_t blocks = tiles < SDP_PART_MAX_GRID ? tiles : SDP_PART_MAX_GRID;
    return ((tiles + blocks - 1) / blocks) * tile;
}

int sdp_part_sample(const sdp_column *col, const sdp_bytes_column *bcol, int32_t n_sample, uint64_t *d_h,
                    const sdp_records *d_out, void *stream) {
    if ((col == nullptr) == (bcol == nullptr) || n_sample < 1) return set_error(SDP_EINVAL, "part_sample: args");
    const int blocks = (n_sample + 255) / 256;
    hipStream_t s = (hipStream_t)stream;
    if (col) {
        hipLaunchKernelGGL(part_sample_u64_kernel, dim3(blocks), dim3(256), 0, s, *col, n_sample, d_h);
    } else {
        if (d_out == nullptr) return set_error(SDP_EINVAL, "part_sample: byte keys need record outputs");
        hipLaunchKernelGGL(part_sample_bytes_kernel, dim3(blocks), dim3(256), 0, s, *bcol, n_sample, d_h, d_out->d_k0,
                           d_out->d_k1, d_out->d_meta);
    }
    return check_launch("part_sample");
}

int sdp_part_sample_batch(const sdp_column *d_cols, int32_t ncols, int32_t n_sample, uint64_t *d_h, void *stream) {
    if (d_cols == nullptr || ncols < 1 || ncols > 65535 || n_sample < 1 || d_h == nullptr)
        return set_error(SDP_EINVAL, "part_sample_batch: args");
    hipLaunchKernelGGL(part_sample_u64_batch_kernel, dim3((n_sample + 255) / 256, ncols), dim3(256), 0,
                       (hipStream_t)stream, d_cols, n_sample, d_h);
    return check_launch("part_sample_batch");
}

int sdp_part_rows_batch(const sdp_rows_task *d_tasks, int32_t ntasks, int32_t dtype, int32_t max_grid, void *stream) {
    if (d_tasks == nullptr || ntasks < 1 || ntasks > 65535 || max_grid < 1 || max_grid > SDP_PART_MAX_GRID)
        return set_error(SDP_EINVAL, "part_rows_batch: args");
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid(max_grid, ntasks);
    const int xm = xcd_map_enabled();
#define ROWS_BATCH(T) hipLaunchKernelGGL((part_scatter_rows_u64_batch_kernel<T>), grid, dim3(ST), 0, s, d_tasks, xm)
    switch (dtype) {
    case SDP_F64: ROWS_BATCH(double); break;
    case SDP_F32: ROWS_BATCH(float); break;
    case SDP_I64: ROWS_BATCH(int64_t); break;
    case SDP_I32: ROWS_BATCH(int32_t); break;
    case SDP_I16: ROWS_BATCH(int16_t); break;
    case SDP_I8: ROWS_BATCH(int8_t); break;
    case SDP_U64: ROWS_BATCH(uint64_t); break;
    case SDP_U32: ROWS_BATCH(uint32_t); break;
    case SDP_U16: ROWS_BATCH(uint16_t); break;
    case SDP_U8: ROWS_BATCH(uint8_t); break;
    default: return set_error(SDP_EINVAL, "part_rows_batch: dtype %d", dtype);
    }
#undef ROWS_BATCH
    return check_launch("part_rows_batch");
}

int sdp_part_rows(const sdp_column *col, const sdp_bytes_column *bcol, const sdp_heavy *heavy, int32_t b1,
                  int32_t phase, uint32_t *d_hist, const uint64_t *d_offsets, const sdp_records *d_out,
                  uint64_t *d_heavy_counts, uint64_t *d_stats, void *stream) {
    if ((col == nullptr) == (bcol == nullptr) || b1 < 0 || b1 > 10 || (phase != 0 && phase != 1))
        return set_error(SDP_EINVAL, "part_rows: args");
    if (phase == 0 && d_hist == nullptr) return set_error(SDP_EINVAL, "part_rows: phase 0 needs d_hist");
    if (phase == 1 && (d_offsets == nullptr || d_out == nullptr || d_out->d_k0 == nullptr))
        return set_error(SDP_EINVAL, "part_rows: phase 1 needs offsets and outputs");
    HeavyArg hv{nullptr, nullptr, nullptr, nullptr, 0};
    if (heavy && heavy->n > 0) {
        if (heavy->n > HEAVY_MAX) return set_error(SDP_EINVAL, "part_rows: %d heavy keys > %d", heavy->n, HEAVY_MAX);
        hv = HeavyArg{heavy->d_h, heavy->d_k0, heavy->d_k1, heavy->d_meta, heavy->n};
        if (bcol && (hv.k0 == nullptr || hv.k1 == nullptr || hv.meta == nullptr))
            return set_error(SDP_EINVAL, "part_rows: byte heavy keys need k0/k1/meta");
    }
    if (phase == 0 && hv.n > 0 && d_heavy_counts == nullptr)
        return set_error(SDP_EINVAL, "part_rows: heavy keys need d_heavy_counts");
    const int64_t n = col ? col->length : bcol->length;
    const int64_t rpb = sdp_part_rows_per_block(n, bcol != nullptr);
    const int grid = (int)((n + rpb - 1) / rpb < 1 ? 1 : (n + rpb - 1) / rpb);
    hipStream_t s = (hipStream_t)stream;
    if (bcol) {
        if (bcol->length >= (int64_t)RMASK40) return set_error(SDP_EINVAL, "part_rows: more than 2^40 rows");
        const int ow = bytes_ow(*bcol);
        if (ow < 0) return set_error(SDP_EINVAL, "part_rows: offset_width must be 4 or 8");
        if (phase == 0)
            hipLaunchKernelGGL(ow == 8 ? part_count_rows_bytes_kernel<8>
                               : ow == 4 ? part_count_rows_bytes_kernel<4> : part_count_rows_bytes_kernel<0>,
                               dim3(grid), dim3(B_CT), 0, s, *bcol, hv, b1, rpb, d_hist, d_heavy_counts, d_stats);
        else
            hipLaunchKernelGGL(ow == 8 ? part_scatter_rows_bytes_kernel<8>
                               : ow == 4 ? part_scatter_rows_bytes_kernel<4> : part_scatter_rows_bytes_kernel<0>,
                               dim3(grid), dim3(B_ST), 0, s, *bcol, hv, b1, rpb, d_offsets, d_out->d_k0, d_out->d_k1,
                               d_out->d_meta);
        return check_launch("part_rows_bytes_kernel");
    }
    uint64_t *out = phase ? d_out->d_k0 : nullptr;
    const sdp_column &c = *col;
    if (c.dtype != SDP_BOOL && !aligned16(c.d_values)) return set_error(SDP_EALIGN, "part_rows: values not 16-byte aligned");
    switch (c.dtype) {
    case SDP_F64: launch_rows_u64<double>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_F32: launch_rows_u64<float>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_I64: launch_rows_u64<int64_t>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_I32: launch_rows_u64<int32_t>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_I16: launch_rows_u64<int16_t>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_I8: launch_rows_u64<int8_t>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_U64: launch_rows_u64<uint64_t>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_U32: launch_rows_u64<uint32_t>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_U16: launch_rows_u64<uint16_t>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_U8: launch_rows_u64<uint8_t>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    case SDP_BOOL: launch_rows_u64<bool>(phase, grid, s, c, hv, b1, rpb, d_hist, d_offsets, out, d_heavy_counts, d_stats); break;
    default: return set_error(SDP_EINVAL, "part_rows: dtype %d", c.dtype);
    }
    return check_launch("part_rows_u64_kernel");
}

// the records kernel's rows per block: whole 4 K-row tiles, at most one
// resident round of workgroups (BR_MINB per CU on 256 CUs)
#ifndef SDP_BREC_GRID
#define SDP_BREC_GRID (BR_MINB * 256)
#endif
static int64_t records_rows_per_block(int64_t length) {
    const int64_t tiles = (length + B_S_TILE - 1) / B_S_TILE;
    if (tiles < 1) return B_S_TILE;
    const int64_t blocks = tiles < SDP_BREC_GRID ? tiles : SDP_BREC_GRID;
    return ((tiles + blocks - 1) / blocks) * B_S_TILE;
}

int64_t sdp_part_records_chunks(int64_t length) {
    const int64_t rpb = records_rows_per_block(length);
    const int64_t grid = (length + rpb - 1) / rpb;
    return (grid < 1 ? 1 : grid) * BR_W;
}

int sdp_part_rows_records(const sdp_bytes_column *bcol, const sdp_heavy *heavy, int32_t b1, uint32_t *d_hist,
                          sdp_chunk *d_chunks, const sdp_records *d_out, uint64_t *d_heavy_counts, uint64_t *d_stats,
                          void *stream) {
    if (bcol == nullptr || b1 < 0 || b1 > 10 || d_hist == nullptr || d_chunks == nullptr || d_stats == nullptr ||
        d_out == nullptr || d_out->d_k0 == nullptr || d_out->d_k1 == nullptr || d_out->d_meta == nullptr)
        return set_error(SDP_EINVAL, "part_rows_records: args");
    if (bcol->length >= (int64_t)RMASK40) return set_error(SDP_EINVAL, "part_rows_records: more than 2^40 rows");
    HeavyArg hv{nullptr, nullptr, nullptr, nullptr, 0};
    if (heavy && heavy->n > 0) {
        if (heavy->n > HEAVY_MAX_REC)
            return set_error(SDP_EINVAL, "part_rows_records: %d heavy keys > %d", heavy->n, HEAVY_MAX_REC);
        hv = HeavyArg{heavy->d_h, heavy->d_k0, heavy->d_k1, heavy->d_meta, heavy->n};
        if (hv.k0 == nullptr || hv.k1 == nullptr || hv.meta == nullptr || d_heavy_counts == nullptr)
            return set_error(SDP_EINVAL, "part_rows_records: byte heavy keys need k0/k1/meta and counts");
    }
    const int64_t n = bcol->length;
    const int64_t rpb = records_rows_per_block(n);
    const int grid = (int)((n + rpb - 1) / rpb < 1 ? 1 : (n + rpb - 1) / rpb);
    const int ow = bytes_ow(*bcol);
    if (ow < 0) return set_error(SDP_EINVAL, "part_records_rows: offset_width must be 4 or 8");
    hipLaunchKernelGGL(ow == 8 ? part_records_rows_bytes_kernel<8>
                       : ow == 4 ? part_records_rows_bytes_kernel<4> : part_records_rows_bytes_kernel<0>,
                       dim3(grid), dim3(BR_T), 0, (hipStream_t)stream, *bcol, hv, b1,
                       rpb, d_hist, (Chunk *)d_chunks, d_out->d_k0, d_out->d_k1, d_out->d_meta, d_heavy_counts,
                       d_stats);
    return check_launch("part_records_rows_bytes_kernel");
}

int sdp_part_recs(const sdp_records *in, int32_t is_bytes, const sdp_chunk *d_chunks, int64_t nchunks, int32_t b1,
                  int32_t b2, int32_t phase, uint32_t *d_hist, const uint64_t *d_offsets, const sdp_records *out,
                  void *stream) {
    if (in == nullptr || d_chunks == nullptr || nchunks < 1 || b2 < 1 || b2 > 10 || b1 < 0 || b1 + b2 > 63 ||
        (phase != 0 && phase != 1))
        return set_error(SDP_EINVAL, "part_recs: args");
    if (phase == 1 && (out == nullptr || d_offsets == nullptr)) return set_error(SDP_EINVAL, "part_recs: outputs");
    const int grid = grid_of(nchunks, 8192);
    hipStream_t s = (hipStream_t)stream;
    const Chunk *ch = (const Chunk *)d_chunks;
    uint64_t *o0 = out ? out->d_k0 : nullptr, *o1 = out ? out->d_k1 : nullptr, *o2 = out ? out->d_meta : nullptr;
    if (is_bytes) {
        if (phase == 0)
            hipLaunchKernelGGL(part_count_recs_kernel<true>, dim3(grid), dim3(CT), 0, s, in->d_k0, in->d_k1, in->d_meta,
                               ch, nchunks, b1, b2, d_hist);
        else if ((1 << b2) <= WcRecs<true>::NBM)       // (more buckets: the tile-sorted scatter)
            hipLaunchKernelGGL(part_scatter_recs_wc_kernel<true>, dim3(grid_of(nchunks, 256)), dim3(ST), 0, s,
                               in->d_k0, in->d_k1, in->d_meta, ch, nchunks, b1, b2, d_offsets, o0, o1, o2,
                               xcd_map_enabled());
        else
            hipLaunchKernelGGL(part_scatter_recs_kernel<true>, dim3(grid), dim3(ST), 0, s, in->d_k0, in->d_k1,
                               in->d_meta, ch, nchunks, b1, b2, d_offsets, o0, o1, o2, xcd_map_enabled());
    } else {
        if (phase == 0)
            hipLaunchKernelGGL(part_count_recs_u64_kernel, dim3(grid), dim3(CT), 0, s, in->d_k0, ch, nchunks, b1, b2,
                               d_hist);
        else                             // one resident workgroup per CU, a contiguous range of chunks each
            hipLaunchKernelGGL(part_scatter_recs_wc_kernel<false>, dim3(grid_of(nchunks, 256)), dim3(ST), 0, s,
                               in->d_k0, nullptr, nullptr, ch, nchunks, b1, b2, d_offsets, o0, nullptr, nullptr,
                               xcd_map_enabled());
    }
    return check_launch("part_recs_kernel");
}

int64_t sdp_part_bucket_target(int32_t is_bytes, int32_t with_counts) {
    return is_bytes ? D_B / 2 : (with_counts ? D_U64C / 2 : WV_SLOTS / 2);
}

int sdp_part_dedup(const sdp_records *in, int32_t is_bytes, const sdp_bytes_column *bcol, const uint64_t *d_starts,
                   int64_t nbuckets, int32_t with_counts, uint64_t *d_out_key, uint64_t *d_out_cnt,
                   uint32_t *d_ngroups, uint64_t *d_stats, void *stream) {
    if (d_starts == nullptr) return set_error(SDP_EINVAL, "part_dedup: args");
    return dedup_launch<false>(in, is_bytes, bcol, d_starts, BlkArg{nullptr, nullptr}, nbuckets, with_counts,
                               d_out_key, d_out_cnt, d_ngroups, d_stats, stream);
}

int sdp_part_dedup_blocks(const sdp_records *in, int32_t is_bytes, const sdp_bytes_column *bcol, const sdp_blocks *blk,
                          int64_t nbuckets, int32_t with_counts, uint64_t *d_out_key, uint64_t *d_out_cnt,
                          uint32_t *d_ngroups, uint64_t *d_stats, void *stream) {
    if (blk == nullptr || blk->d_desc == nullptr || blk->d_list == nullptr)
        return set_error(SDP_EINVAL, "part_dedup_blocks: blocks");
    return dedup_launch<true>(in, is_bytes, bcol, nullptr, BlkArg{blk->d_desc, blk->d_list}, nbuckets,
                              with_counts, d_out_key, d_out_cnt, d_ngroups, d_stats, stream);
}

int sdp_part_l2_blocks(const sdp_records *in, int32_t is_bytes, const sdp_chunk *d_segs, const int64_t *d_soff,
                       int32_t nwg, int32_t b1, int32_t b2, const sdp_records *out, uint64_t *d_bmeta,
                       const sdp_blocks *blk, void *stream) {
    if (in == nullptr || out == nullptr || d_segs == nullptr || d_soff == nullptr || d_bmeta == nullptr ||
        blk == nullptr || blk->d_desc == nullptr || blk->d_list == nullptr ||
        nwg < 1 || nwg > 65535 || b1 < 0 || b2 < 1 || b1 + b2 > 63)
        return set_error(SDP_EINVAL, "part_l2_blocks: args");
    if ((1 << b2) > (is_bytes ? L2BCfg<true>::NBM : L2BCfg<false>::NBM))
        return set_error(SDP_EINVAL, "part_l2_blocks: %d sub-buckets", 1 << b2);
    if (is_bytes && (in->d_k1 == nullptr || in->d_meta == nullptr || out->d_k1 == nullptr || out->d_meta == nullptr))
        return set_error(SDP_EINVAL, "part_l2_blocks: byte records need k1/meta");
    hipStream_t s = (hipStream_t)stream;
    const Chunk *sg = (const Chunk *)d_segs;
    if (is_bytes)
        hipLaunchKernelGGL(part_l2_blocks_kernel<true>, dim3(nwg), dim3(ST), 0, s, in->d_k0, in->d_k1, in->d_meta,
                           sg, d_soff, b1, b2, out->d_k0, out->d_k1, out->d_meta, d_bmeta, blk->d_list, blk->d_desc);
    else
        hipLaunchKernelGGL(part_l2_blocks_kernel<false>, dim3(nwg), dim3(ST), 0, s, in->d_k0, nullptr, nullptr, sg,
                           d_soff, b1, b2, out->d_k0, nullptr, nullptr, d_bmeta, blk->d_list, blk->d_desc);
    return check_launch("part_l2_blocks_kernel");
}

int sdp_part_compact(const uint64_t *d_src_a, const uint64_t *d_src_b, const uint64_t *d_starts,
                     const uint32_t *d_ngroups, const uint64_t *d_out_offsets, int64_t nbuckets, uint64_t *d_dst_a,
                     uint64_t *d_dst_b, void *stream) {
    if (d_src_a == nullptr || d_dst_a == nullptr || nbuckets < 1 || (d_src_b != nullptr) != (d_dst_b != nullptr))
        return set_error(SDP_EINVAL, "part_compact: args");
    hipLaunchKernelGGL(part_compact_kernel<false>, dim3(grid_of(nbuckets, 8192)), dim3(PT), 0, (hipStream_t)stream,
                       d_src_a, d_src_b, d_starts, BlkArg{nullptr, nullptr}, d_ngroups, d_out_offsets,
                       nbuckets, d_dst_a, d_dst_b);
    return check_launch("part_compact_kernel");
}

int sdp_part_compact_blocks(const uint64_t *d_src_a, const uint64_t *d_src_b, const sdp_blocks *blk,
                            const uint32_t *d_ngroups, const uint64_t *d_out_offsets, int64_t nbuckets,
                            uint64_t *d_dst_a, uint64_t *d_dst_b, void *stream) {
    if (d_src_a == nullptr || d_dst_a == nullptr || nbuckets < 1 || (d_src_b != nullptr) != (d_dst_b != nullptr) ||
        blk == nullptr || blk->d_desc == nullptr || blk->d_list == nullptr)
        return set_error(SDP_EINVAL, "part_compact_blocks: args");
    hipLaunchKernelGGL(part_compact_kernel<true>, dim3(grid_of(nbuckets, 8192)), dim3(PT), 0, (hipStream_t)stream,
                       d_src_a, d_src_b, nullptr, BlkArg{blk->d_desc, blk->d_list}, d_ngroups,
                       d_out_offsets, nbuckets, d_dst_a, d_dst_b);
    return check_launch("part_compact_kernel");
}

// (SDP_DEBUG_BOUNDS builds) set the capacities the checks use (cap_rec > 0),
// then read and optionally clear the flags
int sdp_debug_bounds(uint64_t cap_rec, uint64_t cap_blk, uint64_t *flags_out, int32_t reset) {
#ifdef SDP_DEBUG_BOUNDS
    if (cap_rec) {
        unsigned long long a = cap_rec, b = cap_blk;
        hipMemcpyToSymbol(HIP_SYMBOL(dbg_cap_rec), &a, 8);
        hipMemcpyToSymbol(HIP_SYMBOL(dbg_cap_blk), &b, 8);
    }
    unsigned long long f = 0;
    hipMemcpyFromSymbol(&f, HIP_SYMBOL(dbg_flags), 8);
    if (flags_out) *flags_out = f;
    if (reset) {
        f = 0;
        hipMemcpyToSymbol(HIP_SYMBOL(dbg_flags), &f, 8);
    }
    return SDP_OK;
#else
    (void)cap_rec; (void)cap_blk; (void)flags_out; (void)reset;
    return set_error(SDP_EINVAL, "sdp_debug_bounds: not an SDP_DEBUG_BOUNDS build");
#endif
}

int64_t sdp_scan_workspace_bytes(int64_t n) {
    return (int64_t)(((n + SCAN_B - 1) / SCAN_B) + 1) * 8;
}

int sdp_scan_u32(const uint32_t *d_in, int64_t n, uint64_t *d_out, void *d_work, int64_t work_bytes, void *stream) {
    if (d_in == nullptr || d_out == nullptr || n < 1) return set_error(SDP_EINVAL, "scan_u32: args");
    if (work_bytes < sdp_scan_workspace_bytes(n)) return set_error(SDP_ECAP, "scan_u32: workspace too small");
    const int64_t nparts = (n + SCAN_B - 1) / SCAN_B;
    if (nparts > 0x7FFFFFFF) return set_error(SDP_EINVAL, "scan_u32: too long");
    uint64_t *part = (uint64_t *)d_work;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nparts), dim3(SCAN_T), 0, s, d_in, n, part);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(SCAN_T), 0, s, part, nparts);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nparts), dim3(SCAN_T), 0, s, d_in, n, part, d_out, nparts);
    return check_launch("scan_u32");
}

}  // extern "C"

// ---- countDistinct of 32-bit key spaces (d32_* kernels) --------------------------
struct D32Layout {
    int G;
    int64_t rpb;
    uint32_t *hist1, *h2, *recs1, *recs2;
    uint64_t *offs1, *offs2;
    void *scan1, *scan2;
    int64_t scan1_bytes, scan2_bytes, total;
};
static int64_t d32_align(int64_t x) { return (x + 255) / 256 * 256; }
static D32Layout d32_layout(void *d_work, int64_t length) {
    D32Layout L;
    L.rpb = sdp_part_rows_per_block(length, 0);
    L.G = (int)std::max<int64_t>(1, (length + L.rpb - 1) / L.rpb);
    const int64_t n1 = (int64_t)D32_NB1 * L.G, n2 = (int64_t)D32_NF * L.G;
    L.scan1_bytes = sdp_scan_workspace_bytes(n1);
    L.scan2_bytes = sdp_scan_workspace_bytes(n2);
    char *w = (char *)d_work;
    int64_t o = 0;
    auto take = [&](int64_t bytes) { char *p = w ? w + o : nullptr; o += d32_align(bytes); return p; };
    L.hist1 = (uint32_t *)take(4 * n1);
    L.offs1 = (uint64_t *)take(8 * (n1 + 1));
    L.scan1 = take(L.scan1_bytes);
    L.h2 = (uint32_t *)take(4 * n2);
    L.offs2 = (uint64_t *)take(8 * (n2 + 1));
    L.scan2 = take(L.scan2_bytes);
    L.recs1 = (uint32_t *)take(4 * std::max<int64_t>(length, 1));
    L.recs2 = (uint32_t *)take(4 * std::max<int64_t>(length, 1));
    L.total = o;
    return L;
}

int64_t sdp_distinct32_workspace_bytes(int64_t length) {
    if (length < 0) return -1;
    return d32_layout(nullptr, length).total;
}

int sdp_distinct32(const sdp_column *col, int64_t lo, const uint32_t *d_hist1, void *d_work, int64_t work_bytes,
                   uint64_t *d_out, void *stream) {
    if (col == nullptr || d_out == nullptr || d_work == nullptr || col->length < 0)
        return set_error(SDP_EINVAL, "distinct32: args");
    if (col->length > 0 && col->d_values == nullptr) return set_error(SDP_EINVAL, "distinct32: null values");
    if (!aligned16(col->d_values)) return set_error(SDP_EALIGN, "distinct32: values not 16-byte aligned");
    const D32Layout L = d32_layout(d_work, col->length);
    if (work_bytes < L.total) return set_error(SDP_ECAP, "distinct32: workspace %lld < %lld", (long long)work_bytes,
                                               (long long)L.total);
    if (col->length == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const int G = L.G;
    int rc;
    const uint32_t *h1 = d_hist1 ? d_hist1 : L.hist1;
#define D32_LAUNCH_ROWS(T)                                                                                   \
    if (!d_hist1) {                                                                                          \
        hipLaunchKernelGGL(d32_count_kernel<T>, dim3(G), dim3(D32_CT), 0, s, *col, lo, L.rpb, L.hist1, d_out); \
        if ((rc = check_launch("d32_count_kernel"))) return rc;                                              \
    }                                                                                                        \
    if ((rc = sdp_scan_u32(h1, (int64_t)D32_NB1 * G, L.offs1, L.scan1, L.scan1_bytes, stream))) return rc;  \
    hipLaunchKernelGGL(d32_scatter1_kernel<T>, dim3(G), dim3(ST), 0, s, *col, lo, L.rpb, L.offs1, L.recs1, L.h2); \
    if ((rc = check_launch("d32_scatter1_kernel"))) return rc;
    switch (col->dtype) {
    case SDP_F32: { D32_LAUNCH_ROWS(float) } break;
    case SDP_I32: { D32_LAUNCH_ROWS(int32_t) } break;
    case SDP_U32: { D32_LAUNCH_ROWS(uint32_t) } break;
    case SDP_I64: { D32_LAUNCH_ROWS(int64_t) } break;
    case SDP_U64: { D32_LAUNCH_ROWS(uint64_t) } break;
    case SDP_I16: { D32_LAUNCH_ROWS(int16_t) } break;
    case SDP_U16: { D32_LAUNCH_ROWS(uint16_t) } break;
    case SDP_I8: { D32_LAUNCH_ROWS(int8_t) } break;
    case SDP_U8: { D32_LAUNCH_ROWS(uint8_t) } break;
    default: return set_error(SDP_EINVAL, "distinct32: dtype %d", col->dtype);
    }
#undef D32_LAUNCH_ROWS
    if ((rc = sdp_scan_u32(L.h2, (int64_t)D32_NF * G, L.offs2, L.scan2, L.scan2_bytes, stream))) return rc;
    // ~64 K records per workgroup (the column's rows spread evenly over the 64 buckets)
    const int GG = (int)std::max<int64_t>(1, std::min<int64_t>(G, col->length / ((int64_t)D32_NB1 * 65536)));
    hipLaunchKernelGGL(d32_scatter2_kernel, dim3(D32_NB1 * GG), dim3(ST), 0, s, L.recs1, L.offs1, L.offs2, G, GG,
                       L.recs2);
    if ((rc = check_launch("d32_scatter2_kernel"))) return rc;
    hipLaunchKernelGGL(d32_bitmap_kernel, dim3(D32_NF), dim3(1024), 0, s, L.recs2, L.offs2, G, d_out);
    return check_launch("d32_bitmap_kernel");
}
