// sdp_api.cpp -- the coarse C-ABI entries of SURVEY.md §8(b): one call per
// reference operation group, each a C++ orchestrator over libsdp's kernels so
// that a host in any language computes a statistic from include/sdp.h alone.
//
//   sdp_minmax_int          describe.py:233 (date / timestamp min, max)
//   sdp_quantiles           describe.py:203-208 (five percentile jobs)
//   sdp_hash_distinct_count describe.py:143 (countDistinct)
//   sdp_value_counts_topk   describe.py:251-263 (groupBy / orderBy / limit(50))
//   sdp_gram_f64            utils.py:20-36 (na.drop(how='any') + C^2 corr jobs)
//
// The Python engine (spark_df_profiling/engine.py) drives the same kernels
// with whole-table batching; these entries serve one column per call and keep
// to the rules in sdp.h: one caller-owned workspace carved by a bump arena,
// one stream, SYNC entries read small results back between stages.
#include <algorithm>
#include <cmath>
#include <vector>

#include "sdp_common.h"
#include "sdp_internal.h"

namespace sdp {
namespace {

constexpr int64_t ARENA_ALIGN = 256;
// the grouping policy is sdp.h's, shared with the Python engine
constexpr int PART_SAMPLE = SDP_PART_SAMPLE;
constexpr int PART_SAMPLE_BYTES = SDP_PART_SAMPLE_BYTES;
constexpr int HEAVY_MIN = SDP_HEAVY_MIN;
constexpr int64_t PART_CHUNK = SDP_PART_CHUNK;
constexpr int64_t GSORT_MAX = SDP_GSORT_MAX;
constexpr int64_t SMALL_BYTES = 64ll << 20; // headroom for tables, histograms, chunk lists

struct Arena {
    char *base;
    int64_t cap, used = 0;
    bool full = false;
    Arena(void *b, int64_t c) : base((char *)b), cap(c) {}
    template <typename T>
    T *take(int64_t n) {
        const int64_t bytes = ((std::max<int64_t>(n, 1) * (int64_t)sizeof(T)) + ARENA_ALIGN - 1) / ARENA_ALIGN * ARENA_ALIGN;
        if (used + bytes > cap) {
            full = true;
            return nullptr;
        }
        T *p = (T *)(base + used);
        used += bytes;
        return p;
    }
};

#define SDP_TRY(expr)                 \
    do {                              \
        const int rc_ = (expr);       \
        if (rc_) return rc_;          \
    } while (0)
#define SDP_NEED(ptr_, arena_)                                                              \
    do {                                                                                    \
        if ((ptr_) == nullptr)                                                              \
            return set_error(SDP_ECAP, "workspace too small (%lld bytes)", (long long)(arena_).cap); \
    } while (0)

int hip_rc(hipError_t e, const char *what) {
    return e == hipSuccess ? 0 : set_error(SDP_EHIP, "%s: %s", what, hipGetErrorString(e));
}
// device -> host, then wait (SYNC entries only)
int d2h(void *h, const void *d, size_t bytes, hipStream_t s) {
    if (bytes == 0) return 0;
    SDP_TRY(hip_rc(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s), "d2h"));
    return hip_rc(hipStreamSynchronize(s), "d2h sync");
}
// host -> device; waits too, so the host buffer may go out of scope
int h2d(void *d, const void *h, size_t bytes, hipStream_t s) {
    if (bytes == 0) return 0;
    SDP_TRY(hip_rc(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s), "h2d"));
    return hip_rc(hipStreamSynchronize(s), "h2d sync");
}
int zero(void *d, size_t bytes, hipStream_t s) { return hip_rc(hipMemsetAsync(d, 0, bytes, s), "memset"); }

// integral dtypes the numeric kernels (pass 1, keys, bitmaps) take
bool integral(int dt) {
    return dt == SDP_I8 || dt == SDP_I16 || dt == SDP_I32 || dt == SDP_I64 || dt == SDP_U8 || dt == SDP_U16 ||
           dt == SDP_U32;
}
bool floating(int dt) { return dt == SDP_F32 || dt == SDP_F64; }
bool numeric(int dt) { return integral(dt) || floating(dt); }
// fixed-width dtypes the grouping kernels take (adds u64 and bit-packed bools)
bool groupable(int dt) { return numeric(dt) || dt == SDP_U64 || dt == SDP_BOOL; }


int64_t next_pow2_cap(int64_t x) {          // engine._next_pow2: at least 1024 slots
    int64_t c = 1024;
    while (c < x) c <<= 1;
    return c;
}

// ---- small device helpers ------------------------------------------------------
__global__ void minmax_finish_kernel(const sdp_pass1_result *r, sdp_minmax_result *out) {
    out->count = r->count;
    out->imin = r->imin;
    out->imax = r->imax;
    out->dmin = r->dmin;
    out->dmax = r->dmax;
}

struct QProbs {
    double p[SDP_QUANTILES_MAX];
    int n;
};
// 0-based ranks of every probability from the device-side count n (engine.
// _queue_column_selects): integral -> floor / ceil of (n - 1) p; float -> the
// 1-based rank ceil(p n) with Spark's clamps, minus one
__global__ void quantile_ranks_kernel(const uint64_t *d_n, QProbs q, int is_int, int64_t *d_k) {
    const int j = threadIdx.x;
    if (j >= q.n) return;
    const int64_t n = (int64_t)*d_n;
    const double p = q.p[j];
    int64_t lo = 0, hi = 0;
    if (n > 0) {
        if (is_int) {
            const double pos = (double)(n - 1) * p;
            lo = (int64_t)floor(pos);
            hi = (int64_t)ceil(pos);
        } else {
            int64_t r;
            if (p <= 1e-4) r = 1;
            else if (p >= 1.0 - 1e-4) r = n;
            else r = std::min<int64_t>(std::max<int64_t>((int64_t)ceil(p * (double)n), 1), n);
            lo = hi = r - 1;
        }
    }
    d_k[2 * j] = lo;
    d_k[2 * j + 1] = hi;
}
// values from the selected keys (engine._finish_column_quantiles)
__global__ void quantile_values_kernel(const uint64_t *d_n, const uint64_t *res, QProbs q, int is_int, double *out) {
    const int j = threadIdx.x;
    if (j >= q.n) return;
    const int64_t n = (int64_t)*d_n;
    if (n <= 0) {
        out[j] = __builtin_nan("");
        return;
    }
    if (!is_int) {
        out[j] = key_f64(res[2 * j]);
        return;
    }
    const double pos = (double)(n - 1) * q.p[j];
    const int64_t lo = (int64_t)floor(pos), hi = (int64_t)ceil(pos);
    const int64_t lk = key_i64(res[2 * j]), hk = key_i64(res[2 * j + 1]);
    if (lo == hi || lk == hk) out[j] = (double)lk;
    else out[j] = ((double)hi - pos) * (double)lk + (pos - (double)lo) * (double)hk;   // Spark Percentile (A.4)
}

// dst[i] = src[i * stride] (i < n), dst[n] = src[last]: the level-1 bucket
// starts out of the scanned per-(bucket, block) counts
__global__ void gather_strided_kernel(const uint64_t *src, int64_t stride, int64_t n, int64_t last, uint64_t *dst) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = i < n ? src[i * stride] : src[last];
}
__global__ void gather_idx_kernel(const uint64_t *src, const int64_t *idx, int64_t n, uint64_t *dst) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[idx[i]];
}
// {n, sel[0..t), counts[sel], slots[sel]} with entries past n masked to slot 0
__global__ void take_pack_kernel(const uint64_t *sel, const uint64_t *d_n, int64_t t, const uint64_t *slots,
                                 const uint64_t *counts, uint64_t *out) {
    const uint64_t n = *d_n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t ix = (uint64_t)i < n ? sel[i] : 0ull;
        out[1 + i] = ix;
        out[1 + t + i] = counts[ix];
        out[1 + 2 * t + i] = slots[ix];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = n;
}
// each column's shift: the median of its sorted key sample (valid keys sort
// below UINT64_MAX); 0 when the sample holds no valid key
__global__ void sample_median_kernel(const uint64_t *samples, int ns, const int32_t *is_float, double *shift) {
    const int c = blockIdx.x;
    const uint64_t *a = samples + (int64_t)c * ns;
    if (threadIdx.x != 0) return;
    int lo = 0, hi = ns;                       // first EMPTY64
    while (lo < hi) {
        const int m = (lo + hi) / 2;
        if (a[m] == EMPTY64) hi = m; else lo = m + 1;
    }
    if (lo == 0) {
        shift[c] = 0.0;
        return;
    }
    const uint64_t k = a[lo / 2];
    shift[c] = is_float[c] ? key_f64(k) : (double)key_i64(k);
}
// rho from the shifted Gram (utils.corr_from_gram: C = G - s s^T / n)
__global__ void pearson_kernel(const double *G, const double *s, const double *d_n, int nc, double *rho) {
    const double n = *d_n;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)nc * nc;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / nc), j = (int)(e % nc);
        if (n <= 0) {
            rho[e] = __builtin_nan("");
            continue;
        }
        const double cij = G[e] - s[i] * s[j] / n;
        const double cii = G[(int64_t)i * nc + i] - s[i] * s[i] / n;
        const double cjj = G[(int64_t)j * nc + j] - s[j] * s[j] / n;
        rho[e] = cij / sqrt(cii * cjj);
    }
}

int grid_for(int64_t n, int per) {
    const int64_t g = (n + per - 1) / per;
    return (int)std::min<int64_t>(std::max<int64_t>(g, 1), 4096);
}

int scan(Arena &A, const uint32_t *in, int64_t n, uint64_t **out, hipStream_t s) {
    *out = A.take<uint64_t>(n + 1);
    void *w = A.take<char>(sdp_scan_workspace_bytes(n));
    SDP_NEED(*out, A);
    SDP_NEED(w, A);
    return sdp_scan_u32(in, n, *out, w, sdp_scan_workspace_bytes(n), s);
}

// ---- groups of one column (engine.group / _distinct_fixed_table / bytes table) -----
struct Groups {
    // dense (partitioned, with counts) or table arrays the top-k runs on
    uint64_t *slots = nullptr, *counts = nullptr;
    int64_t capacity = 0;
    int flags = 0;                  // bit0 byte keys, bit1 dense arrays
    uint64_t groups = 0;            // distinct values (incl. the special key)
    uint64_t groups_local = 0;      // groups held in slots/counts
    uint64_t special = 0;           // rows of the UINT64_MAX key kept outside a table
    uint64_t rows = 0;
    int path = 0;
};

struct Heavy {
    int n = 0;
    std::vector<uint64_t> h, meta;  // host copies, the most frequent key first
    std::vector<int64_t> cnt;       // sample occurrences of each
    uint64_t *d_h = nullptr, *d_k0 = nullptr, *d_k1 = nullptr, *d_meta = nullptr;
    double rec_frac = 1.0;
    int ns = 1;                     // sample rows
    bool near_unique = false;
    // the first `cap` keys only (engine._hv_cap): the row kernels' LDS tables
    // hold SDP_HEAVY_MAX, the byte records kernel SDP_HEAVY_MAX_REC; rows of
    // the dropped keys become partition records, the groups are the same
    void cap_to(int cap) {
        if (n <= cap) return;
        int64_t dropped = 0;
        for (int i = cap; i < n; ++i) dropped += cnt[i];
        rec_frac += (double)dropped / (double)ns;
        n = cap;
        h.resize(cap);
        cnt.resize(cap);
        if (!meta.empty()) meta.resize(cap);
    }
};

// keys seen >= HEAVY_MIN times in an evenly spaced sample (engine._heavy_keys):
// counted outside the partitions, so skew never piles into one bucket
int heavy_keys(Arena &A, const sdp_column *col, const sdp_bytes_column *bcol, int64_t n, Heavy &hv, hipStream_t s) {
    const int ns = (int)std::min<int64_t>(bcol ? PART_SAMPLE_BYTES : PART_SAMPLE, std::max<int64_t>(n, 1));
    hv.ns = ns;
    uint64_t *dh = A.take<uint64_t>(ns);
    SDP_NEED(dh, A);
    sdp_records rec{nullptr, nullptr, nullptr};
    if (bcol) {
        rec.d_k0 = A.take<uint64_t>(ns);
        rec.d_k1 = A.take<uint64_t>(ns);
        rec.d_meta = A.take<uint64_t>(ns);
        SDP_NEED(rec.d_meta, A);
    }
    SDP_TRY(sdp_part_sample(col, bcol, ns, dh, bcol ? &rec : nullptr, s));
    std::vector<uint64_t> h(ns), k0, k1, meta;
    SDP_TRY(d2h(h.data(), dh, ns * 8, s));
    if (bcol) {
        k0.resize(ns); k1.resize(ns); meta.resize(ns);
        SDP_TRY(d2h(k0.data(), rec.d_k0, ns * 8, s));
        SDP_TRY(d2h(k1.data(), rec.d_k1, ns * 8, s));
        SDP_TRY(d2h(meta.data(), rec.d_meta, ns * 8, s));
    }
    std::vector<std::pair<uint64_t, int>> v;           // (hash, sample index) of valid rows
    int n_valid = 0;
    for (int i = 0; i < ns; ++i) {
        if (h[i] == EMPTY64) continue;
        ++n_valid;
        if (bcol && (meta[i] >> 40) > 16) continue;   // long strings are never heavy
        v.push_back({h[i], i});
    }
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    struct U { uint64_t h; int first, cnt; };
    std::vector<U> u;
    for (size_t i = 0; i < v.size();) {
        size_t j = i;
        while (j < v.size() && v[j].first == v[i].first) ++j;
        u.push_back({v[i].first, v[i].second, (int)(j - i)});
        i = j;
    }
    hv.near_unique = !bcol && (double)u.size() >= 0.9 * (double)v.size();
    std::vector<U> sel;
    for (const U &x : u)
        if (x.cnt >= HEAVY_MIN) sel.push_back(x);
    if (sel.empty()) return 0;
    // the most frequent first (engine._heavy_struct), at most SDP_HEAVY_MAX_REC
    // byte keys / SDP_HEAVY_MAX fixed keys; group_partitioned caps byte keys
    // to SDP_HEAVY_MAX when the row kernels, not the records kernel, take them
    std::stable_sort(sel.begin(), sel.end(), [](const U &a, const U &b) { return a.cnt > b.cnt; });
    const int cap = bcol ? SDP_HEAVY_MAX_REC : SDP_HEAVY_MAX;
    if ((int)sel.size() > cap) sel.resize(cap);
    hv.n = (int)sel.size();
    int64_t heavy_rows = 0;
    std::vector<uint64_t> hk0, hk1;
    for (const U &x : sel) {
        hv.h.push_back(x.h);
        hv.cnt.push_back(x.cnt);
        heavy_rows += x.cnt;
        if (bcol) {
            hk0.push_back(k0[x.first]);
            hk1.push_back(k1[x.first]);
            hv.meta.push_back(meta[x.first]);
        }
    }
    hv.rec_frac = (double)(n_valid - heavy_rows) / (double)ns;
    hv.d_h = A.take<uint64_t>(hv.n);
    SDP_NEED(hv.d_h, A);
    SDP_TRY(h2d(hv.d_h, hv.h.data(), hv.n * 8, s));
    if (bcol) {
        hv.d_k0 = A.take<uint64_t>(hv.n);
        hv.d_k1 = A.take<uint64_t>(hv.n);
        hv.d_meta = A.take<uint64_t>(hv.n);
        SDP_NEED(hv.d_meta, A);
        SDP_TRY(h2d(hv.d_k0, hk0.data(), hv.n * 8, s));
        SDP_TRY(h2d(hv.d_k1, hk1.data(), hv.n * 8, s));
        SDP_TRY(h2d(hv.d_meta, hv.meta.data(), hv.n * 8, s));
    }
    return 0;
}

// Two-level hash partitioning with exact offsets + LDS de-duplication
// (engine._group_prepare / _group_count / _group_middle / _group_end).
// Returns 0 with *ok = false when the column needs the global table (more
// than 20 hash bits of buckets, a 64-bit collision, a full LDS table).
int group_partitioned(Arena &A, const sdp_column *col, const sdp_bytes_column *bcol, int64_t n, bool with_counts,
                      Groups &g, bool *ok, hipStream_t s) {
    *ok = false;
    const bool isb = bcol != nullptr;
    with_counts = with_counts || isb;
    Heavy hv;
    SDP_TRY(heavy_keys(A, col, bcol, n, hv, s));
    const int64_t target = sdp_part_bucket_target(isb, with_counts);
    auto bits_for = [](double x) { return x <= 1.0 ? 0 : (int)std::ceil(std::log2(x)); };
    int total_bits, b1;
    bool one_read;
    while (true) {                                 // (engine._group_prepare)
        int64_t n_rec = n;
        if (isb && hv.n > 0) n_rec = std::min<int64_t>(n, (int64_t)((double)n * (1.25 * hv.rec_frac + 0.02)) + 1);
        total_bits = bits_for((double)n_rec / (double)target);
        b1 = std::min(10, (total_bits + 1) / 2);
        one_read = isb && b1 > 0;
        if (!isb || one_read || hv.n <= SDP_HEAVY_MAX) break;
        hv.cap_to(SDP_HEAVY_MAX);                  // b1 == 0: the row kernels take the bytes
    }
    bool large = false;
    if (total_bits > 20 && !isb && !with_counts) {
        total_bits = std::max(20, bits_for((double)n / (4.0 * (double)target)));
        large = true;
        b1 = std::min(10, (total_bits + 1) / 2);
    }
    const int b2 = total_bits - b1;
    if (b2 > 10) return 0;
    const int64_t nb1 = 1ll << b1, nb2 = 1ll << b2;
    int64_t grid;
    if (one_read) grid = sdp_part_records_chunks(n);
    else {
        const int64_t rpb = sdp_part_rows_per_block(n, isb);
        grid = std::max<int64_t>(1, (n + rpb - 1) / rpb);
    }
    sdp_heavy hstruct{hv.d_h, hv.d_k0, hv.d_k1, hv.d_meta, hv.n, 0};
    const sdp_heavy *hp = hv.n ? &hstruct : nullptr;
    uint64_t *stats = A.take<uint64_t>(68);
    uint64_t *hcnt = A.take<uint64_t>(std::max(hv.n, 1));
    uint32_t *h1 = A.take<uint32_t>(nb1 * grid);
    SDP_NEED(h1, A);
    SDP_TRY(zero(stats, 68 * 8, s));
    SDP_TRY(zero(hcnt, std::max(hv.n, 1) * 8, s));
    auto records = [&](int64_t m, sdp_records &r) -> bool {
        r.d_k0 = A.take<uint64_t>(m);
        r.d_k1 = isb ? A.take<uint64_t>(m) : nullptr;
        r.d_meta = isb ? A.take<uint64_t>(m) : nullptr;
        return r.d_k0 != nullptr && (!isb || r.d_meta != nullptr);
    };
    // level-1 count (byte columns: the strings read once into strip records)
    sdp_records r0{nullptr, nullptr, nullptr};
    sdp_chunk *chunks0 = nullptr;
    if (one_read) {
        if (!records(n, r0)) return set_error(SDP_ECAP, "workspace too small (records)");
        chunks0 = A.take<sdp_chunk>(grid);
        SDP_NEED(chunks0, A);
        SDP_TRY(sdp_part_rows_records(bcol, hp, b1, h1, chunks0, &r0, hcnt, stats, s));
    } else {
        SDP_TRY(sdp_part_rows(col, bcol, hp, b1, 0, h1, nullptr, nullptr, hcnt, stats, s));
    }
    uint64_t *o1 = nullptr;
    SDP_TRY(scan(A, h1, nb1 * grid, &o1, s));
    uint64_t *bsn_d = A.take<uint64_t>(nb1 + 1);
    SDP_NEED(bsn_d, A);
    hipLaunchKernelGGL(gather_strided_kernel, dim3(grid_for(nb1 + 1, 256)), dim3(256), 0, s, o1, grid, nb1,
                       nb1 * grid, bsn_d);
    SDP_TRY(check_launch("gather_strided_kernel"));
    std::vector<uint64_t> bsn(nb1 + 1);
    SDP_TRY(d2h(bsn.data(), bsn_d, (nb1 + 1) * 8, s));
    const int64_t nrec = (int64_t)bsn[nb1];
    // level-1 scatter
    sdp_records r1{nullptr, nullptr, nullptr};
    if (!records(nrec, r1)) return set_error(SDP_ECAP, "workspace too small (records)");
    if (one_read) {
        if (nrec) SDP_TRY(sdp_part_recs(&r0, 1, chunks0, grid, 0, b1, 1, nullptr, o1, &r1, s));
    } else if (nrec) {
        SDP_TRY(sdp_part_rows(col, bcol, hp, b1, 1, nullptr, o1, &r1, hcnt, stats, s));
    }
    // level 2: every L1 bucket -> nb2 sub-buckets, chunk by chunk
    sdp_records rf = r1;
    uint64_t *starts = A.take<uint64_t>(nb1 * nb2 + 1);
    SDP_NEED(starts, A);
    if (b2 == 0 || nrec == 0) {
        if (b2 == 0) SDP_TRY(h2d(starts, bsn.data(), (nb1 + 1) * 8, s));
        else SDP_TRY(zero(starts, (nb1 * nb2 + 1) * 8, s));
    } else {
        std::vector<int64_t> nch(nb1), k0(nb1);
        int64_t K = 0;
        for (int64_t b = 0; b < nb1; ++b) {
            nch[b] = ((int64_t)(bsn[b + 1] - bsn[b]) + PART_CHUNK - 1) / PART_CHUNK;
            k0[b] = K;
            K += nch[b];
        }
        std::vector<sdp_chunk> ch;
        ch.reserve(K);
        for (int64_t b = 0; b < nb1; ++b)
            for (int64_t j = 0; j < nch[b]; ++j) {
                const int64_t st = (int64_t)bsn[b] + j * PART_CHUNK;
                ch.push_back(sdp_chunk{st, std::min<int64_t>((int64_t)bsn[b + 1], st + PART_CHUNK), nb2 * k0[b] + j,
                                       nch[b]});
            }
        sdp_chunk *chunks = A.take<sdp_chunk>(K);
        uint32_t *h2 = A.take<uint32_t>(nb2 * K);
        SDP_NEED(h2, A);
        SDP_NEED(chunks, A);
        SDP_TRY(h2d(chunks, ch.data(), K * sizeof(sdp_chunk), s));
        SDP_TRY(sdp_part_recs(&r1, isb, chunks, K, b1, b2, 0, h2, nullptr, nullptr, s));
        uint64_t *o2 = nullptr;
        SDP_TRY(scan(A, h2, nb2 * K, &o2, s));
        // (byte columns: the strip records are dead after the level-1 scatter)
        if (one_read) rf = r0;
        else if (!records(nrec, rf)) return set_error(SDP_ECAP, "workspace too small (records)");
        SDP_TRY(sdp_part_recs(&r1, isb, chunks, K, b1, b2, 1, nullptr, o2, &rf, s));
        std::vector<int64_t> sidx(nb1 * nb2 + 1);
        for (int64_t b = 0; b < nb1; ++b)
            for (int64_t sub = 0; sub < nb2; ++sub) sidx[b * nb2 + sub] = nb2 * k0[b] + sub * nch[b];
        sidx[nb1 * nb2] = nb2 * K;
        int64_t *d_sidx = A.take<int64_t>(nb1 * nb2 + 1);
        SDP_NEED(d_sidx, A);
        SDP_TRY(h2d(d_sidx, sidx.data(), sidx.size() * 8, s));
        hipLaunchKernelGGL(gather_idx_kernel, dim3(grid_for(nb1 * nb2 + 1, 256)), dim3(256), 0, s, o2, d_sidx,
                           nb1 * nb2 + 1, starts);
        SDP_TRY(check_launch("gather_idx_kernel"));
    }
    // de-duplication of every final bucket in LDS
    const int64_t nfinal = nb1 * nb2;
    uint32_t *ngroups = A.take<uint32_t>(nfinal);
    SDP_NEED(ngroups, A);
    SDP_TRY(zero(ngroups, nfinal * 4, s));
    uint64_t *out_key = nullptr, *out_cnt = nullptr;
    if (with_counts) {
        out_key = A.take<uint64_t>(std::max<int64_t>(nrec, 1));
        out_cnt = A.take<uint64_t>(std::max<int64_t>(nrec, 1));
        SDP_NEED(out_cnt, A);
    }
    if (nrec) {
        const int direct = (!isb && !with_counts && !large && hv.near_unique) ? 4 : 0;
        SDP_TRY(sdp_part_dedup(&rf, isb, bcol, starts, nfinal, (with_counts ? 1 : 0) | (large ? 2 : 0) | direct,
                               out_key, out_cnt, ngroups, stats, s));
    }
    std::vector<uint64_t> st(68), hc(std::max(hv.n, 1));
    SDP_TRY(d2h(st.data(), stats, 68 * 8, s));
    if (hv.n) SDP_TRY(d2h(hc.data(), hcnt, hv.n * 8, s));
    if (st[2] || st[3]) return 0;                  // collision / full table: the caller takes the global table
    uint64_t groups_local = 0;
    for (int i = 4; i < 68; ++i) groups_local += st[i];
    const uint64_t special = st[1];
    std::vector<uint64_t> ek, ec;                  // heavy and special groups, appended to the dense arrays
    for (int i = 0; i < hv.n; ++i)
        if (hc[i]) {
            ek.push_back(isb ? (((hv.h[i] >> 40) << 40) | (hv.meta[i] & ((1ull << 40) - 1))) : inv_mix64(hv.h[i]));
            ec.push_back(hc[i]);
        }
    if (special) {
        ek.push_back(inv_mix64(EMPTY64));
        ec.push_back(special);
    }
    g.groups = groups_local + ek.size();
    g.rows = st[0];
    g.path = 1;
    if (with_counts) {
        const int64_t total = (int64_t)g.groups;
        g.slots = A.take<uint64_t>(std::max<int64_t>(total, 1));
        g.counts = A.take<uint64_t>(std::max<int64_t>(total, 1));
        SDP_NEED(g.counts, A);
        if (groups_local) {
            uint64_t *offs = nullptr;
            SDP_TRY(scan(A, ngroups, nfinal, &offs, s));
            SDP_TRY(sdp_part_compact(out_key, out_cnt, starts, ngroups, offs, nfinal, g.slots, g.counts, s));
        }
        if (!ek.empty()) {
            SDP_TRY(h2d(g.slots + groups_local, ek.data(), ek.size() * 8, s));
            SDP_TRY(h2d(g.counts + groups_local, ec.data(), ec.size() * 8, s));
        }
        g.capacity = std::max<int64_t>(total, 1);
        g.groups_local = g.groups;
        g.flags = (isb ? 1 : 0) | 2;
    }
    *ok = true;
    return 0;
}

// the global open-addressing table (engine._distinct_fixed_table / value_counts_bytes_table)
int group_table(Arena &A, const sdp_column *col, const sdp_bytes_column *bcol, int64_t n, bool with_counts,
                Groups &g, hipStream_t s) {
    const bool isb = bcol != nullptr;
    with_counts = with_counts || isb;
    const int64_t cap = next_pow2_cap(2 * std::max<int64_t>(n, 1));
    g.slots = A.take<uint64_t>(cap);
    g.counts = with_counts ? A.take<uint64_t>(cap) : nullptr;
    uint64_t *stats = A.take<uint64_t>(4);
    SDP_NEED(g.slots, A);
    SDP_NEED(stats, A);
    if (with_counts) SDP_NEED(g.counts, A);
    SDP_TRY(zero(stats, 32, s));
    SDP_TRY(sdp_table_clear(g.slots, g.counts, cap, isb ? 1 : 0, s));
    if (isb) SDP_TRY(sdp_hash_bytes(bcol, nullptr, g.slots, g.counts, cap, stats, s));
    else SDP_TRY(sdp_hash_u64(col, nullptr, g.slots, g.counts, cap, with_counts ? 1 : 0, stats, s));
    uint64_t st[4];
    SDP_TRY(d2h(st, stats, 32, s));
    g.capacity = cap;
    g.flags = isb ? 1 : 0;
    g.groups_local = st[0];
    g.special = isb ? 0 : st[2];
    g.groups = st[0] + (g.special ? 1 : 0);
    g.rows = st[1] + g.special;
    g.path = 2;
    return 0;
}

int check_inputs(const sdp_column *col, const sdp_bytes_column *bcol, const char *who) {
    if ((col == nullptr) == (bcol == nullptr)) return set_error(SDP_EINVAL, "%s: exactly one of col / bcol", who);
    if (col) {
        if (col->length < 0 || (col->length > 0 && col->d_values == nullptr))
            return set_error(SDP_EINVAL, "%s: column", who);
        if (!groupable(col->dtype)) return set_error(SDP_EINVAL, "%s: dtype %d", who, col->dtype);
        if (col->dtype != SDP_BOOL && !aligned16(col->d_values)) return set_error(SDP_EALIGN, "%s: values not 16-byte aligned", who);
    } else if (bcol->length < 0 || (bcol->length > 0 && bcol->d_data == nullptr)) {
        return set_error(SDP_EINVAL, "%s: byte column", who);
    }
    return 0;
}

int groups_of(Arena &A, const sdp_column *col, const sdp_bytes_column *bcol, bool with_counts, Groups &g,
              hipStream_t s) {
    const int64_t n = col ? col->length : bcol->length;
    if (n >= (1 << 16)) {
        const int64_t mark = A.used;
        bool ok = false;
        SDP_TRY(group_partitioned(A, col, bcol, n, with_counts, g, &ok, s));
        if (ok) return 0;
        A.used = mark;                             // the table reuses the partitions' space
        g = Groups();
    }
    return group_table(A, col, bcol, n, with_counts, g, s);
}

// ---- top-k by (count desc, key asc) over a group table (engine.topk) ------------
struct TopK {
    Arena &A;
    const Groups &g;
    const sdp_bytes_column *bcol;
    hipStream_t s;
    std::vector<std::pair<uint64_t, uint64_t>> out;   // (slot value, count)

    int select(uint64_t cmin, uint64_t cmax, int64_t limit, uint64_t **sel, uint64_t **on) {
        *sel = A.take<uint64_t>(std::max<int64_t>(limit, 1));
        *on = A.take<uint64_t>(1);
        SDP_NEED(*on, A);
        SDP_NEED(*sel, A);
        SDP_TRY(zero(*on, 8, s));
        return sdp_table_select(g.slots, g.counts, g.capacity, g.flags, cmin, cmax, *sel, *on,
                                (uint64_t)std::max<int64_t>(limit, 1), s);
    }
    // sort the selected groups (count desc, key asc), append the first `take`
    int sort_take(uint64_t *sel, uint64_t *on, int64_t cap_sel, int64_t take) {
        SDP_TRY(sdp_sort_groups(sel, on, g.slots, g.counts, bcol, s));
        const int64_t t = std::max<int64_t>(1, std::min(take, cap_sel));
        uint64_t *pack = A.take<uint64_t>(1 + 3 * t);
        SDP_NEED(pack, A);
        hipLaunchKernelGGL(take_pack_kernel, dim3(grid_for(t, 256)), dim3(256), 0, s, sel, on, t, g.slots, g.counts,
                           pack);
        SDP_TRY(check_launch("take_pack_kernel"));
        std::vector<uint64_t> h(1 + 3 * t);
        SDP_TRY(d2h(h.data(), pack, h.size() * 8, s));
        const int64_t m = std::min<int64_t>((int64_t)h[0], take);
        for (int64_t i = 0; i < m && i < t; ++i) out.push_back({h[1 + 2 * t + i], h[1 + t + i]});
        return 0;
    }
    int count_hist(uint64_t lo, uint64_t step, std::vector<uint64_t> &c) {
        uint64_t *d = A.take<uint64_t>(2048);
        SDP_NEED(d, A);
        SDP_TRY(zero(d, 2048 * 8, s));
        SDP_TRY(sdp_table_count_hist(g.slots, g.counts, g.capacity, g.flags, lo, step, d, s));
        c.resize(2048);
        return d2h(c.data(), d, 2048 * 8, s);
    }
    // the r groups with the smallest keys among n_eq groups of one count
    // (engine._smallest_keys_among): keys cut by a radix select; byte keys by
    // 8-byte big-endian prefixes, recursively
    int smallest_keys(uint64_t *sel, uint64_t *on, int64_t n, int64_t r) {
        const int64_t sws = sdp_select_kth_workspace_bytes(n);
        if (!(g.flags & 1)) {
            uint64_t *keys = A.take<uint64_t>(n);
            void *ws = A.take<char>(sws);
            uint64_t *kth = A.take<uint64_t>(1);
            SDP_NEED(keys, A);
            SDP_NEED(ws, A);
            SDP_NEED(kth, A);
            hipLaunchKernelGGL(gather_idx_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, g.slots,
                               (const int64_t *)sel, n, keys);
            SDP_TRY(check_launch("gather_idx_kernel"));
            SDP_TRY(sdp_select_kth(keys, on, n, r - 1, 0, EMPTY64, ws, sws, kth, s));
            uint64_t kh;
            SDP_TRY(d2h(&kh, kth, 8, s));
            uint64_t *o = nullptr, *on2 = nullptr;
            o = A.take<uint64_t>(r);
            on2 = A.take<uint64_t>(1);
            SDP_NEED(on2, A);
            SDP_NEED(o, A);
            SDP_TRY(zero(on2, 8, s));
            SDP_TRY(sdp_select_by_value(sel, keys, on, 0, kh, o, nullptr, on2, s));
            return sort_take(o, on2, r, r);
        }
        // buffers taken once for the first (largest) n and reused by every
        // prefix round: the tie set of round i is the selection of round i+1
        // (two tie buffers, alternating); sort_take's small packs are released
        // at the start of each round
        uint64_t *pre = A.take<uint64_t>(n), *kth = A.take<uint64_t>(1);
        const int64_t ws_bytes = sdp_select_kth_workspace_bytes(n);
        void *ws = A.take<char>(ws_bytes);
        uint64_t *below = A.take<uint64_t>(n), *bn = A.take<uint64_t>(1);
        uint64_t *eqb[2] = {A.take<uint64_t>(n), A.take<uint64_t>(n)};
        uint64_t *enb[2] = {A.take<uint64_t>(1), A.take<uint64_t>(1)};
        SDP_NEED(enb[1], A);
        SDP_NEED(enb[0], A);
        SDP_NEED(eqb[1], A);
        SDP_NEED(eqb[0], A);
        SDP_NEED(below, A);
        SDP_NEED(ws, A);
        SDP_NEED(kth, A);
        SDP_NEED(pre, A);
        const int64_t mark = A.used;
        int offset = 0, flip = 0;
        int64_t need = r;
        while (true) {
            A.used = mark;
            uint64_t *eq = eqb[flip], *en = enb[flip];
            flip ^= 1;
            SDP_TRY(sdp_group_prefix(sel, on, g.slots, bcol, offset, pre, s));
            SDP_TRY(sdp_select_kth(pre, on, n, need - 1, 0, EMPTY64, ws, ws_bytes, kth, s));
            uint64_t kh;
            SDP_TRY(d2h(&kh, kth, 8, s));
            SDP_TRY(zero(bn, 8, s));
            SDP_TRY(zero(en, 8, s));
            if (kh > 0) SDP_TRY(sdp_select_by_value(sel, pre, on, 0, kh - 1, below, nullptr, bn, s));
            uint64_t nb = 0;
            SDP_TRY(d2h(&nb, bn, 8, s));
            if (nb) SDP_TRY(sort_take(below, bn, (int64_t)nb, (int64_t)nb));
            need -= (int64_t)nb;
            SDP_TRY(sdp_select_by_value(sel, pre, on, kh, kh, eq, nullptr, en, s));
            uint64_t ne = 0;
            SDP_TRY(d2h(&ne, en, 8, s));
            if ((int64_t)ne <= GSORT_MAX) return sort_take(eq, en, (int64_t)ne, need);
            sel = eq;
            on = en;
            n = (int64_t)ne;
            offset += 8;
        }
    }
    int run(int64_t k) {
        const int64_t groups = (int64_t)g.groups_local;
        if (groups <= k) {
            uint64_t *sel, *on;
            SDP_TRY(select(1, EMPTY64, std::max<int64_t>(groups, 1), &sel, &on));
            return sort_take(sel, on, std::max<int64_t>(groups, 1), k);
        }
        uint64_t *hist = A.take<uint64_t>(64);
        SDP_NEED(hist, A);
        SDP_TRY(zero(hist, 64 * 8, s));
        SDP_TRY(sdp_table_count_log2_hist(g.slots, g.counts, g.capacity, g.flags, hist, s));
        std::vector<uint64_t> h(64);
        SDP_TRY(d2h(h.data(), hist, 64 * 8, s));
        int64_t cum = 0;
        int b = 63;
        for (; b >= 0; --b) {
            cum += (int64_t)h[b];
            if (cum >= k) break;
        }
        b = std::max(b, 0);
        uint64_t lo = 1ull << b;
        if (cum <= GSORT_MAX) {
            uint64_t *sel, *on;
            SDP_TRY(select(lo, EMPTY64, cum, &sel, &on));
            return sort_take(sel, on, cum, k);
        }
        // exact threshold T = the k-th largest count inside [2^b, 2^(b+1))
        int64_t need = k - (cum - (int64_t)h[b]);
        uint64_t width = 1ull << b, T = 0;
        int64_t n_eq = 0;
        while (true) {
            const uint64_t step = std::max<uint64_t>(1, (width + 2047) / 2048);
            std::vector<uint64_t> c;
            SDP_TRY(count_hist(lo, step, c));
            const int64_t nb = (int64_t)std::min<uint64_t>(2048, (width + step - 1) / step);
            int64_t acc = 0, j = nb - 1;
            for (; j >= 0; --j) {
                if (acc + (int64_t)c[j] >= need) break;
                acc += (int64_t)c[j];
            }
            need -= acc;
            if (step == 1) {
                T = lo + (uint64_t)j;
                n_eq = (int64_t)c[j];
                break;
            }
            lo += (uint64_t)j * step;
            width = step;
        }
        uint64_t *sel, *on;
        SDP_TRY(select(T + 1, EMPTY64, k, &sel, &on));
        SDP_TRY(sort_take(sel, on, k, k));            // < k groups, all in the top-k
        const int64_t r_t = k - (int64_t)out.size();
        SDP_TRY(select(T, T, n_eq, &sel, &on));
        if (n_eq <= GSORT_MAX) return sort_take(sel, on, n_eq, r_t);
        return smallest_keys(sel, on, n_eq, r_t);
    }
};

}  // namespace
}  // namespace sdp

using namespace sdp;

// ---- sdp_minmax_int ---------------------------------------------------------------
extern "C" int64_t sdp_minmax_workspace_bytes(int64_t length, int32_t dtype) {
    const int64_t p1 = sdp_pass1_workspace_bytes(length, dtype);
    if (p1 < 0) return -1;
    return 3 * ARENA_ALIGN + (int64_t)sizeof(sdp_qplan) + (int64_t)sizeof(sdp_pass1_result) + p1;
}

extern "C" int sdp_minmax_int(const sdp_column *col, void *d_work, int64_t work_bytes, sdp_minmax_result *d_out,
                              void *stream) {
    if (col == nullptr || d_out == nullptr || d_work == nullptr) return set_error(SDP_EINVAL, "sdp_minmax_int: args");
    hipStream_t s = (hipStream_t)stream;
    Arena A(d_work, work_bytes);
    sdp_qplan *plan = A.take<sdp_qplan>(1);
    sdp_pass1_result *res = A.take<sdp_pass1_result>(1);
    const int64_t pw = sdp_pass1_workspace_bytes(col->length, col->dtype);
    if (pw < 0) return set_error(SDP_EINVAL, "sdp_minmax_int: dtype %d", col->dtype);
    void *w = A.take<char>(pw);
    SDP_NEED(w, A);
    SDP_NEED(res, A);
    SDP_NEED(plan, A);
    SDP_TRY(zero(plan, sizeof(sdp_qplan), s));      // n_windows 0: moments / min / max only
    SDP_TRY(sdp_pass1(col, plan, w, pw, nullptr, nullptr, 0, 0, res, s));
    hipLaunchKernelGGL(minmax_finish_kernel, dim3(1), dim3(1), 0, s, res, d_out);
    return check_launch("minmax_finish_kernel");
}

// ---- sdp_quantiles -----------------------------------------------------------------
extern "C" int64_t sdp_quantiles_workspace_bytes(int64_t length, int32_t n_probs) {
    if (length < 0 || n_probs < 0 || n_probs > SDP_QUANTILES_MAX) return -1;
    return 8 * ARENA_ALIGN + 8 * std::max<int64_t>(length, 1) + 8 + 2 * 16 * SDP_QUANTILES_MAX +
           sdp_select_kth_workspace_bytes(std::max<int64_t>(length, 1));
}

extern "C" int sdp_quantiles(const sdp_column *col, const double *probs, int32_t n_probs, void *d_work,
                             int64_t work_bytes, double *d_out, void *stream) {
    if (col == nullptr || probs == nullptr || d_out == nullptr || n_probs < 1 || n_probs > SDP_QUANTILES_MAX)
        return set_error(SDP_EINVAL, "sdp_quantiles: args");
    if (!numeric(col->dtype)) return set_error(SDP_EINVAL, "sdp_quantiles: dtype %d", col->dtype);
    QProbs q;
    q.n = n_probs;
    for (int i = 0; i < n_probs; ++i) {
        if (!(probs[i] >= 0.0 && probs[i] <= 1.0)) return set_error(SDP_EINVAL, "sdp_quantiles: p = %g", probs[i]);
        q.p[i] = probs[i];
    }
    hipStream_t s = (hipStream_t)stream;
    Arena A(d_work, work_bytes);
    const int64_t ncap = std::max<int64_t>(col->length, 1);
    uint64_t *keys = A.take<uint64_t>(ncap), *dn = A.take<uint64_t>(1);
    int64_t *dk = A.take<int64_t>(2 * SDP_QUANTILES_MAX);
    uint64_t *res = A.take<uint64_t>(2 * SDP_QUANTILES_MAX);
    const int64_t sws = sdp_select_kth_workspace_bytes(ncap);
    void *ws = A.take<char>(sws);
    SDP_NEED(ws, A);
    SDP_NEED(res, A);
    SDP_NEED(dk, A);
    SDP_NEED(dn, A);
    SDP_NEED(keys, A);
    const int is_int = !floating(col->dtype);
    SDP_TRY(zero(dn, 8, s));
    SDP_TRY(sdp_column_keys(col, keys, dn, s));       // the na.drop keys
    hipLaunchKernelGGL(quantile_ranks_kernel, dim3(1), dim3(64), 0, s, dn, q, is_int, dk);
    SDP_TRY(check_launch("quantile_ranks_kernel"));
    for (int j = 0; j < n_probs; ++j) {
        SDP_TRY(select_kth_dev(keys, dn, ncap, 0, dk + 2 * j, 0, EMPTY64, ws, sws, res + 2 * j, stream));
        if (is_int) SDP_TRY(select_kth_dev(keys, dn, ncap, 0, dk + 2 * j + 1, 0, EMPTY64, ws, sws, res + 2 * j + 1, stream));
    }
    hipLaunchKernelGGL(quantile_values_kernel, dim3(1), dim3(64), 0, s, dn, res, q, is_int, d_out);
    return check_launch("quantile_values_kernel");
}

// ---- sdp_hash_distinct_count ------------------------------------------------------
static int64_t groups_workspace(int64_t n, int32_t is_bytes, bool with_counts) {
    n = std::max<int64_t>(n, 1);
    const int64_t recw = is_bytes ? 24 : 8;
    // partitions: strip/level-1/level-2 records (byte columns reuse the strip
    // buffer for level 2) + group outputs + dense arrays; the table reuses it all
    const int64_t part = 2 * recw * n + ((with_counts || is_bytes) ? 32 * n : 0);
    const int64_t cap = next_pow2_cap(2 * n);
    const int64_t table = 8 * cap + ((with_counts || is_bytes) ? 8 * cap : 0);
    return SMALL_BYTES + std::max(part, table);
}

extern "C" int64_t sdp_distinct_workspace_bytes(int64_t length, int32_t is_bytes) {
    if (length < 0) return -1;
    const int64_t bm = sdp_bitmap_workspace_bytes(length, SDP_BITMAP_MAX_BITS);
    const int64_t mm = std::max(sdp_minmax_workspace_bytes(length, SDP_I8), sdp_minmax_workspace_bytes(length, SDP_I64));
    return std::max(groups_workspace(length, is_bytes, false), SMALL_BYTES + mm + (bm > 0 ? bm : 0));
}

extern "C" int sdp_hash_distinct_count(const sdp_column *col, const sdp_bytes_column *bcol, void *d_work,
                                       int64_t work_bytes, sdp_distinct_result *h_out, void *stream) {
    SDP_TRY(check_inputs(col, bcol, "sdp_hash_distinct_count"));
    if (h_out == nullptr || d_work == nullptr) return set_error(SDP_EINVAL, "sdp_hash_distinct_count: args");
    hipStream_t s = (hipStream_t)stream;
    Arena A(d_work, work_bytes);
    memset(h_out, 0, sizeof(*h_out));
    if (col && integral(col->dtype)) {
        // small integral ranges: one bit per possible value in LDS (sdp_bitmap.hip)
        sdp_minmax_result *mm = A.take<sdp_minmax_result>(1);
        const int64_t mw = sdp_minmax_workspace_bytes(col->length, col->dtype);
        void *w = A.take<char>(mw);
        SDP_NEED(w, A);
        SDP_NEED(mm, A);
        SDP_TRY(sdp_minmax_int(col, w, mw, mm, stream));
        sdp_minmax_result h;
        SDP_TRY(d2h(&h, mm, sizeof(h), s));
        if (h.count == 0) return 0;
        const int64_t range = h.imax - h.imin + 1;
        if (range > 0 && range <= SDP_BITMAP_MAX_BITS) {
            const int64_t bw = sdp_bitmap_workspace_bytes(col->length, range);
            void *bwk = A.take<char>(bw);
            uint64_t *d = A.take<uint64_t>(1);
            SDP_NEED(d, A);
            SDP_NEED(bwk, A);
            SDP_TRY(zero(d, 8, s));
            SDP_TRY(sdp_distinct_bitmap(col, h.imin, range, bwk, bw, nullptr, d, s));
            SDP_TRY(d2h(&h_out->distinct, d, 8, s));
            h_out->rows = h.count;
            h_out->path = 0;
            return 0;
        }
        A.used = 0;
    }
    Groups g;
    SDP_TRY(groups_of(A, col, bcol, false, g, s));
    h_out->distinct = g.groups;
    h_out->rows = g.rows;
    h_out->path = g.path;
    return 0;
}

// ---- sdp_value_counts_topk --------------------------------------------------------
extern "C" int64_t sdp_value_counts_workspace_bytes(int64_t length, int32_t is_bytes) {
    if (length < 0) return -1;
    const int64_t n = std::max<int64_t>(length, 1);
    // + the top-k stage: selections, tie-breaking prefixes and a select workspace
    return groups_workspace(length, is_bytes, true) + 40 * n + sdp_select_kth_workspace_bytes(n);
}

extern "C" int sdp_value_counts_topk(const sdp_column *col, const sdp_bytes_column *bcol, int32_t k, void *d_work,
                                     int64_t work_bytes, sdp_topk_result *h_out, sdp_topk_entry *h_top,
                                     void *stream) {
    SDP_TRY(check_inputs(col, bcol, "sdp_value_counts_topk"));
    if (h_out == nullptr || (k > 0 && h_top == nullptr) || k < 0 || d_work == nullptr)
        return set_error(SDP_EINVAL, "sdp_value_counts_topk: args");
    if (k > SDP_GSORT_MAX) return set_error(SDP_EINVAL, "sdp_value_counts_topk: k = %d > %d", k, SDP_GSORT_MAX);
    hipStream_t s = (hipStream_t)stream;
    Arena A(d_work, work_bytes);
    memset(h_out, 0, sizeof(*h_out));
    Groups g;
    SDP_TRY(groups_of(A, col, bcol, true, g, s));
    h_out->groups = g.groups;
    h_out->rows = g.rows;
    h_out->path = g.path;
    if (k == 0 || g.groups == 0) return 0;
    TopK t{A, g, bcol, s, {}};
    if (g.groups_local) SDP_TRY(t.run(k));
    std::vector<std::pair<uint64_t, uint64_t>> top = t.out;
    if (g.special) top.push_back({EMPTY64, g.special});        // the key kept outside the table (largest key)
    const bool isb = bcol != nullptr;
    std::stable_sort(top.begin(), top.end(), [&](const std::pair<uint64_t, uint64_t> &a,
                                                 const std::pair<uint64_t, uint64_t> &b) {
        if (a.second != b.second) return a.second > b.second;
        return !isb && a.first < b.first;          // byte keys: already in key order from sort_groups
    });
    if ((int64_t)top.size() > k) top.resize(k);
    h_out->n_top = (int32_t)top.size();
    for (size_t i = 0; i < top.size(); ++i) {
        // byte groups hold (hash tag << 40 | row + 1): report the row
        h_top[i].key = isb ? ((top[i].first & ((1ull << 40) - 1)) - 1) : top[i].first;
        h_top[i].count = top[i].second;
    }
    return 0;
}

// ---- sdp_gram_f64 -------------------------------------------------------------------
extern "C" int64_t sdp_pearson_workspace_bytes(int64_t length, int32_t ncols) {
    if (length < 0 || ncols < 1) return -1;
    const int64_t gw = sdp_gram_workspace_bytes(length, ncols);
    if (gw < 0) return -1;
    return 16 * ARENA_ALIGN + (int64_t)ncols * (sizeof(sdp_column) + 4 + 8 + 8 + 8 * 16384) +
           ((length + 31) / 32) * 4 + gw + 8 * (int64_t)ncols * ncols + 8;
}

extern "C" int sdp_gram_f64(const sdp_column *cols, int32_t ncols, void *d_work, int64_t work_bytes, double *d_corr,
                            double *d_n, void *stream) {
    if (cols == nullptr || ncols < 1 || d_corr == nullptr || d_n == nullptr || d_work == nullptr)
        return set_error(SDP_EINVAL, "sdp_gram_f64: args");
    const int64_t n = cols[0].length;
    std::vector<int32_t> isf(ncols);
    for (int i = 0; i < ncols; ++i) {
        if (cols[i].length != n) return set_error(SDP_EINVAL, "sdp_gram_f64: column lengths differ");
        if (!numeric(cols[i].dtype)) return set_error(SDP_EINVAL, "sdp_gram_f64: dtype %d", cols[i].dtype);
        isf[i] = floating(cols[i].dtype) ? 1 : 0;
    }
    hipStream_t s = (hipStream_t)stream;
    Arena A(d_work, work_bytes);
    const int ns = 16384;
    sdp_column *dcols = A.take<sdp_column>(ncols);
    int32_t *d_isf = A.take<int32_t>(ncols);
    uint64_t *samples = A.take<uint64_t>((int64_t)ncols * ns);
    double *shift = A.take<double>(ncols), *colsum = A.take<double>(ncols);
    uint32_t *keep = A.take<uint32_t>((n + 31) / 32);
    double *G = A.take<double>((int64_t)ncols * ncols);
    const int64_t gw = sdp_gram_workspace_bytes(n, ncols);
    void *w = A.take<char>(gw);
    SDP_NEED(w, A);
    SDP_NEED(G, A);
    SDP_NEED(keep, A);
    SDP_NEED(colsum, A);
    SDP_NEED(shift, A);
    SDP_NEED(samples, A);
    SDP_NEED(d_isf, A);
    SDP_NEED(dcols, A);
    SDP_TRY(h2d(dcols, cols, ncols * sizeof(sdp_column), s));
    SDP_TRY(h2d(d_isf, isf.data(), ncols * 4, s));
    // shift K = each column's sample median (any K gives the same rho; a K
    // near the mean keeps the shifted products well conditioned)
    SDP_TRY(sdp_sample_keys_batch(dcols, ncols, ns, samples, s));
    SDP_TRY(sdp_sort_small_batch(samples, ns, ncols, s));
    hipLaunchKernelGGL(sample_median_kernel, dim3(ncols), dim3(64), 0, s, samples, ns, d_isf, shift);
    SDP_TRY(check_launch("sample_median_kernel"));
    SDP_TRY(sdp_rowmask(cols, isf.data(), ncols, w, gw, keep, s));
    SDP_TRY(sdp_gram(cols, ncols, keep, shift, w, gw, G, colsum, d_n, s));
    hipLaunchKernelGGL(pearson_kernel, dim3(grid_for((int64_t)ncols * ncols, 256)), dim3(256), 0, s, G, colsum, d_n,
                       ncols, d_corr);
    return check_launch("pearson_kernel");
}
