/*
 * sdp.h -- C ABI of libsdp.so, the MI355X (gfx950) statistics engine behind
 * spark_df_profiling's describe().
 *
 * The reference has no FFI: every statistic is a Spark SQL aggregate issued from
 * Python (/root/reference/spark_df_profiling/describe.py).  Each entry point below
 * replaces one group of those Spark calls; the comment on each names the
 * reference lines it stands in for.  Python binds these through ctypes
 * (spark-df-profiling_amd/spark_df_profiling/_native.py).
 *
 * Conventions (all entry points):
 *   - pointers named d_* are DEVICE pointers (HBM), owned by the caller (the torch
 *     caching allocator); the library never allocates or frees them;
 *   - work is enqueued on `stream` (a hipStream_t passed as void*); nothing
 *     synchronises unless the name says so;
 *   - return value: 0 on success, otherwise an SDP_E* code; sdp_last_error()
 *     returns a message for the calling thread;
 *   - value buffers must be 16-byte aligned; validity bitmaps are Arrow LSB-first
 *     bitmaps addressed with a bit offset and may be NULL (all rows valid).
 */
#ifndef SDP_H
#define SDP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- element types ------------------------------------------------------ */
enum sdp_dtype {
    SDP_I8 = 1, SDP_I16 = 2, SDP_I32 = 3, SDP_I64 = 4,
    SDP_F32 = 5, SDP_F64 = 6,
    SDP_U8 = 7, SDP_U16 = 8, SDP_U32 = 9, SDP_U64 = 10,
    SDP_BOOL = 11            /* Arrow bit-packed booleans */
};

enum sdp_status {
    SDP_OK = 0, SDP_EINVAL = 1, SDP_EALIGN = 2, SDP_EHIP = 3, SDP_ECAP = 4
};

#define SDP_MAX_WINDOWS 5     /* quantile windows per pass-1 launch */

/* ---- grouping policy (describe.py:143 countDistinct, :251 groupBy count) ---
 * One set of constants for every orchestrator: the library's coarse entries
 * (sdp_api.cpp) and the Python engine (engine.py reads them from _native.py,
 * which checks them against sdp_layout_info() at load). */
#define SDP_HEAVY_MAX         256      /* heavy keys the row kernels' LDS tables hold       */
#define SDP_HEAVY_MAX_REC     1024     /* heavy byte keys the records kernel holds          */
#define SDP_HEAVY_MIN         3        /* sample occurrences that make a key heavy          */
#define SDP_PART_SAMPLE       16384    /* heavy-key sample rows, fixed-width keys           */
#define SDP_PART_SAMPLE_BYTES 65536    /* heavy-key sample rows, byte keys                  */
#define SDP_PART_CHUNK        131072   /* level-2 records per chunk                         */
#define SDP_L2_BLOCK          64       /* records per block of sdp_part_l2_blocks           */
#define SDP_GSORT_MAX         8192     /* groups one sdp_sort_groups launch orders          */

/* ---- layout handshake ------------------------------------------------------
 * SDP_ABI_VERSION changes whenever a struct below, a record layout or its hash
 * (6: fixed-key records are the one-multiply mix64 of sdp_common.h; 7: level-2
 * block layout, sdp_blocks) or a policy
 * constant above changes.  A host binding compares sdp_layout_info() with its
 * own view and refuses a library that disagrees (a record-layout mismatch
 * between the engine and the library once turned garbage metas into row
 * indices on the GPU). */
#define SDP_ABI_VERSION 7
#define SDP_LAYOUT_NSIZES 18
typedef struct sdp_layout {
    int32_t abi_version;
    int32_t n_sizes;                   /* SDP_LAYOUT_NSIZES                           */
    /* byte-key records: byte_record_arrays parallel uint64 arrays (k0, k1, meta),
     * one record every byte_record_stride bytes in each */
    int32_t byte_record_arrays;
    int32_t byte_record_stride;
    int32_t fixed_record_bytes;        /* fixed-key level-1 / level-2 records (mix64 h) */
    int32_t heavy_max, heavy_max_rec, heavy_min;
    int32_t part_sample, part_sample_bytes, gsort_max, l2_block;
    int64_t part_chunk;
    /* sizeof: sdp_column, sdp_bytes_column, sdp_records, sdp_heavy, sdp_chunk,
     * sdp_qplan, sdp_pass1_result, sdp_select_task, sdp_compact_task,
     * sdp_pass1_task, sdp_pass2_task, sdp_rows_task, sdp_pass2_result,
     * sdp_minmax_result, sdp_distinct_result, sdp_topk_entry, sdp_topk_result,
     * sdp_blocks */
    int64_t sizes[SDP_LAYOUT_NSIZES];
} sdp_layout;
int sdp_layout_info(sdp_layout *out);      /* host only; always 0 */

/* One Arrow column slice resident in HBM. */
typedef struct sdp_column {
    const void    *d_values;           /* element 0 of the slice; 16-B aligned      */
    const uint8_t *d_validity;         /* Arrow bitmap or NULL                      */
    int64_t        validity_bit_offset;
    int64_t        length;             /* rows                                      */
    int32_t        dtype;              /* enum sdp_dtype                            */
    int32_t        _pad;
} sdp_column;

/* Variable-length byte keys (Arrow utf8 / binary, or fixed width). */
typedef struct sdp_bytes_column {
    const uint8_t *d_data;             /* value bytes (+16 readable padding bytes)  */
    const void    *d_offsets;          /* int32 or int64 offsets (length+1), or NULL */
    const uint8_t *d_validity;
    int64_t        validity_bit_offset;
    int64_t        length;
    int32_t        offset_width;       /* 4 or 8; ignored when fixed_width > 0      */
    int32_t        fixed_width;        /* >0: row i = d_data[i*w .. (i+1)*w)        */
} sdp_bytes_column;

/* Quantile windows chosen from a row sample (see sdp_quantile_plan). */
typedef struct sdp_qplan {
    uint64_t lo[SDP_MAX_WINDOWS];      /* order-preserving keys, inclusive         */
    uint64_t hi[SDP_MAX_WINDOWS];
    int32_t  in_sample[SDP_MAX_WINDOWS]; /* sample keys strictly inside window w */
    double   shift;                    /* moment shift K (sample median)           */
    int32_t  n_windows;
    int32_t  n_sample;                 /* valid, non-NaN sample elements           */
    /* bit w set: window w keeps its bounds exclusive (candidates strictly inside,
     * keys equal to a bound counted apart) -- a bound key repeated in the sample
     * or lo == 0; windows with the bit clear take bound keys as candidates. */
    int32_t  excl_mask;
    int32_t  _pad;
} sdp_qplan;

/* Pass-1 result: replaces describe.py:143-144 (count), :193-201 (one agg of
 * mean/min/max/variance/kurtosis/stddev/skewness/sum) and :220 (n_zeros). */
typedef struct sdp_pass1_result {
    uint64_t count;                    /* valid and not NaN (na.drop)              */
    uint64_t n_valid;                  /* valid (not null), NaN included           */
    uint64_t n_nan;
    uint64_t n_zero;                   /* x == 0.0 over valid rows (NaN never 0)   */
    int64_t  isum;                     /* integral: two's-complement wrapping sum  */
    int64_t  imin, imax;               /* integral min/max                         */
    double   dmin, dmax;               /* floating min/max (NaN excluded)          */
    double   shift;                    /* K used for the power sums                */
    double   s1_hi, s1_lo;             /* sum (x-K), compensated                   */
    double   s2;                       /* sum (x-K)^2                              */
    double   s3_hi, s3_lo;             /* sum (x-K)^3, compensated                 */
    double   s4;                       /* sum (x-K)^4                              */
    /* per quantile window w */
    uint64_t w_gt[SDP_MAX_WINDOWS];    /* #(key > hi)                              */
    uint64_t w_eq_lo[SDP_MAX_WINDOWS]; /* #(key == lo); 0 for inclusive windows    */
    uint64_t w_eq_hi[SDP_MAX_WINDOWS]; /* #(key == hi), 0 when hi == lo or incl.   */
    uint64_t w_in[SDP_MAX_WINDOWS];    /* candidates: #(lo < key < hi), or         */
                                       /* #(lo <= key <= hi) (excl_mask bit clear) */
    uint32_t w_overflow;               /* bit w: a block overflowed its slots       */
    uint32_t _pad;
} sdp_pass1_result;

/* Pass-2 result: replaces describe.py:215-218 (mad), :222-223 (high/low idx)
 * and :49 (the CASE-WHEN histogram groupBy).  hist counts follow separately. */
typedef struct sdp_pass2_result {
    double   abs_dev_sum;              /* sum |x - mean| over na.drop rows         */
    uint64_t n_high;                   /* #(x > hi_t), NaN counts (Spark order)    */
    uint64_t n_low;                    /* #(x < lo_t)                              */
    uint64_t n_unbinned;               /* na.drop rows matching no CASE branch     */
} sdp_pass2_result;

/* ---- diagnostics ---------------------------------------------------------- */
const char *sdp_last_error(void);
const char *sdp_version(void);

/* ---- workspace sizing (host-only, no device work) --------------------------- */
/* Bytes of d_work each entry point needs for a column of `length` rows. */
int64_t sdp_pass1_workspace_bytes(int64_t length, int32_t dtype);
int64_t sdp_pass2_workspace_bytes(int64_t length, int32_t dtype, int32_t bins);

/* ---- numeric column path (describe_numeric_1d, describe.py:192-229) ------- */

/* Sample up to `n_sample` rows at evenly spaced positions; writes their
 * order-preserving keys (UINT64_MAX for null/NaN rows) to d_sample. */
int sdp_sample_keys(const sdp_column *col, int32_t n_sample, uint64_t *d_sample,
                    void *stream);

/* sdp_sample_keys of n_cols columns in one launch: d_cols is a DEVICE array of
 * column structs (any numeric dtypes); column c's sample at d_sample + c * n_sample. */
int sdp_sample_keys_batch(const sdp_column *d_cols, int32_t n_cols, int32_t n_sample,
                          uint64_t *d_sample, void *stream);

/* Sort a key sample (<= 16384 keys) and choose one value window per target
 * probability around its sample rank, merged where windows overlap.  Replaces
 * the five `percentile`/`percentile_approx` jobs of describe.py:203-208 (the
 * windows let pass 1 resolve them in the same scan). */
int sdp_quantile_plan(uint64_t *d_sample, int32_t n_sample, const double *probs,
                      int32_t n_probs, int32_t is_float, sdp_qplan *d_plan,
                      void *stream);
/* Narrows the windows of n_cols plans (d_plans, as sdp_quantile_plan_batch
 * wrote them) with a second, larger row sample per column (n_sample2 keys at
 * d_samples2 + i * n_sample2, EMPTY64 = null/NaN): around each probability a
 * window of +-(4 sigma + 2) ranks of the larger sample inside its first-sample
 * window.  A plan whose windows hold more sample keys than one LDS sort (16 K)
 * is left as it was. */
int sdp_quantile_refine_batch(const uint64_t *d_samples2, int32_t n_sample2, int32_t n_cols,
                              const double *d_probs, int32_t n_probs, sdp_qplan *d_plans, void *stream);

/* sdp_quantile_plan of n_cols columns in one launch (one workgroup each):
 * samples [n_cols][n_sample], is_float [n_cols] (device), plans [n_cols]. */
int sdp_quantile_plan_batch(uint64_t *d_samples, int32_t n_sample, int32_t n_cols,
                            const double *probs, int32_t n_probs, const int32_t *d_is_float,
                            sdp_qplan *d_plans, void *stream);

/* Spark 2.x percentile_approx emulation (opt-in; describe(quantile_mode='gk')):
 * the element ApproximatePercentile's QuantileSummaries returns for
 * percentile_approx(c, p, accuracy) (describe.py:205-206) when the column's
 * rows form n_partitions Spark partitions [p*n/P, (p+1)*n/P) whose partial
 * digests are merged in partition order.  float/double columns; nulls and NaN
 * are dropped (na.drop).  d_out[k] = the value for d_probs[k] (NaN when the
 * column has no value); d_status = {error (0 ok, 1/2 summary capacity), values,
 * samples}.  Sequential by nature (one workgroup per partition), so a
 * correctness mode rather than the default exact-rank path. */
int64_t sdp_gk_workspace_bytes(int32_t n_partitions);
int sdp_gk_quantiles(const sdp_column *col, int32_t n_partitions, int32_t accuracy,
                     const double *d_probs, int32_t n_probs, void *d_work, int64_t work_bytes,
                     double *d_out, int64_t *d_status, void *stream);
/* The two halves of sdp_gk_quantiles, for a row-sharded table: every rank
 * builds the digests of its own partitions (sdp_gk_partitions), the digests
 * are gathered into one workspace laid out as sdp_gk_layout describes
 * (out4 = {first partition state, bytes per partition, offset of the sample
 * buffers, samples per buffer}; a partition state is int64 {len, count,
 * buffer, status}), and sdp_gk_merge merges them in partition order. */
int sdp_gk_layout(int32_t n_partitions, int64_t *out4);
int sdp_gk_partitions(const sdp_column *col, int32_t n_partitions, int32_t accuracy, void *d_work,
                      int64_t work_bytes, void *stream);
int sdp_gk_merge(int32_t n_partitions, int32_t accuracy, const double *d_probs, int32_t n_probs,
                 void *d_work, int64_t work_bytes, double *d_out, int64_t *d_status, void *stream);

#define SDP_PASS1_WAVES 4     /* waves per pass-1 workgroup = candidate segments per block */

/* Fused pass 1 over one numeric column (see sdp_pass1_result).  Candidates
 * (keys inside window w) go to wave-private slot ranges: segment
 * s = (w*grid + b)*SDP_PASS1_WAVES + wave holds d_cand[s*slot_capacity ...], its
 * count (clamped to slot_capacity; overflow flagged in w_overflow) in
 * d_cand_counts[s].  slot_capacity 0 = the plan has no windows (moments and min/max
 * only).  flags & SDP_PASS1_INCLUSIVE: the caller has read *d_plan and no used
 * window has its excl_mask bit set -- every window then collects its bound keys
 * as candidates (w_eq_lo = w_eq_hi = 0), which costs fewer compares per row. */
#define SDP_PASS1_INCLUSIVE 1
int sdp_pass1(const sdp_column *col, const sdp_qplan *d_plan, void *d_work,
              int64_t work_bytes, uint64_t *d_cand, uint32_t *d_cand_counts,
              int64_t slot_capacity, int32_t flags, sdp_pass1_result *d_result, void *stream);

/* Grid size sdp_pass1 uses for `length` rows (host-only). */
int32_t sdp_pass1_grid(int64_t length, int32_t dtype);

/* One column of sdp_pass1_batch: sdp_pass1's arguments, with the workspace
 * holding `grid` (= sdp_pass1_grid of the column) block partials. */
typedef struct sdp_pass1_task {
    sdp_column         col;
    const sdp_qplan   *d_plan;
    void              *d_work;
    uint64_t          *d_cand;
    uint32_t          *d_cand_counts;
    int64_t            slot_capacity;
    sdp_pass1_result  *d_result;
    int32_t            grid;
    int32_t            _pad;
} sdp_pass1_task;

/* sdp_pass1 of `ntasks` columns of ONE dtype and one window mode (flags,
 * slot_capacity > 0 or == 0 for all) in two launches (grid: max_grid x ntasks
 * blocks, then one merge block per column) -- wide tables (SURVEY.md §8d C5:
 * 512 columns) pay two launches instead of two per column.  d_tasks lives in
 * device memory.  Replaces the per-column aggregate jobs of describe.py:193-220
 * exactly as sdp_pass1 does. */
int sdp_pass1_batch(const sdp_pass1_task *d_tasks, int32_t ntasks, int32_t dtype, int32_t windowed,
                    int32_t flags, int32_t max_grid, void *stream);

/* Gather `nseg` segments of `slot_capacity` u64 slots (segment s holds
 * d_cand_counts[s] entries) into a dense array, in segment order;
 * *d_out_count receives the total.  d_offsets_work: nseg u64 of workspace.
 * Used for pass-1 candidates (nseg = windows' grid*SDP_PASS1_WAVES) and for the
 * groups sdp_group_dedup leaves at the front of each bucket. */
int sdp_compact_candidates(const uint64_t *d_cand, const uint32_t *d_cand_counts,
                           int32_t nseg, int64_t slot_capacity, uint64_t *d_offsets_work,
                           uint64_t *d_out, uint64_t *d_out_count, void *stream);

/* Radix-select support: 2048-bin histogram of key bits [shift, shift+11) over
 * keys whose bits above shift+11 equal `prefix` (prefix_bits = 64-shift-11). */
int sdp_radix_hist(const uint64_t *d_keys, const uint64_t *d_n, uint64_t prefix,
                   int32_t shift, uint64_t *d_hist, void *stream);
/* Keep keys whose bits >= shift equal `prefix`; append to d_out. */
int sdp_radix_filter(const uint64_t *d_keys, const uint64_t *d_n, uint64_t prefix,
                     int32_t shift, uint64_t *d_out, uint64_t *d_out_n, void *stream);
/* k-th smallest (0-based) of d_keys[:*d_n] (all within [lo_key, hi_key]) into
 * *d_result, UINT64_MAX when k >= *d_n.  Every radix round's digit is chosen on
 * the device, so the call queues its kernels without synchronising; n_cap
 * bounds *d_n.  Single rank (sharded runs all-reduce per round through
 * sdp_radix_hist / sdp_radix_filter).  Replaces the per-percentile Spark jobs
 * of describe.py:203-208. */
int64_t sdp_select_kth_workspace_bytes(int64_t n_cap);
int sdp_select_kth(const uint64_t *d_keys, const uint64_t *d_n, int64_t n_cap, int64_t k,
                   uint64_t lo_key, uint64_t hi_key, void *d_work, int64_t work_bytes,
                   uint64_t *d_result, void *stream);
/* The same select for a row-sharded table, one radix round per call: every
 * rank calls sdp_select_init and sdp_select_hist (round 0's local digit
 * histogram into d_hist[2048]) once, then for round r = 0 .. rounds-1 an
 * all-reduce (sum) of d_hist by the caller on the same stream and
 * sdp_select_step (digit from the summed histogram; unless last, the local
 * keys are filtered and counted by the next digit into d_hist, i.e. the
 * histogram of round r + 1).  rounds = sdp_select_rounds(lo_key, hi_key).  No
 * host round trip per round.  Workspace: sdp_select_kth_workspace_bytes(n_cap). */
int sdp_select_rounds(uint64_t lo_key, uint64_t hi_key);
int sdp_select_init(int64_t k, uint64_t lo_key, uint64_t hi_key, void *d_work, int64_t work_bytes,
                    int64_t n_cap, uint64_t *d_hist, void *stream);
int sdp_select_hist(const uint64_t *d_keys, const uint64_t *d_n, int64_t n_cap, int32_t round,
                    void *d_work, int64_t work_bytes, uint64_t *d_hist, void *stream);
int sdp_select_step(const uint64_t *d_keys, const uint64_t *d_n, int64_t n_cap, int32_t round,
                    int32_t last, void *d_work, int64_t work_bytes, uint64_t *d_hist,
                    uint64_t *d_result, void *stream);
/* Sort <= 16384 keys in place (one workgroup, LDS bitonic). */
int sdp_sort_small(uint64_t *d_keys, const uint64_t *d_n, void *stream);
/* n_sets independent in-place sorts of n_each (<= 16384) keys, one launch
 * (heavy-key samples of all columns). */
int sdp_sort_small_batch(uint64_t *d_keys, int32_t n_each, int32_t n_sets, void *stream);
/* Batched selects: Q independent k-th-key selects (each as sdp_select_kth:
 * keys in [lo_key, hi_key], workspace sdp_select_kth_workspace_bytes(n_cap) at
 * d_work, result written to *d_result) queued with ~2 launches per radix
 * round for all of them -- the per-quantile Spark jobs of describe.py:203-208
 * for every numeric column at once.  d_tasks is a DEVICE array of Q tasks;
 * d_hist holds Q x 2048 u64 digit histograms.  rounds = the max over tasks of
 * sdp_select_rounds(lo, hi).  Row-sharded callers use the split form:
 * sdp_select_batch_init (round 0's local histograms), then per round r an
 * all-reduce of d_hist followed by sdp_select_batch_step(r, last). */
typedef struct sdp_select_task {
    const uint64_t *d_keys;
    const uint64_t *d_n;               /* device count of keys (<= n_cap)           */
    int64_t         n_cap;
    int64_t         k;                 /* 0-based rank                              */
    uint64_t        lo_key, hi_key;
    void           *d_work;
    uint64_t       *d_result;
} sdp_select_task;

int sdp_select_batch(const sdp_select_task *d_tasks, int32_t q, int32_t rounds, uint64_t *d_hist, void *stream);
int sdp_select_batch_init(const sdp_select_task *d_tasks, int32_t q, uint64_t *d_hist, void *stream);
int sdp_select_batch_step(const sdp_select_task *d_tasks, int32_t q, int32_t round, int32_t last, uint64_t *d_hist,
                          void *stream);

/* Batched sdp_compact_candidates: task i copies the d_counts[s] keys of each
 * of its nseg wave segments (cap slots apart in d_cand) densely to d_out and
 * their total to *d_out_count (d_offsets_work: nseg u64). */
typedef struct sdp_compact_task {
    const uint64_t *d_cand;
    const uint32_t *d_counts;
    int64_t         nseg;
    int64_t         cap;
    uint64_t       *d_offsets_work;
    uint64_t       *d_out;
    uint64_t       *d_out_count;
} sdp_compact_task;

int sdp_compact_batch(const sdp_compact_task *d_tasks, int32_t q, int64_t max_nseg, void *stream);

/* Write the order-preserving keys of all na.drop rows (fallback select). */
int sdp_column_keys(const sdp_column *col, uint64_t *d_out, uint64_t *d_out_n,
                    void *stream);

/* The same for the keys lo_key <= key <= hi_key only: the quantile fallback
 * re-collects just the key range a missed rank lies in (between two pass-1
 * windows, or one overflowed window), sized by pass 1's exact counts
 * (replaces the whole-column copy for describe.py:203-208's order statistics). */
int sdp_column_keys_range(const sdp_column *col, uint64_t lo_key, uint64_t hi_key,
                          uint64_t *d_out, uint64_t *d_out_n, void *stream);

/* countDistinct of a column whose na.drop keys are non-decreasing in row
 * order (describe.py:143 for ids / timestamps / pre-sorted data): d_out[4] =
 * {distinct (1 + key changes between consecutive valid rows), violation
 * (a decrease, or a null run too long to walk: group the column instead),
 * first valid key, last valid key (UINT64_MAX when none)}; one read. */
int sdp_sorted_distinct(const sdp_column *col, uint64_t *d_out, void *stream);

/* Fused pass 2: mad, histogram over host-built CASE edges, outlier counts. */
int sdp_pass2(const sdp_column *col, double mean, const double *d_edges,
              int32_t bins, int32_t edges_monotone, double hi_t, double lo_t,
              void *d_work, int64_t work_bytes, sdp_pass2_result *d_result,
              uint64_t *d_hist, void *stream);

/* ---- distinct / value counts (describe.py:143, :250-271) ------------------ */

/* Open-addressing tables: capacity must be a power of two >= 2 x the groups
 * expected; d_slots must be pre-filled by sdp_table_clear. */
int sdp_table_clear(uint64_t *d_slots, uint64_t *d_counts, int64_t capacity,
                    int32_t bytes_keys, void *stream);

/* countDistinct over a fixed-width column: NaN one value, -0.0 == 0.0, nulls
 * ignored.  with_counts != 0 also accumulates per-key row counts (CAT path).
 * d_row_counts (nullable): row i stands for d_row_counts[i] rows (re-aggregating
 * groups received from other ranks).
 * d_stats: [0] groups, [1] rows inserted, [2] rows with key UINT64_MAX. */
int sdp_hash_u64(const sdp_column *col, const uint64_t *d_row_counts, uint64_t *d_slots,
                 uint64_t *d_counts, int64_t capacity, int32_t with_counts,
                 uint64_t *d_stats, void *stream);

/* Same for byte keys; slots hold (24-bit hash tag << 40 | row+1), equal keys
 * are confirmed by byte comparison. d_stats: [0] groups, [1] rows inserted. */
int sdp_hash_bytes(const sdp_bytes_column *col, const uint64_t *d_row_counts,
                   uint64_t *d_slots, uint64_t *d_counts, int64_t capacity,
                   uint64_t *d_stats, void *stream);

/* Top-k groups by (count desc, key asc) from a table built with counts.
 * `bytes_keys` is a flag word: bit0 byte keys (EMPTY slot = 0), bit1 dense
 * group arrays (every slot is a group, as compacted from sdp_group_dedup).
 * Histogram of floor(log2(count)) over occupied slots (64 bins). */
int sdp_table_count_log2_hist(const uint64_t *d_slots, const uint64_t *d_counts,
                              int64_t capacity, int32_t bytes_keys, uint64_t *d_hist,
                              void *stream);
/* Histogram of counts in [lo, lo + 2048*step) with bucket width `step`. */
int sdp_table_count_hist(const uint64_t *d_slots, const uint64_t *d_counts,
                         int64_t capacity, int32_t bytes_keys, uint64_t lo,
                         uint64_t step, uint64_t *d_hist, void *stream);
/* Slot indices with count >= min_count (and <= max_count), appended; with
 * d_counts == NULL (distinct-only table) every group counts as 1. */
int sdp_table_select(const uint64_t *d_slots, const uint64_t *d_counts, int64_t capacity,
                     int32_t bytes_keys, uint64_t min_count, uint64_t max_count,
                     uint64_t *d_out, uint64_t *d_out_n, uint64_t out_capacity,
                     void *stream);
/* Sort <= 16384 selected slots by (count desc, key asc), in place. */
int sdp_sort_groups(uint64_t *d_sel, const uint64_t *d_n, const uint64_t *d_slots,
                    const uint64_t *d_counts, const sdp_bytes_column *bytes_col,
                    void *stream);
/* 8-byte big-endian prefix at byte `offset` of each selected group's key
 * (byte keys) -- radix keys for tie-breaking among equal counts. */
int sdp_group_prefix(const uint64_t *d_sel, const uint64_t *d_n, const uint64_t *d_slots,
                     const sdp_bytes_column *col, int32_t offset, uint64_t *d_out,
                     void *stream);

/* Keep entries of d_sel whose parallel value d_vals[i] is in [lo, hi]. */
int sdp_select_by_value(const uint64_t *d_sel, const uint64_t *d_vals, const uint64_t *d_n,
                        uint64_t lo, uint64_t hi, uint64_t *d_out, uint64_t *d_out_vals,
                        uint64_t *d_out_n, void *stream);

/* Number of set validity bits (non-null rows), accumulated into *d_out. */
int sdp_count_valid(const uint8_t *d_validity, int64_t bit_offset, int64_t length,
                    uint64_t *d_out, void *stream);

/* ---- small-range integral columns (sdp_bitmap.hip) -------------------------
 * countDistinct (describe.py:143) of an integral / date column whose values lie
 * in [lo, lo + range), range <= SDP_BITMAP_MAX_BITS (lo, range from pass-1
 * min/max): one bit per possible value, per-workgroup LDS bitmaps OR-reduced.
 * Nulls are skipped.  d_bitmap (nullable, ceil(range/32) u32): the OR-ed bitmap
 * (ranks all-gather and re-reduce it with sdp_bitmap_reduce); *d_out += the
 * number of set bits (d_out zeroed by the caller). */
#define SDP_BITMAP_MAX_BITS (1 << 20)
int64_t sdp_bitmap_workspace_bytes(int64_t length, int64_t range);
int sdp_distinct_bitmap(const sdp_column *col, int64_t lo, int64_t range, void *d_work,
                        int64_t work_bytes, uint32_t *d_bitmap, uint64_t *d_out, void *stream);
/* OR of nparts bitmaps of nwords words (d_parts[p * nwords + w]) + popcount. */
int sdp_bitmap_reduce(const uint32_t *d_parts, int32_t nparts, int64_t nwords, uint32_t *d_bitmap,
                      uint64_t *d_out, void *stream);

/* ---- two-level hash partitioning with exact offsets (sdp_part.hip) ---------
 * Replaces countDistinct (describe.py:143) and groupBy(c).count()
 * (describe.py:251).  Records are structure-of-arrays: fixed-width keys are one
 * u64 h = mix64(key) in d_k0; byte keys are (k0, k1) = first 16 bytes, zero
 * padded, and meta = len << 40 | row + 1 (strings > 16 bytes: k0 = 64-bit hash,
 * compared byte for byte against the column).
 * Flow: sdp_part_rows phase 0 (per-block histogram of the top b1 hash bits,
 * H1[bucket][block]) -> sdp_scan_u32 -> phase 1 (scatter at exact offsets) ->
 * sdp_part_recs phase 0/1 per chunk with the next b2 bits -> sdp_scan_u32 ->
 * sdp_part_dedup (one workgroup per final bucket, LDS table).
 * d_stats (68 x u64, zeroed): [0] valid rows, [1] fixed-key rows whose
 * h == UINT64_MAX (counted by phase 0, never made records), [2] 64-bit hash collision between
 * different byte strings, [3] LDS table full, [4..67] groups (64 counters). */
#define SDP_PART_MAX_GRID 1024
typedef struct sdp_records {
    uint64_t *d_k0;
    uint64_t *d_k1;     /* byte keys only */
    uint64_t *d_meta;   /* byte keys only */
} sdp_records;
/* Keys counted outside the partitions (n <= 256; n <= 1024 for
 * sdp_part_rows_records): hashes, and for byte keys
 * the (k0, k1, meta) of one representative row; counts go to d_heavy_counts. */
typedef struct sdp_heavy {
    const uint64_t *d_h;
    const uint64_t *d_k0;
    const uint64_t *d_k1;
    const uint64_t *d_meta;
    int32_t n;
    int32_t _pad;
} sdp_heavy;
/* One L1-bucket chunk of records [start, end); its phase-0 histogram entry for
 * sub-bucket s is written at hbase + s * hstride. */
typedef struct sdp_chunk {
    int64_t start, end, hbase, hstride;
} sdp_chunk;

/* sdp_pass2 fused with sdp_part_rows phase 0 (the level-1 count of the
 * column's distinct-count partitioning, describe.py:143): the same pass-2
 * outputs, plus d_part_hist / d_heavy_counts / d_stats exactly as
 * sdp_part_rows(col, NULL, heavy, b1, 0, ...) writes them -- one read of the
 * column instead of two.  Workspace: sdp_pass2_count_workspace_bytes. */
int64_t sdp_pass2_count_workspace_bytes(int64_t length, int32_t bins);
int sdp_pass2_count(const sdp_column *col, double mean, const double *d_edges, int32_t bins,
                    int32_t edges_monotone, double hi_t, double lo_t, void *d_work, int64_t work_bytes,
                    sdp_pass2_result *d_result, uint64_t *d_hist, const sdp_heavy *heavy, int32_t b1,
                    uint32_t *d_part_hist, uint64_t *d_heavy_counts, uint64_t *d_stats, void *stream);

/* One column of sdp_pass2_count_batch: sdp_pass2_count's arguments (the
 * workspace of sdp_pass2_count_workspace_bytes; grid and rows_per_block as
 * sdp_part_rows_per_block gives them for the column's length). */
typedef struct sdp_pass2_task {
    sdp_column         col;
    const double      *d_edges;
    double             mean, hi_t, lo_t;
    void              *d_work;
    sdp_pass2_result  *d_result;
    uint64_t          *d_hist;
    sdp_heavy          heavy;            /* d_h and n used (fixed keys) */
    uint32_t          *d_part_hist;
    uint64_t          *d_heavy_counts;
    uint64_t          *d_stats;
    int64_t            rows_per_block;
    int32_t            bins, edges_monotone, b1, grid;
    /* b1 = -1: the count is sdp_distinct32's level-1 count instead (64
     * buckets of mix32(key - key32_lo) into d_part_hist [64][grid], non-null
     * rows added to d_stats[1]; heavy keys unused) -- its pre-count argument.
     * Only for SDP_F32 and integral dtypes (32-bit key spaces); an SDP_F64
     * task with b1 = -1 counts nothing. */
    int64_t            key32_lo;
} sdp_pass2_task;

/* sdp_pass2_count of `ntasks` columns of one dtype, bin count and edge kind
 * in two launches (wide tables); d_tasks lives in device memory. */
int sdp_pass2_count_batch(const sdp_pass2_task *d_tasks, int32_t ntasks, int32_t dtype, int32_t bins,
                          int32_t edges_monotone, int32_t max_grid, void *stream);


/* Packs the key bytes of n groups -- bytes [d_starts[i], d_starts[i] + d_lens[i])
 * of d_data -- at d_out + d_offs[i] (the sharded string exchange's payload). */
int sdp_gather_bytes(const uint8_t *d_data, const int64_t *d_starts, const int64_t *d_lens,
                     const int64_t *d_offs, int64_t n, uint8_t *d_out, void *stream);

/* Owner order of the sharded exchange (replaces the torch sort + searchsorted +
 * prefix sum + gathers of distributed.py's exchange_fixed_groups /
 * exchange_bytes_groups_batch, round 5).  Group i is entry e = d_sel[i] (or i
 * when d_sel is NULL) of d_keys / d_counts; the groups come out ordered by
 * owner rank, stable within an owner, at positions p = 0 .. n-1.
 *   bcol NULL (fixed keys): owner = ((key * 0x9E3779B97F4A7C15) >> 40 & 0xFFFFFF)
 *     % world; d_out_keys[p] = key, d_out_counts[p] = d_counts[e] (if non-NULL).
 *   bcol set (d_keys = byte-table slots, tag << 40 | row + 1): owner = tag % world;
 *     d_starts[p] / d_lens[p] = the row's key bytes in bcol (lengths < 2^32),
 *     d_meta[2p], d_meta[2p+1] = (length, d_counts[e]), d_offs[0 .. n] = exclusive
 *     prefix of the lengths (the key's place in the owner-major payload).
 * d_per[o] = groups of owner o, d_per[world + o] = their key bytes (0 for fixed
 * keys).  world <= 2048; d_work: sdp_owner_order_workspace_bytes(n, world). */
int64_t sdp_owner_order_workspace_bytes(int64_t n, int32_t world);
int sdp_owner_order(const uint64_t *d_keys, const uint64_t *d_sel, const int64_t *d_counts, int64_t n,
                    int32_t world, const sdp_bytes_column *bcol, uint64_t *d_out_keys, int64_t *d_out_counts,
                    int64_t *d_starts, int64_t *d_lens, int64_t *d_meta, uint64_t *d_offs, int64_t *d_per,
                    void *d_work, int64_t work_bytes, void *stream);

/* Rows per partition workgroup (grid = ceil(length / this)). */
int64_t sdp_part_rows_per_block(int64_t length, int32_t is_bytes);
/* Mean records per final bucket the dedup tables are sized for. */
int64_t sdp_part_bucket_target(int32_t is_bytes, int32_t with_counts);
/* Evenly spaced sample: hashes (UINT64_MAX for nulls) and, for byte keys, the
 * records.  Exactly one of col / bcol is non-NULL (as for every sdp_part_*). */
int sdp_part_sample(const sdp_column *col, const sdp_bytes_column *bcol, int32_t n_sample,
                    uint64_t *d_h, const sdp_records *d_out, void *stream);
/* sdp_part_sample of `ncols` fixed-width columns (d_cols: device array) in one
 * launch; column c's n_sample hashes land in d_h[c * n_sample ..). */
int sdp_part_sample_batch(const sdp_column *d_cols, int32_t ncols, int32_t n_sample, uint64_t *d_h,
                          void *stream);
/* phase 0: d_hist[b * grid + block] (u32) + heavy counts + d_stats[0];
 * phase 1: records scattered to d_out at d_offsets (exclusive scan of d_hist). */
int sdp_part_rows(const sdp_column *col, const sdp_bytes_column *bcol, const sdp_heavy *heavy,
                  int32_t b1, int32_t phase, uint32_t *d_hist, const uint64_t *d_offsets,
                  const sdp_records *d_out, uint64_t *d_heavy_counts, uint64_t *d_stats,
                  void *stream);

/* One column of sdp_part_rows_batch (phase 1, fixed keys): the level-1 scatter
 * of `col` with its scanned counts d_offsets into d_out; grid and
 * rows_per_block as sdp_part_rows_per_block gives them. */
typedef struct sdp_rows_task {
    sdp_column        col;
    sdp_heavy         heavy;            /* d_h and n used */
    const uint64_t   *d_offsets;
    uint64_t         *d_out;
    int64_t           rows_per_block;
    int32_t           b1, grid;
} sdp_rows_task;

/* The level-1 scatters of `ntasks` columns of one dtype (every fixed-width
 * dtype but SDP_BOOL) in one launch (wide tables); d_tasks lives in device
 * memory, so the caller checks each task as sdp_part_rows does (16-byte aligned
 * values, heavy.n <= 256, grid <= max_grid). */
int sdp_part_rows_batch(const sdp_rows_task *d_tasks, int32_t ntasks, int32_t dtype, int32_t max_grid, void *stream);
/* Byte columns, one read of the strings (replaces sdp_part_rows phase 0 + 1 for
 * bcol): every wave of every workgroup compacts the records of its strip of
 * rows to d_out at the strip's first row position (d_out holds length records),
 * counts the strip's level-1 buckets into d_hist[b * nchunks + chunk] and
 * writes d_chunks[chunk] = {strip start, start + records, chunk, nchunks};
 * heavy counts (up to 1024 heavy keys) and d_stats[0] as sdp_part_rows
 * phase 0.  The level-1 scatter
 * is then sdp_part_recs(d_out, 1, d_chunks, nchunks, 0, b1, 1, ...) with the
 * exclusive scan of d_hist.  nchunks = sdp_part_records_chunks(length). */
int64_t sdp_part_records_chunks(int64_t length);
int sdp_part_rows_records(const sdp_bytes_column *bcol, const sdp_heavy *heavy, int32_t b1,
                          uint32_t *d_hist, sdp_chunk *d_chunks, const sdp_records *d_out,
                          uint64_t *d_heavy_counts, uint64_t *d_stats, void *stream);
/* L1 records -> sub-buckets by hash bits [64-b1-b2, 64-b1). */
int sdp_part_recs(const sdp_records *in, int32_t is_bytes, const sdp_chunk *d_chunks,
                  int64_t nchunks, int32_t b1, int32_t b2, int32_t phase, uint32_t *d_hist,
                  const uint64_t *d_offsets, const sdp_records *out, void *stream);
/* Final bucket f = records [d_starts[f], d_starts[f+1]).  Distinct only (fixed
 * keys, !with_counts): group totals in d_stats; buckets are sized for
 * sdp_part_bucket_target distinct keys, or (with_counts == 2) for 4 x that
 * when the hash bits run out (more than 2^30 rows on one device); with_counts
 * bit 4 (distinct only) claims slots with a single CAS (near-unique keys); a
 * non-NULL d_ngroups then receives every bucket's group count (one launch over
 * several columns' buckets).  Otherwise the groups of f go to
 * d_out_key/d_out_cnt at [d_starts[f], + d_ngroups[f]): fixed keys as the
 * order-preserving u64 key, byte keys as (hash tag << 40 | row + 1). */
int sdp_part_dedup(const sdp_records *in, int32_t is_bytes, const sdp_bytes_column *bcol,
                   const uint64_t *d_starts, int64_t nbuckets, int32_t with_counts,
                   uint64_t *d_out_key, uint64_t *d_out_cnt, uint32_t *d_ngroups,
                   uint64_t *d_stats, void *stream);
/* countDistinct (describe.py:143) of a column whose keys fit 32 bits: float32
 * (NaN one value, -0.0 == 0.0), or an integral column with imax - imin < 2^32
 * (key = v - lo, lo = imin).  Nulls are skipped.  h = mix32(key) (a bijection)
 * is partitioned as 4-byte records into 64 x 64 buckets (the level-1 scatter
 * also counts the level-2 buckets, so no count pass of records) and every
 * final bucket's low 20 bits are set in a 128 KB LDS bitmap: no hash table.
 * Stream-ordered, no host round trip.  d_out[0] += distinct values, d_out[1]
 * += non-null rows (d_out zeroed by the caller).  Workspace:
 * sdp_distinct32_workspace_bytes(length) (two 4-byte record buffers + scans). */
int64_t sdp_distinct32_workspace_bytes(int64_t length);
/* d_hist1 (nullable): the level-1 counts [64][grid] already taken (by
 * sdp_pass2_count_batch with b1 = -1, which also added the rows to d_out[1]):
 * the column is then read once here instead of twice. */
int sdp_distinct32(const sdp_column *col, int64_t lo, const uint32_t *d_hist1, void *d_work, int64_t work_bytes,
                   uint64_t *d_out, void *stream);
/* ---- level 2 without a count pass (round 6) --------------------------------
 * One workgroup owns a whole level-1 bucket and splits its records by hash
 * bits [64-b1-b2, 64-b1) into blocks of SDP_L2_BLOCK records that it hands
 * out in LDS from the bucket's block region: no count pass and no offsets.
 * Workgroup g (nwg of them) walks the segments d_segs[d_soff[g] ..
 * d_soff[g+1]): segment = records [start, end) of `in` belonging to bucket
 * hbase; hstride = the region's first block (bits 0-31; a multiple of 8) |
 * bit 32: first segment of the bucket | bit 33: its last | R (bits 40-63).
 * A bucket's segments are consecutive in one workgroup's list.
 * Sub-bucket j of a bucket fills a run of R blocks (hstride bits 40-63) at
 * region block + j * R, then overflow blocks after the bucket's 2^b2 runs (the
 * region holds 2^b2 * R + ceil(S / SDP_L2_BLOCK) + 8 blocks for S records).
 * Output: block b holds out[b * SDP_L2_BLOCK ..); final bucket
 * f = bucket * 2^b2 + j is described by d_desc[f * SDP_L2_DESC_W ..] = {records
 * n, first overflow-list entry l, run block, run records rl}: record r < rl
 * lies at run block * SDP_L2_BLOCK + r, record r >= rl at block
 * d_list[l + (r - rl) / SDP_L2_BLOCK], slot r % SDP_L2_BLOCK.  d_list needs 32
 * entries of padding past the last block.  d_bmeta: scratch, one u64 per
 * block.  2^b2 <= 1024 (fixed keys) / 512 (byte keys). */
#define SDP_L2_DESC_W 4
typedef struct sdp_blocks {
    uint32_t *d_desc;       /* SDP_L2_DESC_W u32 per final bucket      */
    uint32_t *d_list;       /* block ids, in order within each bucket */
} sdp_blocks;
int sdp_part_l2_blocks(const sdp_records *in, int32_t is_bytes, const sdp_chunk *d_segs, const int64_t *d_soff,
                       int32_t nwg, int32_t b1, int32_t b2, const sdp_records *out, uint64_t *d_bmeta,
                       const sdp_blocks *blk, void *stream);
/* Test builds only (-DSDP_DEBUG_BOUNDS): bounds flags of the block layout. */
int sdp_debug_bounds(uint64_t cap_rec, uint64_t cap_blk, uint64_t *flags_out, int32_t reset);
/* sdp_part_dedup over the final buckets of sdp_part_l2_blocks (the same modes
 * and outputs; groups of f go to the block positions of its records 0 ..
 * d_ngroups[f]). */
int sdp_part_dedup_blocks(const sdp_records *in, int32_t is_bytes, const sdp_bytes_column *bcol,
                          const sdp_blocks *blk, int64_t nbuckets, int32_t with_counts,
                          uint64_t *d_out_key, uint64_t *d_out_cnt, uint32_t *d_ngroups,
                          uint64_t *d_stats, void *stream);
/* sdp_part_compact over block-laid buckets. */
int sdp_part_compact_blocks(const uint64_t *d_src_a, const uint64_t *d_src_b, const sdp_blocks *blk,
                            const uint32_t *d_ngroups, const uint64_t *d_out_offsets, int64_t nbuckets,
                            uint64_t *d_dst_a, uint64_t *d_dst_b, void *stream);
/* Pack the per-bucket groups: src[d_starts[f] ..+ngroups[f]) -> dst[d_out_offsets[f] ..). */
int sdp_part_compact(const uint64_t *d_src_a, const uint64_t *d_src_b, const uint64_t *d_starts,
                     const uint32_t *d_ngroups, const uint64_t *d_out_offsets, int64_t nbuckets,
                     uint64_t *d_dst_a, uint64_t *d_dst_b, void *stream);
/* Exclusive scan of n u32 counts into n + 1 u64 offsets (d_out[n] = total). */
int64_t sdp_scan_workspace_bytes(int64_t n);
int sdp_scan_u32(const uint32_t *d_in, int64_t n, uint64_t *d_out, void *d_work,
                 int64_t work_bytes, void *stream);

/* ---- first rows (describe.py:276 limit(1), :282 limit(50)) ---------------- */
/* Indices of the first k rows that survive na.drop (null, and NaN for floats). */
int sdp_first_valid(const sdp_column *col, int32_t k, int64_t *d_idx, int64_t *d_found,
                    void *stream);

/* ---- Pearson matrix (utils.py:20-36) -------------------------------------- */
/* Listwise-deletion row mask over `ncols` columns (host array): bit r set iff
 * every column is valid and (where check_nan[i]) not NaN at row r.  d_keep has
 * ceil(length/32) uint32 words; d_work >= sdp_gram_workspace_bytes.  The column
 * descriptors are staged through d_work; this call synchronises the stream once
 * (the host descriptor copy), as does sdp_gram. */
int sdp_rowmask(const sdp_column *cols, const int32_t *check_nan, int32_t ncols,
                void *d_work, int64_t work_bytes, uint32_t *d_keep, void *stream);
/* Shifted Gram: G[i][j] = sum_r keep_r (x_ir - K_i)(x_jr - K_j), s[i] = sum_r keep_r
 * (x_ir - K_i), n = sum keep_r, on v_mfma_f64_16x16x4_f64.  Writes G (ncols^2,
 * row-major, upper and lower), s (ncols) and n (1, as double). */
int64_t sdp_gram_workspace_bytes(int64_t length, int32_t ncols);
int sdp_gram(const sdp_column *cols, int32_t ncols, const uint32_t *d_keep,
             const double *d_shift, void *d_work, int64_t work_bytes,
             double *d_gram, double *d_colsum, double *d_n, void *stream);

/* ---- coarse entry points: one call per reference operation group ----------
 * SURVEY.md §8(b)'s contract.  Each is a C++ orchestrator (sdp_api.cpp) over the
 * kernels above for ONE column (or one set of columns) on one device, so a host
 * in any language gets a statistic from this header alone (INTEGRATION.md §2
 * shows a C caller).  Common rules:
 *   - d_work: ONE caller-owned device workspace of at least the matching
 *     *_workspace_bytes(...) bytes (the library carves it up; nothing is
 *     allocated or freed);
 *   - work is queued on `stream`; entries marked SYNC read small results back
 *     between stages (bucket starts, group counts, count thresholds) and so
 *     synchronise `stream` -- their outputs are HOST structs; the others are
 *     fully stream-ordered and write DEVICE outputs;
 *   - NaN is one value (countDistinct / groupBy), -0.0 groups with 0.0, nulls
 *     are ignored (na.drop), as Spark does. */

/* describe.py:233 (date / timestamp min and max over na.drop, and the count of
 * describe.py:144): one pass, stream-ordered.  Integral / date (int32 days) /
 * timestamp (int64) columns fill imin/imax; float columns dmin/dmax. */
typedef struct sdp_minmax_result {
    uint64_t count;                    /* valid, non-NaN rows                      */
    int64_t  imin, imax;
    double   dmin, dmax;
} sdp_minmax_result;
int64_t sdp_minmax_workspace_bytes(int64_t length, int32_t dtype);
int sdp_minmax_int(const sdp_column *col, void *d_work, int64_t work_bytes, sdp_minmax_result *d_out,
                   void *stream);

/* describe.py:203-208: the percentiles of one numeric column at the host
 * probabilities probs[0 .. n_probs) (n_probs <= 16), as describe() reports
 * them -- integral columns: Spark `percentile` (linear interpolation at
 * (N-1) p between the exact order statistics); float columns: the element of
 * rank ceil(p N) (`percentile_approx`'s answer within its rank bound; p <=
 * 1e-4 -> rank 1, p >= 1 - 1e-4 -> rank N).  N = na.drop rows; d_out[i] = NaN
 * when N = 0.  Exact radix selects over the column's keys; stream-ordered (the
 * ranks are computed on the device from the device-side N). */
#define SDP_QUANTILES_MAX 16
int64_t sdp_quantiles_workspace_bytes(int64_t length, int32_t n_probs);
int sdp_quantiles(const sdp_column *col, const double *probs, int32_t n_probs, void *d_work, int64_t work_bytes,
                  double *d_out, void *stream);

/* describe.py:143: countDistinct of one column (exactly one of col / bcol
 * non-NULL; byte keys compared bytewise).  SYNC.  Path: integral ranges <=
 * 2^20 -> LDS bitmaps; >= 64 K rows -> two-level hash partitioning with exact
 * offsets + LDS de-duplication (sdp_part_*); otherwise, or when the
 * partitioning reports a collision / full table, the global table. */
typedef struct sdp_distinct_result {
    uint64_t distinct;                 /* groups among non-null rows               */
    uint64_t rows;                     /* non-null rows                            */
    int32_t  path;                     /* 0 bitmap, 1 partitioned, 2 global table  */
    int32_t  _pad;
} sdp_distinct_result;
int64_t sdp_distinct_workspace_bytes(int64_t length, int32_t is_bytes);
int sdp_hash_distinct_count(const sdp_column *col, const sdp_bytes_column *bcol, void *d_work, int64_t work_bytes,
                            sdp_distinct_result *h_out, void *stream);

/* describe.py:251-263: value counts of one column (groupBy(c).count() over
 * na.drop rows) and the first k groups by (count desc, key asc) -- the
 * orderBy + limit(50) of the reference, with the tie order defined.  SYNC.
 * h_top[0 .. h_out->n_top) receive {key, count}: fixed-width columns the
 * order-preserving 64-bit key (key_f64 / key_i64 inverses: sign-flip for
 * integers; sign-flip / invert for floats), byte columns the 0-based row index
 * of one row holding the value.  ***Other Values*** = rows - sum(counts);
 * ***Other Values Distinct Count*** = groups - n_top.  0 <= k <= SDP_GSORT_MAX
 * (SDP_EINVAL otherwise: the candidates are ordered by one sort launch). */
typedef struct sdp_topk_entry {
    uint64_t key;
    uint64_t count;
} sdp_topk_entry;
typedef struct sdp_topk_result {
    uint64_t groups;                   /* distinct values among non-null rows      */
    uint64_t rows;                     /* non-null rows                            */
    int32_t  n_top;                    /* min(k, groups)                           */
    int32_t  path;                     /* 1 partitioned, 2 global table            */
} sdp_topk_result;
int64_t sdp_value_counts_workspace_bytes(int64_t length, int32_t is_bytes);
int sdp_value_counts_topk(const sdp_column *col, const sdp_bytes_column *bcol, int32_t k, void *d_work,
                          int64_t work_bytes, sdp_topk_result *h_out, sdp_topk_entry *h_top, void *stream);

/* utils.py:20-36: the Pearson matrix of ncols numeric columns (host array of
 * column structs) with listwise deletion (a row counts only if every column is
 * valid and, for float columns, not NaN), rho[i][j] = C_ij / sqrt(C_ii C_jj)
 * from the shifted fp64 Gram on MFMA (C = G - s s^T / n, shift = each column's
 * sample median).  d_corr: ncols x ncols row-major doubles (device); *d_n: the
 * rows kept (device double).  SYNC (the column descriptors are staged once). */
int64_t sdp_pearson_workspace_bytes(int64_t length, int32_t ncols);
int sdp_gram_f64(const sdp_column *cols, int32_t ncols, void *d_work, int64_t work_bytes, double *d_corr,
                 double *d_n, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SDP_H */
