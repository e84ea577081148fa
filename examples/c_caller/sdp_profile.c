/*
 * sdp_profile.c -- a non-Python host computing every statistic group of
 * describe() (/root/reference/spark_df_profiling/describe.py) through the C ABI
 * of libsdp.so (include/sdp.h) alone: no Python, no torch.
 *
 *   sdp_quantiles            describe.py:203-208  5 percentiles
 *   sdp_pass1                describe.py:144,193-201,220  count, moments, zeros
 *   sdp_pass2                describe.py:38-63,215-223  histogram, mad, outliers
 *   sdp_hash_distinct_count  describe.py:143  countDistinct
 *   sdp_value_counts_topk    describe.py:251-263  top-50 + Other rows
 *   sdp_minmax_int           describe.py:233  date min / max
 *   sdp_gram_f64             utils.py:20-36  Pearson matrix
 *
 * Input: a manifest, one column per line (raw little-endian files; "-" = no
 * validity bitmap, i.e. every row valid):
 *   num  NAME DTYPE ROWS VALUES VALIDITY        (DTYPE: enum sdp_dtype code)
 *   date NAME ROWS VALUES(int32 days) VALIDITY
 *   str  NAME ROWS OFFSETS(int64) DATA VALIDITY
 * Output: one JSON object on stdout.  Build: make -C examples/c_caller
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sdp.h"

#define CHECK_HIP(x)                                                                  \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                  \
        }                                                                             \
    } while (0)
#define CHECK_SDP(x)                                                                  \
    do {                                                                              \
        int r_ = (x);                                                                 \
        if (r_) {                                                                     \
            fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, r_, sdp_last_error()); \
            exit(3);                                                                  \
        }                                                                             \
    } while (0)

static const double PROBS[5] = {0.05, 0.25, 0.5, 0.75, 0.95};
enum { BINS = 10, TOPK = 50 };

static void *read_file(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void *buf = malloc(n + 16);
    if (n && fread(buf, 1, n, f) != (size_t)n) { perror(path); exit(1); }
    memset((char *)buf + n, 0, 16);
    fclose(f);
    if (len) *len = (size_t)n;
    return buf;
}

/* host buffer -> new device buffer (+16 readable padding bytes) */
static void *upload(const void *h, size_t n) {
    void *d = NULL;
    CHECK_HIP(hipMalloc(&d, n + 16));
    CHECK_HIP(hipMemset(d, 0, n + 16));
    if (n) CHECK_HIP(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
    return d;
}

static void *dev_alloc(int64_t n) {
    void *d = NULL;
    CHECK_HIP(hipMalloc(&d, n > 0 ? (size_t)n : 16));
    return d;
}

static void json_double(double v) {
    if (isnan(v)) printf("NaN");
    else if (isinf(v)) printf(v > 0 ? "Infinity" : "-Infinity");
    else printf("%.17g", v);
}

static void json_string(const char *s, size_t n) {
    putchar('"');
    for (size_t i = 0; i < n; ++i) {
        unsigned char c = (unsigned char)s[i];
        if (c == '"' || c == '\\') printf("\\%c", c);
        else if (c < 0x20) printf("\\u%04x", c);
        else putchar(c);
    }
    putchar('"');
}

static const uint8_t *load_validity(const char *path, void **dev) {
    if (strcmp(path, "-") == 0) { *dev = NULL; return NULL; }
    size_t n;
    uint8_t *h = read_file(path, &n);
    *dev = upload(h, n);
    return h;
}

static int dtype_is_float(int dt) { return dt == SDP_F32 || dt == SDP_F64; }

/* Spark Average / CentralMomentAgg from the shifted power sums (engine.moments) */
static void numeric_column(const char *name, sdp_column col, hipStream_t s, int first) {
    int is_float = dtype_is_float(col.dtype);
    /* percentiles first: the median is pass 1's shift K */
    int64_t qw = sdp_quantiles_workspace_bytes(col.length, 5);
    void *work = dev_alloc(qw);
    double *d_q = dev_alloc(5 * sizeof(double)), q[5];
    CHECK_SDP(sdp_quantiles(&col, PROBS, 5, work, qw, d_q, s));
    CHECK_HIP(hipMemcpyAsync(q, d_q, sizeof q, hipMemcpyDeviceToHost, s));
    CHECK_HIP(hipStreamSynchronize(s));
    CHECK_HIP(hipFree(work));
    /* pass 1 without windows, shifted by the median */
    sdp_qplan plan;
    memset(&plan, 0, sizeof plan);
    plan.shift = isfinite(q[2]) ? q[2] : 0.0;
    sdp_qplan *d_plan = upload(&plan, sizeof plan);
    int64_t pw = sdp_pass1_workspace_bytes(col.length, col.dtype);
    work = dev_alloc(pw);
    sdp_pass1_result *d_r1 = dev_alloc(sizeof(sdp_pass1_result)), r1;
    CHECK_SDP(sdp_pass1(&col, d_plan, work, pw, NULL, NULL, 0, 0, d_r1, s));
    CHECK_HIP(hipMemcpyAsync(&r1, d_r1, sizeof r1, hipMemcpyDeviceToHost, s));
    CHECK_HIP(hipStreamSynchronize(s));
    CHECK_HIP(hipFree(work));
    double n = (double)r1.count, K = r1.shift;
    double s1 = r1.s1_hi + r1.s1_lo, s2 = r1.s2, s3 = r1.s3_hi + r1.s3_lo, s4 = r1.s4;
    double dsum = (double)((long double)K * (long double)r1.count + (long double)r1.s1_hi + (long double)r1.s1_lo);
    double mean = n > 0 ? dsum / n : NAN;
    double m = n > 0 ? s1 / n : 0.0;
    double M2 = n > 0 ? s2 - s1 * s1 / n : 0.0;
    double M3 = s3 - 3.0 * m * s2 + 2.0 * n * m * m * m;
    double M4 = s4 - 4.0 * m * s3 + 6.0 * m * m * s2 - 3.0 * n * m * m * m * m;
    if (M2 < 0) M2 = 0;
    double var = n > 1 ? M2 / (n - 1.0) : NAN, sd = n > 1 ? sqrt(var) : NAN;
    double skew = M2 == 0 ? NAN : sqrt(n) * M3 / sqrt(M2 * M2 * M2);
    double kurt = M2 == 0 ? NAN : n * M4 / (M2 * M2) - 3.0;
    double mn = is_float ? r1.dmin : (double)r1.imin, mx = is_float ? r1.dmax : (double)r1.imax;
    double sum = is_float ? dsum : (double)r1.isum;
    /* pass 2: edges accumulated as describe.py:40-45 does, thresholds :222-223 */
    double edges[BINS + 1], w = (mx - mn) / (double)BINS;
    edges[0] = mn;
    for (int i = 0; i < BINS; ++i) edges[i + 1] = edges[i] + w;
    int mono = 1;
    for (int i = 0; i < BINS; ++i) mono &= isfinite(edges[i]) && (i == 0 || edges[i - 1] <= edges[i]);
    double q1 = q[1], q3 = q[3];
    double hi_t = q3 + 2 * (q3 - q1), lo_t = q1 - 2 * (q3 - q1);
    double *d_edges = upload(edges, BINS * sizeof(double));
    int64_t p2w = sdp_pass2_workspace_bytes(col.length, col.dtype, BINS);
    work = dev_alloc(p2w);
    sdp_pass2_result *d_r2 = dev_alloc(sizeof(sdp_pass2_result)), r2;
    uint64_t *d_hist = dev_alloc(BINS * 8), hist[BINS];
    CHECK_SDP(sdp_pass2(&col, mean, d_edges, BINS, mono, hi_t, lo_t, work, p2w, d_r2, d_hist, s));
    CHECK_HIP(hipMemcpyAsync(&r2, d_r2, sizeof r2, hipMemcpyDeviceToHost, s));
    CHECK_HIP(hipMemcpyAsync(hist, d_hist, sizeof hist, hipMemcpyDeviceToHost, s));
    CHECK_HIP(hipStreamSynchronize(s));
    CHECK_HIP(hipFree(work));
    /* countDistinct */
    int64_t dw = sdp_distinct_workspace_bytes(col.length, 0);
    work = dev_alloc(dw);
    sdp_distinct_result dr;
    CHECK_SDP(sdp_hash_distinct_count(&col, NULL, work, dw, &dr, s));
    CHECK_HIP(hipFree(work));

    printf("%s\"", first ? "" : ",");
    printf("%s\": {\"kind\": \"num\", \"count\": %llu, \"n_valid\": %llu, \"n_zeros\": %llu, \"distinct\": %llu, "
           "\"distinct_path\": %d, \"min\": ", name, (unsigned long long)r1.count, (unsigned long long)r1.n_valid,
           (unsigned long long)r1.n_zero, (unsigned long long)dr.distinct, dr.path);
    json_double(mn);
    printf(", \"max\": "); json_double(mx);
    printf(", \"sum\": "); json_double(sum);
    printf(", \"mean\": "); json_double(mean);
    printf(", \"variance\": "); json_double(var);
    printf(", \"std\": "); json_double(sd);
    printf(", \"skewness\": "); json_double(skew);
    printf(", \"kurtosis\": "); json_double(kurt);
    printf(", \"mad\": "); json_double(n > 0 ? r2.abs_dev_sum / n : NAN);
    printf(", \"high_idx\": %llu, \"low_idx\": %llu, \"quantiles\": [", (unsigned long long)r2.n_high,
           (unsigned long long)r2.n_low);
    for (int i = 0; i < 5; ++i) { if (i) printf(", "); json_double(q[i]); }
    printf("], \"hist\": [");
    for (int i = 0; i < BINS; ++i) printf("%s%llu", i ? ", " : "", (unsigned long long)hist[i]);
    printf("]}");
    CHECK_HIP(hipFree(d_q)); CHECK_HIP(hipFree(d_plan)); CHECK_HIP(hipFree(d_r1)); CHECK_HIP(hipFree(d_edges));
    CHECK_HIP(hipFree(d_r2)); CHECK_HIP(hipFree(d_hist));
}

static void date_column(const char *name, sdp_column col, hipStream_t s, int first) {
    int64_t mw = sdp_minmax_workspace_bytes(col.length, col.dtype);
    void *work = dev_alloc(mw);
    sdp_minmax_result *d_mm = dev_alloc(sizeof(sdp_minmax_result)), mm;
    CHECK_SDP(sdp_minmax_int(&col, work, mw, d_mm, s));
    CHECK_HIP(hipMemcpyAsync(&mm, d_mm, sizeof mm, hipMemcpyDeviceToHost, s));
    CHECK_HIP(hipStreamSynchronize(s));
    CHECK_HIP(hipFree(work));
    int64_t dw = sdp_distinct_workspace_bytes(col.length, 0);
    work = dev_alloc(dw);
    sdp_distinct_result dr;
    CHECK_SDP(sdp_hash_distinct_count(&col, NULL, work, dw, &dr, s));
    CHECK_HIP(hipFree(work));
    printf("%s\"%s\": {\"kind\": \"date\", \"count\": %llu, \"min\": %lld, \"max\": %lld, \"distinct\": %llu}",
           first ? "" : ",", name, (unsigned long long)mm.count, (long long)mm.imin, (long long)mm.imax,
           (unsigned long long)dr.distinct);
    CHECK_HIP(hipFree(d_mm));
}

static void string_column(const char *name, sdp_bytes_column bc, const int64_t *h_offs, const char *h_data,
                          hipStream_t s, int first) {
    int64_t vw = sdp_value_counts_workspace_bytes(bc.length, 1);
    void *work = dev_alloc(vw);
    sdp_topk_result tr;
    sdp_topk_entry top[TOPK];
    CHECK_SDP(sdp_value_counts_topk(NULL, &bc, TOPK, work, vw, &tr, top, s));
    CHECK_HIP(hipFree(work));
    int64_t dw = sdp_distinct_workspace_bytes(bc.length, 1);
    work = dev_alloc(dw);
    sdp_distinct_result dr;
    CHECK_SDP(sdp_hash_distinct_count(NULL, &bc, work, dw, &dr, s));
    CHECK_HIP(hipFree(work));
    printf("%s\"%s\": {\"kind\": \"str\", \"rows\": %llu, \"groups\": %llu, \"distinct\": %llu, \"path\": %d, "
           "\"top\": [", first ? "" : ",", name, (unsigned long long)tr.rows, (unsigned long long)tr.groups,
           (unsigned long long)dr.distinct, tr.path);
    for (int i = 0; i < tr.n_top; ++i) {
        const int64_t r = (int64_t)top[i].key;
        printf("%s[", i ? ", " : "");
        json_string(h_data + h_offs[r], (size_t)(h_offs[r + 1] - h_offs[r]));
        printf(", %llu]", (unsigned long long)top[i].count);
    }
    printf("]}");
}

int main(int argc, char **argv) {
    if (argc != 2) {
        fprintf(stderr, "usage: %s MANIFEST\n", argv[0]);
        return 1;
    }
    FILE *m = fopen(argv[1], "r");
    if (!m) { perror(argv[1]); return 1; }
    hipStream_t s;
    CHECK_HIP(hipStreamCreate(&s));
    sdp_column num[256];
    char numname[256][128];
    int nnum = 0, first = 1;
    char kind[16], name[128], a[1024], b[1024], c[1024];
    int dtype;
    long long rows;
    printf("{\"version\": \"%s\", \"columns\": {", sdp_version());
    while (fscanf(m, "%15s", kind) == 1) {
        void *dval;
        if (strcmp(kind, "num") == 0) {
            if (fscanf(m, "%127s %d %lld %1023s %1023s", name, &dtype, &rows, a, b) != 5) return 1;
            size_t n;
            void *h = read_file(a, &n);
            sdp_column col = {upload(h, n), NULL, 0, rows, dtype, 0};
            free(h);
            free((void *)load_validity(b, &dval));
            col.d_validity = dval;
            numeric_column(name, col, s, first);
            if (nnum < 256) { num[nnum] = col; snprintf(numname[nnum], 128, "%s", name); ++nnum; }
        } else if (strcmp(kind, "date") == 0) {
            if (fscanf(m, "%127s %lld %1023s %1023s", name, &rows, a, b) != 4) return 1;
            size_t n;
            void *h = read_file(a, &n);
            sdp_column col = {upload(h, n), NULL, 0, rows, SDP_I32, 0};
            free(h);
            free((void *)load_validity(b, &dval));
            col.d_validity = dval;
            date_column(name, col, s, first);
        } else if (strcmp(kind, "str") == 0) {
            if (fscanf(m, "%127s %lld %1023s %1023s %1023s", name, &rows, a, b, c) != 5) return 1;
            size_t no, nd;
            int64_t *offs = read_file(a, &no);
            char *data = read_file(b, &nd);
            sdp_bytes_column bc = {upload(data, nd), upload(offs, no), NULL, 0, rows, 8, 0};
            free((void *)load_validity(c, &dval));
            bc.d_validity = dval;
            string_column(name, bc, offs, data, s, first);
            free(offs);
            free(data);
        } else {
            fprintf(stderr, "unknown column kind %s\n", kind);
            return 1;
        }
        first = 0;
    }
    printf("}");
    if (nnum > 0) {
        /* the Pearson matrix of every numeric column (utils.py:20-36) */
        int64_t gw = sdp_pearson_workspace_bytes(num[0].length, nnum);
        void *work = dev_alloc(gw);
        double *d_corr = dev_alloc((int64_t)nnum * nnum * 8), *d_n = dev_alloc(8);
        CHECK_SDP(sdp_gram_f64(num, nnum, work, gw, d_corr, d_n, s));
        double *corr = malloc((size_t)nnum * nnum * 8), kept;
        CHECK_HIP(hipMemcpyAsync(corr, d_corr, (size_t)nnum * nnum * 8, hipMemcpyDeviceToHost, s));
        CHECK_HIP(hipMemcpyAsync(&kept, d_n, 8, hipMemcpyDeviceToHost, s));
        CHECK_HIP(hipStreamSynchronize(s));
        printf(", \"corr_rows\": %.0f, \"corr_names\": [", kept);
        for (int i = 0; i < nnum; ++i) printf("%s\"%s\"", i ? ", " : "", numname[i]);
        printf("], \"corr\": [");
        for (int i = 0; i < nnum * nnum; ++i) { if (i) printf(", "); json_double(corr[i]); }
        printf("]");
        free(corr);
    }
    printf("}\n");
    fclose(m);
    return 0;
}
