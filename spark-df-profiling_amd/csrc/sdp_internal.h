// sdp_internal.h -- C++ entry points shared between libsdp's translation units
// (not part of the C ABI in include/sdp.h).
#pragma once
#include <stdint.h>

// sdp_select_kth with the rank optionally read from device memory (d_k
// non-NULL: *d_k replaces k), so a caller whose rank depends on a device-side
// count (sdp_quantiles) queues the select without a host round trip.
int select_kth_dev(const uint64_t *d_keys, const uint64_t *d_n, int64_t n_cap, int64_t k, const int64_t *d_k,
                   uint64_t lo_key, uint64_t hi_key, void *d_work, int64_t work_bytes, uint64_t *d_result,
                   void *stream);

// pass2_merge_batch_kernel over `ntasks` sdp_pass2_task (device array): the
// per-column merge of block partials that sdp_pass2_count_batch ends with
// (sdp_pass2_gram reuses it).
int launch_pass2_merge_batch(const struct sdp_pass2_task *d_tasks, int ntasks, void *stream);
// gram_reduce_kernel<16> over S row-block partials of one 16-column tile
// (part_g [S][256], part_cs [S][16], part_n [S]) -> G (ncols x ncols), column sums, kept rows.
int launch_gram_reduce16(const double *part_g, const double *part_cs, const double *part_n, int ncols, int S,
                         double *d_gram, double *d_colsum, double *d_n, void *stream);
