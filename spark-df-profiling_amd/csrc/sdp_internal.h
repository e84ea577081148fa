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
