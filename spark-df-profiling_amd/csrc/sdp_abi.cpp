// sdp_abi.cpp -- error reporting and version for the libsdp C ABI.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include "sdp_common.h"

namespace sdp {

static thread_local char g_err[512] = "";

int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(SDP_EHIP, "%s: %s", what, hipGetErrorString(e));
    return SDP_OK;
}

bool aligned16(const void *p) { return (((uintptr_t)p) & 15u) == 0; }

}  // namespace sdp

extern "C" const char *sdp_last_error(void) { return sdp::g_err; }
extern "C" const char *sdp_version(void) { return "sdp-mi355x 0.6.0 (gfx950)"; }

// The layout this library was built with (include/sdp.h, SDP_ABI_VERSION): the
// host binding refuses a library whose structs, record layout or grouping
// policy differ from its own view.
extern "C" int sdp_layout_info(sdp_layout *out) {
    if (out == nullptr) return sdp::set_error(SDP_EINVAL, "sdp_layout_info: out");
    *out = sdp_layout{};
    out->abi_version = SDP_ABI_VERSION;
    out->n_sizes = SDP_LAYOUT_NSIZES;
    out->byte_record_arrays = 3;           // k0[], k1[], meta[] (sdp_records)
    out->byte_record_stride = (int32_t)sizeof(uint64_t);
    out->fixed_record_bytes = (int32_t)sizeof(uint64_t);
    out->heavy_max = SDP_HEAVY_MAX;
    out->heavy_max_rec = SDP_HEAVY_MAX_REC;
    out->heavy_min = SDP_HEAVY_MIN;
    out->part_sample = SDP_PART_SAMPLE;
    out->part_sample_bytes = SDP_PART_SAMPLE_BYTES;
    out->gsort_max = SDP_GSORT_MAX;
    out->part_chunk = SDP_PART_CHUNK;
    out->l2_block = SDP_L2_BLOCK;
    const int64_t sz[SDP_LAYOUT_NSIZES] = {
        sizeof(sdp_column), sizeof(sdp_bytes_column), sizeof(sdp_records), sizeof(sdp_heavy), sizeof(sdp_chunk),
        sizeof(sdp_qplan), sizeof(sdp_pass1_result), sizeof(sdp_select_task), sizeof(sdp_compact_task),
        sizeof(sdp_pass1_task), sizeof(sdp_pass2_task), sizeof(sdp_rows_task), sizeof(sdp_pass2_result),
        sizeof(sdp_minmax_result), sizeof(sdp_distinct_result), sizeof(sdp_topk_entry), sizeof(sdp_topk_result),
        sizeof(sdp_blocks)};
    for (int i = 0; i < SDP_LAYOUT_NSIZES; ++i) out->sizes[i] = sz[i];
    return SDP_OK;
}
