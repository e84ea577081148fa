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
extern "C" const char *sdp_version(void) { return "sdp-mi355x 0.1.0 (gfx950)"; }
