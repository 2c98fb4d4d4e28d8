// capi_common.cpp -- version, thread-local error text, launch checking.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "acn_internal.h"

namespace {
thread_local char g_err[512] = {0};
}

int acn_set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int acn_check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return acn_set_error((int)e, "%s: launch failed: %s", what, hipGetErrorString(e));
    return ACN_OK;
}

extern "C" int acn_version(void) { return ACN_ABI_VERSION; }

extern "C" int acn_last_error(char* buf, size_t n) {
    size_t len = strlen(g_err);
    if (buf && n) {
        size_t c = len < n - 1 ? len : n - 1;
        memcpy(buf, g_err, c);
        buf[c] = 0;
    }
    return (int)len;
}
