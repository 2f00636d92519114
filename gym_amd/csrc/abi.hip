// Library-level entry points and the thread-local error string.
#include "ga_common.h"

#include <string.h>

namespace ga {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = 0; }

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
        return GA_EHIP;
    }
    return GA_OK;
}

}  // namespace ga

extern "C" GA_API int ga_abi_version(void) { return 100; }

extern "C" GA_API const char* ga_last_error(void) { return ga::g_err; }
