// Library status / error plumbing for the hgsr C ABI.
#include <stdarg.h>
#include <string.h>

#include "common.h"

namespace hgsr {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
        return HGSR_ELAUNCH;
    }
    return HGSR_OK;
}

}  // namespace hgsr

extern "C" int hgsr_version(void) { return 1; }
extern "C" const char* hgsr_last_error(void) { return hgsr::g_err; }
