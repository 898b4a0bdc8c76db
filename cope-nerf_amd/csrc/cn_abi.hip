// cn_abi.hip — version / error plumbing of libcopenerf.so (include/copenerf.h).
#include "cn_common.h"

#include <cstring>

namespace cn {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return CN_ERR_LAUNCH;
    }
    return CN_OK;
}

}  // namespace cn

extern "C" int cn_abi_version(void) { return CN_ABI_VERSION; }

extern "C" const char* cn_last_error(void) { return cn::g_last_error; }
