// Error state and device queries for the C ABI.
#include <cstdarg>
#include <cstdio>
#include <string>

#include "common.hpp"

namespace smc {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return SMC_ERR_LAUNCH;
    }
    return SMC_OK;
}

int device_cu_count() {
    static thread_local int cached_dev = -1;
    static thread_local int cached_cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (dev != cached_dev) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            cached_cus = cus;
        cached_dev = dev;
    }
    return cached_cus;
}

}  // namespace smc

SMC_API int smc_abi_version(void) { return SMC_ABI_VERSION; }

SMC_API const char* smc_last_error(void) { return smc::g_last_error.c_str(); }
