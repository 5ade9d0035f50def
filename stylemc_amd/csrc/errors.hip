// Error state and device queries for the C ABI.
#include <algorithm>
#include <atomic>
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

__global__ __launch_bounds__(256) void zero_kernel(uint4* p, int64_t n16, uint32_t* tail, int64_t ntail) {
    const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x, step = (int64_t)gridDim.x * 256;
    for (int64_t i = i0; i < n16; i += step) p[i] = make_uint4(0u, 0u, 0u, 0u);
    for (int64_t i = i0; i < ntail; i += step) tail[i] = 0u;
}

int zero_async(void* p, size_t bytes, hipStream_t st, const char* what) {
    if (bytes == 0) return SMC_OK;
    const int64_t n16 = ((reinterpret_cast<uintptr_t>(p) & 15) == 0) ? (int64_t)(bytes / 16) : 0;
    uint32_t* tail = reinterpret_cast<uint32_t*>(static_cast<char*>(p) + n16 * 16);
    const int64_t ntail = (int64_t)(bytes - n16 * 16) / 4;  // (an unaligned buffer: word stores only)
    int64_t blocks = std::max<int64_t>(ceil_div(std::max<int64_t>(n16, ntail), 256), 1);
    blocks = std::min<int64_t>(blocks, (int64_t)device_cu_count() * 8);
    hipLaunchKernelGGL(zero_kernel, dim3((unsigned)blocks), dim3(256), 0, st, reinterpret_cast<uint4*>(p), n16, tail,
                       ntail);
    return check_launch(what);
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

// (plan, local) packed into one word: process-wide (the autograd engine runs backward calls on its own thread), set
// by the host thread that enqueues a step before it enqueues it
static std::atomic<int64_t> g_plan{0};

int64_t plan_rows(int64_t m) {
    const int64_t v = g_plan.load(std::memory_order_relaxed);
    const int64_t plan = v >> 32, local = v & 0xffffffff;
    if (plan <= 0 || local <= 0 || plan == local) return m;
    const int64_t r = (m * plan + local / 2) / local;
    return r < 1 ? 1 : r;
}

int plan_batch(int n) { return (int)plan_rows(n); }

}  // namespace smc

SMC_API int smc_set_plan_batch(int plan, int local) {
    SMC_CHECK(plan >= 0 && local >= 0 && (plan == 0) == (local == 0), "smc_set_plan_batch: bad arguments (%d, %d)",
              plan, local);
    smc::g_plan.store(((int64_t)plan << 32) | (int64_t)local, std::memory_order_relaxed);
    return SMC_OK;
}

SMC_API int smc_abi_version(void) { return SMC_ABI_VERSION; }

SMC_API const char* smc_last_error(void) { return smc::g_last_error.c_str(); }
