// Shared helpers for the gfx950 kernels of stylemc_amd (error state, launch checks, activations).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "stylemc_hip.h"

#define SMC_API extern "C" __attribute__((visibility("default")))

namespace smc {

void set_error(const char* fmt, ...);
int check_launch(const char* what);
int device_cu_count();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------------------------
// Activations of the modconv epilogue path (linear / relu / lrelu), forward and y-referenced grad.
// Semantics restate bias_act.cu:51-142 for these three (mask on the *clamped* output).

__device__ __forceinline__ float act_fwd(int act, float x, float alpha) {
    if (act == SMC_ACT_RELU) return x > 0.f ? x : 0.f;
    if (act == SMC_ACT_LRELU) return x > 0.f ? x : x * alpha;
    return x;
}

__device__ __forceinline__ float clamp_fwd(float y, float clamp) {
    if (clamp >= 0.f) return (y > -clamp && y < clamp) ? y : (y >= 0.f ? clamp : -clamp);
    return y;
}

// dz given the incoming gradient g and the forward output y.
__device__ __forceinline__ float act_grad_y(int act, float g, float y, float alpha, float gain, float clamp) {
    float yy = gain != 0.f ? y / gain : 0.f;
    float r = g;
    if (act == SMC_ACT_RELU) r = yy > 0.f ? g : 0.f;
    if (act == SMC_ACT_LRELU) r = yy > 0.f ? g : g * alpha;
    r *= gain;
    if (clamp >= 0.f) r = (y > -clamp && y < clamp) ? r : 0.f;
    return r;
}

// Modconv epilogue: y = clamp(act(u * d + noise + bias) * gain).  Every kernel that produces or
// re-derives y from u goes through this one function so forward and backward see the same rounding.
__device__ __forceinline__ float epi_y(float u, float d, float nz, float bias, int act, float alpha, float gain,
                                       float clamp) {
    float z = __fmaf_rn(u, d, nz) + bias;
    return clamp_fwd(act_fwd(act, z, alpha) * gain, clamp);
}

}  // namespace smc

#define SMC_CHECK(cond, ...)                 \
    do {                                     \
        if (!(cond)) {                       \
            smc::set_error(__VA_ARGS__);     \
            return SMC_ERR_INVALID;          \
        }                                    \
    } while (0)
