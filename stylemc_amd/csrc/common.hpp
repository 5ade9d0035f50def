// Shared helpers for the gfx950 kernels of stylemc_amd (error state, launch checks, activations).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "stylemc_hip.h"

#define SMC_API extern "C" __attribute__((visibility("default")))

namespace smc {

void set_error(const char* fmt, ...);
// smc_conv_gemm_f32 under the IR-SE50 executor's kernel names (TAG 1; conv_gemm.hip)
int conv_gemm_aux(const float* x, int n, int cin, int in_h, int in_w, float* y, int cout, int y_h, int y_w,
                  const smc_conv_phase* phases, int nphases, const float* s_in, const smc_conv_epilogue* epi,
                  float* workspace, int64_t workspace_bytes, void* stream);
// smc_conv_gemm_workspace_size for conv_gemm_aux (its split-K plan differs)
int64_t conv_gemm_aux_workspace_size(int n, int cin, int cout, int y_h, int y_w, const smc_conv_phase* phases,
                                     int nphases);
int check_launch(const char* what);
int device_cu_count();
// Zero `bytes` (a multiple of 4) at p with a kernel on `st` (in place of hipMemsetAsync; errors.hip).
int zero_async(void* p, size_t bytes, hipStream_t st, const char* what);
// Planning batch (smc_set_plan_batch): every launch decision that depends on the batch -- split-K factors, tile
// configurations, channel splits, all of which change a result's fp32 summation order -- is made for
// plan_batch(n) images (plan_rows(m) rows of a token-major GEMM) instead of the call's own n.  Default: n itself.
int plan_batch(int n);
int64_t plan_rows(int64_t m);

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
// bias_act.cu tests (yref / gain) > 0; the sign test below is the same predicate without the per-element
// IEEE division (it differs only where y / gain underflows to zero, |y| < 2^-149 |gain|).
__device__ __forceinline__ float act_grad_y(int act, float g, float y, float alpha, float gain, float clamp) {
    const bool pos = gain > 0.f ? y > 0.f : (gain < 0.f ? y < 0.f : false);
    float r = g;
    if (act == SMC_ACT_RELU) r = pos ? g : 0.f;
    if (act == SMC_ACT_LRELU) r = pos ? g : g * alpha;
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

// The compile-time lrelu + gain + clamp body of the synthesis epilogues (0 <= alpha <= 1, clamp >= 0): lrelu(z) =
// max(z, alpha z) and the clamp as one v_med3_f32 (= min(max(., -clamp), clamp) for every non-NaN value), bit-identical
// to epi_y for finite values.
__device__ __forceinline__ float lrelu_gain_clamp(float z, float alpha, float gain, float clamp) {
    return __builtin_amdgcn_fmed3f(fmaxf(z, z * alpha) * gain, -clamp, clamp);
}

// Epilogue fields beyond the modconv ones (IR-SE50 modes, per-channel scale, strided residual).
struct EpiExt {
    const float* scale_c;
    const float* alpha_c;
    const float* act_ref;
    const float* residual;
    int rs;
};

inline EpiExt epi_ext(const smc_conv_epilogue* e) {
    EpiExt x{};
    x.rs = 1;
    if (e) {
        x.scale_c = e->scale_c; x.alpha_c = e->alpha_c; x.act_ref = e->act_ref; x.residual = e->residual;
        x.rs = e->residual_stride > 0 ? e->residual_stride : 1;
    }
    return x;
}

// Modes PRELU / PRELU_GRAD / AFFINE and the residual (all modes) for output element idx = (n, o, yy, xx)
// of a [.][cout][y_h][y_w] tensor.  MODACT's own math stays in epi_y (scale_c folded into its d).
__device__ __forceinline__ float epi_ext_apply(int mode, float v, int n, int o, int64_t idx, int yy, int xx, int cout,
                                               int y_h, int y_w, const float* bias, float* u_save, const EpiExt& x) {
    if (mode == SMC_EPI_PRELU) {
        const float z = v * (x.scale_c ? x.scale_c[o] : 1.f) + (bias ? bias[o] : 0.f);
        if (u_save) u_save[idx] = z;
        v = z >= 0.f ? z : z * x.alpha_c[o];
    } else if (mode == SMC_EPI_PRELU_GRAD) {
        v = x.act_ref[idx] >= 0.f ? v : v * x.alpha_c[o];
    } else if (mode == SMC_EPI_AFFINE) {
        v = v * (x.scale_c ? x.scale_c[o] : 1.f) + (bias ? bias[o] : 0.f);
    }
    if (x.residual && yy % x.rs == 0 && xx % x.rs == 0) {
        const int rh = y_h / x.rs, rw = y_w / x.rs;
        v += x.residual[(((int64_t)n * cout + o) * rh + yy / x.rs) * rw + xx / x.rs];
    }
    return v;
}

}  // namespace smc

#define SMC_CHECK(cond, ...)                 \
    do {                                     \
        if (!(cond)) {                       \
            smc::set_error(__VA_ARGS__);     \
            return SMC_ERR_INVALID;          \
        }                                    \
    } while (0)
