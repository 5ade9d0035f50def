// bias_act for gfx950: fused bias + activation + gain + clamp, and its 1st/2nd-order gradients.
//
// Replaces the reference's `_plugin.bias_act` (torch_utils/ops/bias_act.cpp:32-90, kernel
// bias_act.cu:23-147).  HBM-bound elementwise: 16-B (float4) loads/stores whenever the bias index is
// constant across each 4-element vector (step_b % 4 == 0), grid-stride loop sized for the 256 CUs.
#include <cmath>

#include "common.hpp"

namespace {

struct BAParams {
    const float* x;
    const float* b;
    const float* xref;
    const float* yref;
    const float* dy;
    float* y;
    int64_t numel;
    int64_t size_b;
    int64_t step_b;
    float alpha, gain, clamp;
};

// One element.  For G == 0, `x` is the forward input; for G >= 1 it is the incoming gradient and
// `xr`/`yr` are the saved forward input (pre-bias) / output.
template <int A, int G>
__device__ __forceinline__ float ba_one(float x, float bias, float xr, float yr, float dyv, const BAParams& p) {
    const float alpha = p.alpha, gain = p.gain, clamp = p.clamp;
    const float kRange = 80.f, kHalfRange = 40.f;
    const float kSeluScale = 1.0507009873554804934193349852946f;
    const float kSeluAlpha = 1.6732632423543772848170429916717f;
    float yy = (gain != 0.f) ? yr / gain : 0.f;  // forward output before the gain
    float r = 0.f;
    if (G == 0) x += bias; else xr += bias;

    if (A == SMC_ACT_LINEAR) {
        r = x;
    } else if (A == SMC_ACT_RELU) {
        if (G == 0) r = x > 0.f ? x : 0.f;
        if (G == 1) r = yy > 0.f ? x : 0.f;
    } else if (A == SMC_ACT_LRELU) {
        if (G == 0) r = x > 0.f ? x : x * alpha;
        if (G == 1) r = yy > 0.f ? x : x * alpha;
    } else if (A == SMC_ACT_TANH) {
        if (G == 0) r = x < -kRange ? -1.f : x > kRange ? 1.f : tanhf(x);
        if (G == 1) r = x * (1.f - yy * yy);
        if (G == 2) r = x * (1.f - yy * yy) * (-2.f * yy);
    } else if (A == SMC_ACT_SIGMOID) {
        if (G == 0) r = x < -kRange ? 0.f : 1.f / (1.f + expf(-x));
        if (G == 1) r = x * yy * (1.f - yy);
        if (G == 2) r = x * yy * (1.f - yy) * (1.f - 2.f * yy);
    } else if (A == SMC_ACT_ELU) {
        if (G == 0) r = x >= 0.f ? x : expf(x) - 1.f;
        if (G == 1) r = yy >= 0.f ? x : x * (yy + 1.f);
        if (G == 2) r = yy >= 0.f ? 0.f : x * (yy + 1.f);
    } else if (A == SMC_ACT_SELU) {
        if (G == 0) r = x >= 0.f ? kSeluScale * x : (kSeluScale * kSeluAlpha) * (expf(x) - 1.f);
        if (G == 1) r = yy >= 0.f ? x * kSeluScale : x * (yy + kSeluScale * kSeluAlpha);
        if (G == 2) r = yy >= 0.f ? 0.f : x * (yy + kSeluScale * kSeluAlpha);
    } else if (A == SMC_ACT_SOFTPLUS) {
        if (G == 0) r = x > kRange ? x : log1pf(expf(x));
        if (G == 1) r = x * (1.f - expf(-yy));
        if (G == 2) { float c = expf(-yy); r = x * c * (1.f - c); }
    } else if (A == SMC_ACT_SWISH) {
        if (G == 0) {
            r = x < -kRange ? 0.f : x / (1.f + expf(-x));
        } else {
            float e = expf(xr), d = e + 1.f;
            if (G == 1) r = xr > kHalfRange ? x : x * e * (xr + d) / (d * d);
            else        r = xr > kHalfRange ? 0.f : x * e * (xr * (2.f - d) + 2.f * d) / (d * d * d);
            yr = xr < -kRange ? 0.f : xr / (1.f + expf(-xr)) * gain;  // swish references x, not y
        }
    }
    r *= gain * dyv;
    if (clamp >= 0.f) {
        if (G == 0) r = (r > -clamp && r < clamp) ? r : (r >= 0.f ? clamp : -clamp);
        else        r = (yr > -clamp && yr < clamp) ? r : 0.f;
    }
    return r;
}

template <int A, int G>
__global__ __launch_bounds__(256) void bias_act_vec4(BAParams p) {
    const int64_t nvec = p.numel >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
        const int64_t i = v << 2;
        float4 xv = reinterpret_cast<const float4*>(p.x)[v];
        float bias = p.b ? p.b[(i / p.step_b) % p.size_b] : 0.f;
        float4 xr = p.xref ? reinterpret_cast<const float4*>(p.xref)[v] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 yr = p.yref ? reinterpret_cast<const float4*>(p.yref)[v] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 dv = p.dy ? reinterpret_cast<const float4*>(p.dy)[v] : make_float4(1.f, 1.f, 1.f, 1.f);
        float4 o;
        o.x = ba_one<A, G>(xv.x, bias, xr.x, yr.x, dv.x, p);
        o.y = ba_one<A, G>(xv.y, bias, xr.y, yr.y, dv.y, p);
        o.z = ba_one<A, G>(xv.z, bias, xr.z, yr.z, dv.z, p);
        o.w = ba_one<A, G>(xv.w, bias, xr.w, yr.w, dv.w, p);
        reinterpret_cast<float4*>(p.y)[v] = o;
    }
}

template <int A, int G>
__global__ __launch_bounds__(256) void bias_act_scalar(BAParams p) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.numel; i += stride) {
        float bias = p.b ? p.b[(i / p.step_b) % p.size_b] : 0.f;
        float xr = p.xref ? p.xref[i] : 0.f;
        float yr = p.yref ? p.yref[i] : 0.f;
        float dv = p.dy ? p.dy[i] : 1.f;
        p.y[i] = ba_one<A, G>(p.x[i], bias, xr, yr, dv, p);
    }
}

template <int A, int G>
int launch_ba(const BAParams& p, bool vec, hipStream_t st) {
    const int threads = 256;
    const int64_t work = vec ? (p.numel >> 2) : p.numel;
    int64_t blocks = smc::ceil_div(work, threads);
    const int64_t cap = (int64_t)smc::device_cu_count() * 16;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    if (vec) hipLaunchKernelGGL((bias_act_vec4<A, G>), dim3((unsigned)blocks), dim3(threads), 0, st, p);
    else     hipLaunchKernelGGL((bias_act_scalar<A, G>), dim3((unsigned)blocks), dim3(threads), 0, st, p);
    return smc::check_launch("smc_bias_act_f32");
}

template <int A>
int dispatch_grad(int grad, const BAParams& p, bool vec, hipStream_t st) {
    if (grad == 0) return launch_ba<A, 0>(p, vec, st);
    if (grad == 1) return launch_ba<A, 1>(p, vec, st);
    return launch_ba<A, 2>(p, vec, st);
}

inline bool aligned16(const void* ptr) { return ptr == nullptr || (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

}  // namespace

SMC_API int smc_bias_act_f32(const float* x, const float* b, const float* xref, const float* yref, const float* dy,
                             float* y, int64_t numel, int64_t size_b, int64_t step_b, int grad, int act, float alpha,
                             float gain, float clamp, void* stream) {
    SMC_CHECK(numel >= 0, "smc_bias_act_f32: numel < 0");
    SMC_CHECK(grad >= 0 && grad <= 2, "smc_bias_act_f32: grad must be 0, 1 or 2 (got %d)", grad);
    SMC_CHECK(act >= SMC_ACT_LINEAR && act <= SMC_ACT_SWISH, "smc_bias_act_f32: unknown act %d", act);
    SMC_CHECK(b == nullptr || (size_b > 0 && step_b > 0), "smc_bias_act_f32: bad bias geometry");
    SMC_CHECK(numel == 0 || (x != nullptr && y != nullptr), "smc_bias_act_f32: null x/y");
    SMC_CHECK(grad == 0 || xref != nullptr || yref != nullptr || act == SMC_ACT_LINEAR,
              "smc_bias_act_f32: grad %d needs xref/yref", grad);
    if (numel == 0) return SMC_OK;
    BAParams p{x, b, xref, yref, dy, y, numel, b ? size_b : 1, b ? step_b : 1, alpha, gain, clamp};
    const bool vec = (numel % 4 == 0) && (b == nullptr || step_b % 4 == 0) && aligned16(x) && aligned16(y) &&
                     aligned16(xref) && aligned16(yref) && aligned16(dy);
    hipStream_t st = smc::as_stream(stream);
    switch (act) {
        case SMC_ACT_LINEAR: return dispatch_grad<SMC_ACT_LINEAR>(grad, p, vec, st);
        case SMC_ACT_RELU: return dispatch_grad<SMC_ACT_RELU>(grad, p, vec, st);
        case SMC_ACT_LRELU: return dispatch_grad<SMC_ACT_LRELU>(grad, p, vec, st);
        case SMC_ACT_TANH: return dispatch_grad<SMC_ACT_TANH>(grad, p, vec, st);
        case SMC_ACT_SIGMOID: return dispatch_grad<SMC_ACT_SIGMOID>(grad, p, vec, st);
        case SMC_ACT_ELU: return dispatch_grad<SMC_ACT_ELU>(grad, p, vec, st);
        case SMC_ACT_SELU: return dispatch_grad<SMC_ACT_SELU>(grad, p, vec, st);
        case SMC_ACT_SOFTPLUS: return dispatch_grad<SMC_ACT_SOFTPLUS>(grad, p, vec, st);
        default: return dispatch_grad<SMC_ACT_SWISH>(grad, p, vec, st);
    }
}
