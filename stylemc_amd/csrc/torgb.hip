// ToRGB for gfx950: 1x1 modulated conv without demodulation + linear bias_act (clamped).
//
// Replaces the [upstream] ToRGBLayer.forward path (modulated_conv2d(demodulate=False) -> cuDNN 1x1
// grouped conv, conv2d_resample.py:29-54, then bias_act.py:153) called at utils.py:47.  With 3 output
// channels this is an HBM-bound channel reduction, not a GEMM: each thread streams one float4 of
// positions through all input channels, the [3 x cin] modulated weights of its sample sit in LDS.
#include "common.hpp"

namespace {

constexpr int kMaxOut = 4;
constexpr int kMaxIn = 1024;

template <bool VEC>
__global__ __launch_bounds__(256) void torgb_fwd_kernel(const float* x, const float* w, const float* s, const float* b,
                                                        float* y, int cin, int cout, int64_t hw, float clamp) {
    __shared__ float ws[kMaxOut * kMaxIn];
    const int nn = blockIdx.y;
    for (int i = threadIdx.x; i < cout * cin; i += 256) {
        const int c = i / cin, k = i - c * cin;
        ws[i] = w[i] * s[(int64_t)nn * cin + k];
    }
    __syncthreads();
    const float* xp = x + (int64_t)nn * cin * hw;
    float* yp = y + (int64_t)nn * cout * hw;
    constexpr int V = VEC ? 4 : 1;
    const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * V;
    if (p0 >= hw) return;
    float acc[kMaxOut][V];
#pragma unroll
    for (int c = 0; c < kMaxOut; ++c)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[c][v] = 0.f;
    // 8 channels per round: the 8 independent 16-B loads are all in flight before the first FMA.
    constexpr int U = 8;
    int k = 0;
    for (; k + U <= cin; k += U) {
        float xv[U][V];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (VEC) {
                const float4 t = *reinterpret_cast<const float4*>(xp + (int64_t)(k + u) * hw + p0);
                xv[u][0] = t.x; xv[u][V > 1 ? 1 : 0] = t.y; xv[u][V > 2 ? 2 : 0] = t.z; xv[u][V > 3 ? 3 : 0] = t.w;
            } else {
                xv[u][0] = xp[(int64_t)(k + u) * hw + p0];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < kMaxOut; ++c) {
                if (c >= cout) break;
                const float wv = ws[c * cin + k + u];
#pragma unroll
                for (int v = 0; v < V; ++v) acc[c][v] += wv * xv[u][v];
            }
    }
    for (; k < cin; ++k) {
        float xv[V];
        if (VEC) {
            const float4 t = *reinterpret_cast<const float4*>(xp + (int64_t)k * hw + p0);
            xv[0] = t.x; xv[V > 1 ? 1 : 0] = t.y; xv[V > 2 ? 2 : 0] = t.z; xv[V > 3 ? 3 : 0] = t.w;
        } else {
            xv[0] = xp[(int64_t)k * hw + p0];
        }
#pragma unroll
        for (int c = 0; c < kMaxOut; ++c) {
            if (c >= cout) break;
            const float wv = ws[c * cin + k];
#pragma unroll
            for (int v = 0; v < V; ++v) acc[c][v] += wv * xv[v];
        }
    }
#pragma unroll
    for (int c = 0; c < kMaxOut; ++c) {
        if (c >= cout) break;
        const float bv = b ? b[c] : 0.f;
        float r[V];
#pragma unroll
        for (int v = 0; v < V; ++v) r[v] = smc::clamp_fwd(acc[c][v] + bv, clamp);
        if (VEC) *reinterpret_cast<float4*>(yp + (int64_t)c * hw + p0) = make_float4(r[0], r[V > 1 ? 1 : 0],
                                                                                      r[V > 2 ? 2 : 0], r[V > 3 ? 3 : 0]);
        else yp[(int64_t)c * hw + p0] = r[0];
    }
}

template <bool VEC>
__global__ __launch_bounds__(256) void torgb_bwd_kernel(const float* g, const float* y, const float* w, const float* s,
                                                        float* dx, int cin, int cout, int64_t hw, float clamp,
                                                        int scale, int accumulate) {
    __shared__ float ws[kMaxOut * kMaxIn];
    const int nn = blockIdx.y;
    for (int i = threadIdx.x; i < cout * cin; i += 256) {
        const int c = i / cin, k = i - c * cin;
        ws[i] = w[i] * (scale ? s[(int64_t)nn * cin + k] : 1.f);
    }
    __syncthreads();
    constexpr int V = VEC ? 4 : 1;
    const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * V;
    if (p0 >= hw) return;
    float gm[kMaxOut][V];
#pragma unroll
    for (int c = 0; c < kMaxOut; ++c) {
#pragma unroll
        for (int v = 0; v < V; ++v) gm[c][v] = 0.f;
        if (c >= cout) continue;
        const int64_t off = ((int64_t)nn * cout + c) * hw + p0;
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const float yv = y[off + v];
            const bool pass = clamp < 0.f || (yv > -clamp && yv < clamp);  // bias_act.cu:136-141 (grad=1)
            gm[c][v] = pass ? g[off + v] : 0.f;
        }
    }
    float* dp = dx + (int64_t)nn * cin * hw + p0;
    for (int k = 0; k < cin; ++k) {
        float r[V];
#pragma unroll
        for (int v = 0; v < V; ++v) r[v] = 0.f;
#pragma unroll
        for (int c = 0; c < kMaxOut; ++c) {
            if (c >= cout) break;
            const float wv = ws[c * cin + k];
#pragma unroll
            for (int v = 0; v < V; ++v) r[v] += wv * gm[c][v];
        }
        float* dst = dp + (int64_t)k * hw;
        if (VEC) {
            float4 o = make_float4(r[0], r[V > 1 ? 1 : 0], r[V > 2 ? 2 : 0], r[V > 3 ? 3 : 0]);
            if (accumulate) {
                const float4 prev = *reinterpret_cast<const float4*>(dst);
                o.x += prev.x; o.y += prev.y; o.z += prev.z; o.w += prev.w;
            }
            *reinterpret_cast<float4*>(dst) = o;
        } else {
            dst[0] = accumulate ? dst[0] + r[0] : r[0];
        }
    }
}

// Block-tail backward: a synthesis block's output y (conv1's output, read by this block's ToRGB and by the next
// block's conv0) gets g_y = g_next + ToRGB^T(g_rgb), and conv1's epilogue backward turns it into du = act'(g_y; y) *
// d[n,k] -- three passes (ToRGB data gradient, autograd's sum, act_bwd) in one.  The ToRGB gradient and the sum are
// the same fp32 operations as the separate kernels (a + b is commutative), and the epilogue backward is act_bwd's
// grad_from_y form, so du is bit-identical to the unfused path.
template <bool VEC>
__global__ __launch_bounds__(256) void torgb_act_bwd_kernel(const float* g_rgb, const float* y_rgb, const float* w,
                                                            const float* s, float clamp_rgb, const float* g_next,
                                                            const float* y, float* du, int cin, int cout, int64_t hw,
                                                            const float* d, int act, float alpha, float gain,
                                                            float clamp, int kch) {
    __shared__ float ws[kMaxOut * kMaxIn];
    const int nn = blockIdx.y;
    for (int i = threadIdx.x; i < cout * cin; i += 256) {
        const int c = i / cin, k = i - c * cin;
        ws[i] = w[i] * s[(int64_t)nn * cin + k];
    }
    __syncthreads();
    constexpr int V = VEC ? 4 : 1;
    const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * V;
    if (p0 >= hw) return;
    float gm[kMaxOut][V];
#pragma unroll
    for (int c = 0; c < kMaxOut; ++c) {
#pragma unroll
        for (int v = 0; v < V; ++v) gm[c][v] = 0.f;
        if (c >= cout) continue;
        const int64_t off = ((int64_t)nn * cout + c) * hw + p0;
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const float yv = y_rgb[off + v];
            const bool pass = clamp_rgb < 0.f || (yv > -clamp_rgb && yv < clamp_rgb);
            gm[c][v] = pass ? g_rgb[off + v] : 0.f;
        }
    }
    const int64_t base = (int64_t)nn * cin * hw + p0;
    // this workgroup's channels: grid.z splits them when the position grid alone is small (kch = cin otherwise)
    const int kbeg = blockIdx.z * kch, kend = min(cin, kbeg + kch);
    // Channels in chunks of KC: every load of a chunk is issued before its stores (one at a time, each channel's
    // loads would wait for the previous channel's store: vmcnt counts both).
    constexpr int KC = 8;
    for (int k0 = kbeg; k0 < kend; k0 += KC) {
        float gn[KC][V], yk[KC][V], dkv[KC];
#pragma unroll
        for (int kk = 0; kk < KC; ++kk) {
            const int k = min(k0 + kk, kend - 1);
            const int64_t off = base + (int64_t)k * hw;
            dkv[kk] = d ? d[(int64_t)nn * cin + k] : 1.f;
            if (VEC) {
                const float4 a = g_next ? *reinterpret_cast<const float4*>(g_next + off) : make_float4(0.f, 0.f, 0.f, 0.f);
                const float4 b = *reinterpret_cast<const float4*>(y + off);
                gn[kk][0] = a.x; gn[kk][V > 1 ? 1 : 0] = a.y; gn[kk][V > 2 ? 2 : 0] = a.z; gn[kk][V > 3 ? 3 : 0] = a.w;
                yk[kk][0] = b.x; yk[kk][V > 1 ? 1 : 0] = b.y; yk[kk][V > 2 ? 2 : 0] = b.z; yk[kk][V > 3 ? 3 : 0] = b.w;
            } else {
                gn[kk][0] = g_next ? g_next[off] : 0.f;
                yk[kk][0] = y[off];
            }
        }
#pragma unroll
        for (int kk = 0; kk < KC; ++kk) {
            const int k = k0 + kk;
            if (k >= kend) break;
            const int64_t off = base + (int64_t)k * hw;
            const float dk = dkv[kk];
            float r[V];
#pragma unroll
            for (int v = 0; v < V; ++v) {
                float t = 0.f;
#pragma unroll
                for (int c = 0; c < kMaxOut; ++c) {
                    if (c >= cout) break;
                    t += ws[c * cin + k] * gm[c][v];
                }
                const float gy = g_next ? gn[kk][v] + t : t;
                r[v] = smc::act_grad_y(act, gy, yk[kk][v], alpha, gain, clamp) * dk;
            }
            if (VEC) *reinterpret_cast<float4*>(du + off) = make_float4(r[0], r[V > 1 ? 1 : 0], r[V > 2 ? 2 : 0],
                                                                        r[V > 3 ? 3 : 0]);
            else du[off] = r[0];
        }
    }
}

// Low-resolution forms (hw <= kSmallHw: the 4..64-px blocks, 512 input channels).  The per-position kernels
// above give each thread the whole channel reduction, which at these sizes is 1-4 workgroups per image and a
// chain of 64 dependent load rounds (~90 us for 16 positions).  Here the channels are split over the
// workgroup and over more workgroups: forward = 16 positions x 16 channel groups per workgroup + an LDS
// reduction; backward (no reduction over input channels) = 64 positions x 4 channel lanes, KCH channels per
// workgroup in grid.y.
constexpr int64_t kSmallHw = 4096;
constexpr int kFwdP = 16, kFwdG = 16;
constexpr int kBwdP = 64, kBwdKCH = 32;

__global__ __launch_bounds__(256) void torgb_fwd_small_kernel(const float* x, const float* w, const float* s,
                                                              const float* b, float* y, int cin, int cout, int64_t hw,
                                                              float clamp) {
    __shared__ float red[kFwdG][kMaxOut][kFwdP];
    const int nn = blockIdx.y;
    const int pl = threadIdx.x % kFwdP, grp = threadIdx.x / kFwdP;
    const int64_t p = (int64_t)blockIdx.x * kFwdP + pl;
    const bool pv = p < hw;
    const float* xp = x + (int64_t)nn * cin * hw + (pv ? p : 0);
    const float* sp = s + (int64_t)nn * cin;
    float acc[kMaxOut] = {0.f, 0.f, 0.f, 0.f};
    constexpr int U = 8;
    int k = grp;
    for (; k + (U - 1) * kFwdG < cin; k += U * kFwdG) {
        float xv[U], sv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            xv[u] = xp[(int64_t)(k + u * kFwdG) * hw];
            sv[u] = sp[k + u * kFwdG];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < kMaxOut; ++c) {
                if (c >= cout) break;
                acc[c] += (w[c * cin + k + u * kFwdG] * sv[u]) * xv[u];
            }
    }
    for (; k < cin; k += kFwdG) {
        const float xv = xp[(int64_t)k * hw];
#pragma unroll
        for (int c = 0; c < kMaxOut; ++c) {
            if (c >= cout) break;
            acc[c] += (w[c * cin + k] * sp[k]) * xv;
        }
    }
#pragma unroll
    for (int c = 0; c < kMaxOut; ++c) red[grp][c][pl] = acc[c];
    __syncthreads();
    if (threadIdx.x < kMaxOut * kFwdP) {
        const int c = threadIdx.x / kFwdP, q = threadIdx.x % kFwdP;
        const int64_t pp = (int64_t)blockIdx.x * kFwdP + q;
        if (c < cout && pp < hw) {
            float t = 0.f;
#pragma unroll
            for (int g2 = 0; g2 < kFwdG; ++g2) t += red[g2][c][q];
            y[((int64_t)nn * cout + c) * hw + pp] = smc::clamp_fwd(t + (b ? b[c] : 0.f), clamp);
        }
    }
}

__global__ __launch_bounds__(256) void torgb_bwd_small_kernel(const float* g, const float* y, const float* w,
                                                              const float* s, float* dx, int cin, int cout, int64_t hw,
                                                              float clamp, int scale, int accumulate) {
    const int nn = blockIdx.z;
    const int pl = threadIdx.x % kBwdP, kl = threadIdx.x / kBwdP;
    const int64_t p = (int64_t)blockIdx.x * kBwdP + pl;
    if (p >= hw) return;
    float gm[kMaxOut];
#pragma unroll
    for (int c = 0; c < kMaxOut; ++c) {
        gm[c] = 0.f;
        if (c >= cout) continue;
        const int64_t off = ((int64_t)nn * cout + c) * hw + p;
        const float yv = y[off];
        const bool pass = clamp < 0.f || (yv > -clamp && yv < clamp);  // bias_act.cu:136-141 (grad=1)
        gm[c] = pass ? g[off] : 0.f;
    }
    const int k0 = blockIdx.y * kBwdKCH;
    for (int k = k0 + kl; k < k0 + kBwdKCH && k < cin; k += 256 / kBwdP) {
        const float sk = scale ? s[(int64_t)nn * cin + k] : 1.f;
        float r = 0.f;
#pragma unroll
        for (int c = 0; c < kMaxOut; ++c) {
            if (c >= cout) break;
            r += (w[c * cin + k] * sk) * gm[c];
        }
        float* dst = dx + ((int64_t)nn * cin + k) * hw + p;
        *dst = accumulate ? *dst + r : r;
    }
}

}  // namespace

SMC_API int smc_torgb_fwd_f32(const float* x, const float* w, const float* s, const float* b, float* y, int n, int cin,
                              int cout, int h, int w_, float clamp, void* stream) {
    SMC_CHECK(x && w && s && y && n >= 1 && cin >= 1 && h >= 1 && w_ >= 1, "smc_torgb_fwd_f32: bad args");
    SMC_CHECK(n < 65536, "smc_torgb_fwd_f32: batch too large");
    if (cout < 1 || cout > kMaxOut || cin > kMaxIn) {
        smc::set_error("smc_torgb_fwd_f32: cout=%d (max %d) cin=%d (max %d)", cout, kMaxOut, cin, kMaxIn);
        return SMC_ERR_UNSUPPORTED;
    }
    const int64_t hw = (int64_t)h * w_;
    if (hw <= kSmallHw) {
        hipLaunchKernelGGL(torgb_fwd_small_kernel, dim3((unsigned)smc::ceil_div(hw, kFwdP), (unsigned)n), dim3(256), 0,
                           smc::as_stream(stream), x, w, s, b, y, cin, cout, hw, clamp);
        return smc::check_launch("smc_torgb_fwd_f32");
    }
    const bool vec = hw % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0;
    const int64_t per = vec ? hw / 4 : hw;
    dim3 grid((unsigned)smc::ceil_div(per, 256), (unsigned)n);
    if (vec) hipLaunchKernelGGL(torgb_fwd_kernel<true>, grid, dim3(256), 0, smc::as_stream(stream), x, w, s, b, y, cin,
                                cout, hw, clamp);
    else hipLaunchKernelGGL(torgb_fwd_kernel<false>, grid, dim3(256), 0, smc::as_stream(stream), x, w, s, b, y, cin,
                            cout, hw, clamp);
    return smc::check_launch("smc_torgb_fwd_f32");
}

SMC_API int smc_torgb_bwd_f32(const float* g, const float* y, const float* w, const float* s, float* dx, int n, int cin,
                              int cout, int h, int w_, float clamp, int scale, int accumulate, void* stream) {
    SMC_CHECK(g && y && w && dx && n >= 1 && cin >= 1 && h >= 1 && w_ >= 1, "smc_torgb_bwd_f32: bad args");
    SMC_CHECK(!scale || s, "smc_torgb_bwd_f32: scale needs s");
    SMC_CHECK(n < 65536, "smc_torgb_bwd_f32: batch too large");
    if (cout < 1 || cout > kMaxOut || cin > kMaxIn) {
        smc::set_error("smc_torgb_bwd_f32: cout=%d (max %d) cin=%d (max %d)", cout, kMaxOut, cin, kMaxIn);
        return SMC_ERR_UNSUPPORTED;
    }
    const int64_t hw = (int64_t)h * w_;
    if (hw <= kSmallHw) {
        dim3 grid((unsigned)smc::ceil_div(hw, kBwdP), (unsigned)smc::ceil_div(cin, kBwdKCH), (unsigned)n);
        hipLaunchKernelGGL(torgb_bwd_small_kernel, grid, dim3(256), 0, smc::as_stream(stream), g, y, w, s, dx, cin,
                           cout, hw, clamp, scale, accumulate);
        return smc::check_launch("smc_torgb_bwd_f32");
    }
    const bool vec = hw % 4 == 0 && (reinterpret_cast<uintptr_t>(dx) & 15) == 0;
    const int64_t per = vec ? hw / 4 : hw;
    dim3 grid((unsigned)smc::ceil_div(per, 256), (unsigned)n);
    if (vec) hipLaunchKernelGGL(torgb_bwd_kernel<true>, grid, dim3(256), 0, smc::as_stream(stream), g, y, w, s, dx, cin,
                                cout, hw, clamp, scale, accumulate);
    else hipLaunchKernelGGL(torgb_bwd_kernel<false>, grid, dim3(256), 0, smc::as_stream(stream), g, y, w, s, dx, cin,
                            cout, hw, clamp, scale, accumulate);
    return smc::check_launch("smc_torgb_bwd_f32");
}

SMC_API int smc_torgb_act_bwd_f32(const float* g_rgb, const float* y_rgb, const float* w, const float* s,
                                  float clamp_rgb, const float* g_next, const float* y, float* du, int n, int cin,
                                  int cout, int h, int w_, const smc_conv_epilogue* epi, void* stream) {
    SMC_CHECK(g_rgb && y_rgb && w && s && y && du && n >= 1 && cin >= 1 && h >= 1 && w_ >= 1,
              "smc_torgb_act_bwd_f32: bad args");
    SMC_CHECK(epi && epi->mode == SMC_EPI_MODACT && epi->grad_from_y,
              "smc_torgb_act_bwd_f32: needs conv1's MODACT epilogue with grad_from_y");
    SMC_CHECK(n < 65536, "smc_torgb_act_bwd_f32: batch too large");
    if (cout < 1 || cout > kMaxOut || cin > kMaxIn) {
        smc::set_error("smc_torgb_act_bwd_f32: cout=%d (max %d) cin=%d (max %d)", cout, kMaxOut, cin, kMaxIn);
        return SMC_ERR_UNSUPPORTED;
    }
    const int64_t hw = (int64_t)h * w_;
    const uintptr_t al = (uintptr_t)g_next | (uintptr_t)y | (uintptr_t)du;
    const bool vec = hw % 4 == 0 && (al & 15) == 0;
    const int64_t per = vec ? hw / 4 : hw;
    dim3 grid((unsigned)smc::ceil_div(per, 256), (unsigned)n);
    // Each thread walks its positions' channels one 8-channel chunk after another (a chain of dependent load rounds):
    // a small position grid (the 128..512-px blocks) also splits the channels over grid.z, in whole chunks, until the
    // launch holds ~4 workgroups per CU (r = 128: 64 workgroups walking 256 channels took 264 us).
    int nz = 1;
    const int64_t plan_wg = (int64_t)grid.x * smc::plan_batch(n);   // grid.y = n: the split from the planning batch
    while (plan_wg * nz < 4 * (int64_t)smc::device_cu_count() && cin % (16 * nz) == 0) nz *= 2;
    grid.z = (unsigned)nz;
    const int kch = cin / nz;
    if (vec)
        hipLaunchKernelGGL(torgb_act_bwd_kernel<true>, grid, dim3(256), 0, smc::as_stream(stream), g_rgb, y_rgb, w, s,
                           clamp_rgb, g_next, y, du, cin, cout, hw, epi->d, epi->act, epi->alpha, epi->gain, epi->clamp,
                           kch);
    else
        hipLaunchKernelGGL(torgb_act_bwd_kernel<false>, grid, dim3(256), 0, smc::as_stream(stream), g_rgb, y_rgb, w, s,
                           clamp_rgb, g_next, y, du, cin, cout, hw, epi->d, epi->act, epi->alpha, epi->gain, epi->clamp,
                           kch);
    return smc::check_launch("smc_torgb_act_bwd_f32");
}
