// CLIP input preprocessing for gfx950, forward and image gradient, in two forms:
//   StyleMC (find_direction.py:49-52, MODE 0):
//     y = (bicubic(clamp(img * 127.5 + 128, 0, 255), (out_h, out_w)) / 255 - mean[c]) / std[c]
//   StyleGAN-NADA (clip_loss_nada.py:72-75,109-111, MODE 1): Normalize(-1, 2) -> Resize(BICUBIC) -> CenterCrop
//   -> CLIP Normalize, no clamp:
//     y = (bicubic((img + 1) / 2, (out_h, out_w)) - mean[c]) / std[c]
// with the torchvision-0.8 tensor Resize (F.interpolate bicubic, align_corners=False, A = -0.75, border
// replicate) restated from aten's upsample_bicubic2d (source index s = scale * (dst + 0.5) - 0.5, taps
// floor(s) - 1 .. floor(s) + 2, rows interpolated first along x then along y).
// Forward: one thread per output; only the 4 x 4 taps of each output are read (no antialias: at 1024 -> 224
// a fifth of the image), instead of three full-resolution elementwise passes + the resize.
// Backward: gather form -- one thread per input pixel sums the (at most a few) outputs whose taps cover it
// and writes the whole gradient (zeros elsewhere); aten's resize backward scatters with atomics.
#include "common.hpp"

namespace {

constexpr float kA = -0.75f;

__device__ __forceinline__ float cc1(float x) { return ((kA + 2.f) * x - (kA + 3.f)) * x * x + 1.f; }
__device__ __forceinline__ float cc2(float x) { return ((kA * x - 5.f * kA) * x + 8.f * kA) * x - 4.f * kA; }

__device__ __forceinline__ void cubic_coeffs(float t, float (&c)[4]) {
    c[0] = cc2(t + 1.f);
    c[1] = cc1(t);
    c[2] = cc1(1.f - t);
    c[3] = cc2(2.f - t);
}

template <int MODE>
__device__ __forceinline__ float pre(float v) {
    if (MODE == 0) {  // img * 127.5 + 128 (two roundings, as torch), clamped
        const float x = __fadd_rn(__fmul_rn(v, 127.5f), 128.f);
        return fminf(fmaxf(x, 0.f), 255.f);
    }
    return __fadd_rn(v, 1.f) * 0.5f;  // torchvision Normalize(-1, 2): (v - (-1)) / 2
}

template <int MODE>
__device__ __forceinline__ float post(float s, float mean, float std_) {
    return MODE == 0 ? __fsub_rn(s / 255.f, mean) / std_ : __fsub_rn(s, mean) / std_;
}

struct Unproc {
    int in_h, in_w, out_h, out_w, channels;
    float sy, sx;  // in / out
    const float* mean;
    const float* std_;
};

template <int MODE>
__global__ __launch_bounds__(256) void unprocess_fwd_kernel(const float* img, float* y, int64_t planes, Unproc q) {
    const int64_t per = (int64_t)q.out_h * q.out_w;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= planes * per) return;
    const int64_t pl = idx / per;
    const int rem = (int)(idx - pl * per);
    const int oy = rem / q.out_w, ox = rem - oy * q.out_w;
    const float ry = q.sy * (oy + 0.5f) - 0.5f, rx = q.sx * (ox + 0.5f) - 0.5f;
    const int iy = (int)floorf(ry), ix = (int)floorf(rx);
    float cy[4], cx[4];
    cubic_coeffs(ry - iy, cy);
    cubic_coeffs(rx - ix, cx);
    const float* p = img + pl * (int64_t)q.in_h * q.in_w;
    float rows[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int yy = min(max(iy - 1 + a, 0), q.in_h - 1);
        const float* r = p + (int64_t)yy * q.in_w;
        float v[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) v[b] = pre<MODE>(r[min(max(ix - 1 + b, 0), q.in_w - 1)]);
        rows[a] = v[0] * cx[0] + v[1] * cx[1] + v[2] * cx[2] + v[3] * cx[3];
    }
    const float s = rows[0] * cy[0] + rows[1] * cy[1] + rows[2] * cy[2] + rows[3] * cy[3];
    const int c = (int)(pl % q.channels);
    y[idx] = post<MODE>(s, q.mean[c], q.std_[c]);
}

// the (output index, tap weight) pairs of one axis that read input index i (border taps may repeat)
__device__ __forceinline__ int taps_of(int i, int in, int out, float scale, int (&o)[8], float (&w)[8]) {
    int n = 0;
    const int c0 = (int)floorf((i + 0.5f) / scale - 0.5f);
    for (int d = c0 - 2; d <= c0 + 2; ++d) {
        if (d < 0 || d >= out) continue;
        const float r = scale * (d + 0.5f) - 0.5f;
        const int f = (int)floorf(r);
        float c[4];
        cubic_coeffs(r - f, c);
        float acc = 0.f;
        bool hit = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (min(max(f - 1 + k, 0), in - 1) == i) {
                acc += c[k];
                hit = true;
            }
        }
        if (hit && n < 8) {
            o[n] = d;
            w[n] = acc;
            ++n;
        }
    }
    return n;
}

// taps_of in a fixed-size form: the candidate outputs d0 .. d0 + 4 of input index i, bit t of `mask` set when
// output d0 + t reads i (w[t] its combined weight) -- the same entries in the same order as taps_of, but with
// compile-time indices, so the per-column tables stay in registers.
struct Taps5 {
    int d0;
    unsigned mask;
    float w[5];
};

__device__ __forceinline__ Taps5 taps5(int i, int in, int out, float scale) {
    Taps5 t;
    t.d0 = (int)floorf((i + 0.5f) / scale - 0.5f) - 2;
    t.mask = 0;
#pragma unroll
    for (int u = 0; u < 5; ++u) {
        const int d = t.d0 + u;
        t.w[u] = 0.f;
        if (d < 0 || d >= out) continue;
        const float r = scale * (d + 0.5f) - 0.5f;
        const int f = (int)floorf(r);
        float c[4];
        cubic_coeffs(r - f, c);
        float acc = 0.f;
        bool hit = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (min(max(f - 1 + k, 0), in - 1) == i) {
                acc += c[k];
                hit = true;
            }
        }
        if (hit) {
            t.w[u] = acc;
            t.mask |= 1u << u;
        }
    }
    return t;
}

// One workgroup per band of UB_R rows of one plane, UB_C consecutive 256-column strides per thread: the column taps
// depend only on the column and are computed once per workgroup (not once per pixel), the row taps once per row and
// thread.  Per pixel the terms and their order are those of the one-thread-per-pixel form (gather over the outputs
// whose taps read the pixel, rows outer), so dimg is bit-identical.
constexpr int UB_R = 8, UB_C = 4;

template <int MODE>
__global__ __launch_bounds__(256) void unprocess_bwd_kernel(const float* img, const float* dy, float* dimg,
                                                            int64_t planes, Unproc q) {
    const int bands = (q.in_h + UB_R - 1) / UB_R;
    const int64_t pl = blockIdx.x / bands;
    const int r0 = (int)(blockIdx.x - pl * bands) * UB_R;
    const int c = (int)(pl % q.channels);
    const float* d = dy + pl * (int64_t)q.out_h * q.out_w;
    const int64_t pbase = pl * (int64_t)q.in_h * q.in_w;
    for (int k0 = 0; k0 * 256 < q.in_w; k0 += UB_C) {
        Taps5 tx[UB_C];
#pragma unroll
        for (int k = 0; k < UB_C; ++k) {
            const int xx = threadIdx.x + 256 * (k0 + k);
            tx[k] = taps5(min(xx, q.in_w - 1), q.in_w, q.out_w, q.sx);
        }
        for (int yy = r0; yy < min(r0 + UB_R, q.in_h); ++yy) {
            const Taps5 ty = taps5(yy, q.in_h, q.out_h, q.sy);
#pragma unroll
            for (int k = 0; k < UB_C; ++k) {
                const int xx = threadIdx.x + 256 * (k0 + k);
                if (xx >= q.in_w) continue;
                const int64_t idx = pbase + (int64_t)yy * q.in_w + xx;
                float g = 0.f;
                if (ty.mask) {
#pragma unroll
                    for (int a = 0; a < 5; ++a) {
                        if (!((ty.mask >> a) & 1u)) continue;
                        const float* drow = d + (int64_t)(ty.d0 + a) * q.out_w;
                        float r = 0.f;
#pragma unroll
                        for (int bb = 0; bb < 5; ++bb)
                            if ((tx[k].mask >> bb) & 1u) r += drow[tx[k].d0 + bb] * tx[k].w[bb];
                        g += r * ty.w[a];
                    }
                    if (MODE == 0) {
                        const float x = __fadd_rn(__fmul_rn(img[idx], 127.5f), 128.f);
                        // d/dimg of (pre(img) / 255 - mean) / std; torch.clamp passes the gradient at the bounds
                        g = (x >= 0.f && x <= 255.f) ? g / q.std_[c] / 255.f * 127.5f : 0.f;
                    } else {
                        g = g / q.std_[c] * 0.5f;  // d/dimg of ((img + 1) / 2 - mean) / std after the (linear) resize
                    }
                }
                dimg[idx] = g;
            }
        }
    }
}

}  // namespace

namespace {

template <int MODE>
int preprocess_fwd(const char* name, const float* img, int n, int channels, int in_h, int in_w, int out_h, int out_w,
                   const float* mean, const float* std_, float* y, void* stream) {
    SMC_CHECK(img && y && mean && std_ && n >= 1 && channels >= 1, "%s: bad args", name);
    SMC_CHECK(in_h >= 1 && in_w >= 1 && out_h >= 1 && out_w >= 1, "%s: bad shape", name);
    const Unproc q{in_h, in_w, out_h, out_w, channels, (float)in_h / (float)out_h, (float)in_w / (float)out_w, mean,
                   std_};
    const int64_t planes = (int64_t)n * channels;
    hipLaunchKernelGGL(unprocess_fwd_kernel<MODE>, dim3((unsigned)smc::ceil_div(planes * out_h * out_w, 256)),
                       dim3(256), 0, smc::as_stream(stream), img, y, planes, q);
    return smc::check_launch(name);
}

template <int MODE>
int preprocess_bwd(const char* name, const float* img, const float* dy, int n, int channels, int in_h, int in_w,
                   int out_h, int out_w, const float* mean, const float* std_, float* dimg, void* stream) {
    SMC_CHECK(img && dy && dimg && mean && std_ && n >= 1 && channels >= 1, "%s: bad args", name);
    SMC_CHECK(in_h >= 1 && in_w >= 1 && out_h >= 1 && out_w >= 1, "%s: bad shape", name);
    const Unproc q{in_h, in_w, out_h, out_w, channels, (float)in_h / (float)out_h, (float)in_w / (float)out_w, mean,
                   std_};
    const int64_t planes = (int64_t)n * channels;
    const int64_t blocks = planes * smc::ceil_div(in_h, UB_R);
    hipLaunchKernelGGL(unprocess_bwd_kernel<MODE>, dim3((unsigned)blocks), dim3(256), 0, smc::as_stream(stream), img, dy,
                       dimg, planes, q);
    return smc::check_launch(name);
}

}  // namespace

SMC_API int smc_clip_unprocess_f32(const float* img, int n, int channels, int in_h, int in_w, int out_h, int out_w,
                                   const float* mean, const float* std_, float* y, void* stream) {
    return preprocess_fwd<0>("smc_clip_unprocess_f32", img, n, channels, in_h, in_w, out_h, out_w, mean, std_, y,
                             stream);
}

SMC_API int smc_clip_unprocess_bwd_f32(const float* img, const float* dy, int n, int channels, int in_h, int in_w,
                                       int out_h, int out_w, const float* mean, const float* std_, float* dimg,
                                       void* stream) {
    return preprocess_bwd<0>("smc_clip_unprocess_bwd_f32", img, dy, n, channels, in_h, in_w, out_h, out_w, mean,
                             std_, dimg, stream);
}

SMC_API int smc_clip_preprocess_nada_f32(const float* img, int n, int channels, int in_h, int in_w, int out_h,
                                         int out_w, const float* mean, const float* std_, float* y, void* stream) {
    return preprocess_fwd<1>("smc_clip_preprocess_nada_f32", img, n, channels, in_h, in_w, out_h, out_w, mean, std_,
                             y, stream);
}

SMC_API int smc_clip_preprocess_nada_bwd_f32(const float* img, const float* dy, int n, int channels, int in_h,
                                             int in_w, int out_h, int out_w, const float* mean, const float* std_,
                                             float* dimg, void* stream) {
    return preprocess_bwd<1>("smc_clip_preprocess_nada_bwd_f32", img, dy, n, channels, in_h, in_w, out_h, out_w,
                             mean, std_, dimg, stream);
}
