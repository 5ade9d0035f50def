// IDLoss face crop for gfx950: adaptive-avg-pool to (pool_h, pool_w) -> crop -> adaptive-avg-pool to
// (out_h, out_w) in one pass, and its gradient.
//
// Replaces the three PyTorch ops of id_loss.py:20-23 (F.adaptive_avg_pool2d(x, 256), the [35:223, 32:220]
// crop, F.adaptive_avg_pool2d(., 112)) on the IR-SE50 input path: at 1024 px the first pool is an exact
// 4x4 mean, the second averages windows [floor(i*188/112), ceil((i+1)*188/112)) of 1-2 pooled cells.
// Forward: one thread per output element, float4 row reads of each 4-wide pooled cell.  Backward: one
// thread per 4 input pixels of a row (they share a pooled cell), writing the whole input gradient
// (zeros outside the crop) -- the atomic scatter of aten's adaptive-pool backward is not needed because
// every pooled cell knows the <= 2 x 2 output windows that cover it.
#include "common.hpp"

namespace {

struct FaceCrop {
    int in_h, in_w, kh, kw;           // first pool: integer factors (in = pool * k)
    int cy0, cx0, ch, cw;             // crop of the pooled image
    int out_h, out_w;
};

__device__ __forceinline__ int win_lo(int i, int in, int out) { return (i * in) / out; }
__device__ __forceinline__ int win_hi(int i, int in, int out) { return ((i + 1) * in + out - 1) / out; }

// mean of the pooled cell (py, px) of plane xp
__device__ __forceinline__ float pooled(const float* xp, const FaceCrop& q, int py, int px, bool vec) {
    float s = 0.f;
    const float* row = xp + (int64_t)py * q.kh * q.in_w + (int64_t)px * q.kw;
    for (int a = 0; a < q.kh; ++a) {
        const float* r = row + (int64_t)a * q.in_w;
        if (vec) {
            const float4 v = *reinterpret_cast<const float4*>(r);
            s += ((v.x + v.y) + v.z) + v.w;
        } else {
            for (int b = 0; b < q.kw; ++b) s += r[b];
        }
    }
    return s / (float)(q.kh * q.kw);
}

__global__ __launch_bounds__(256) void face_crop_fwd_kernel(const float* x, float* y, int64_t planes, FaceCrop q,
                                                            bool vec) {
    const int64_t per = (int64_t)q.out_h * q.out_w;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= planes * per) return;
    const int64_t pl = idx / per;
    const int rem = (int)(idx - pl * per);
    const int i = rem / q.out_w, j = rem - (rem / q.out_w) * q.out_w;
    const float* xp = x + pl * (int64_t)q.in_h * q.in_w;
    const int y0 = win_lo(i, q.ch, q.out_h), y1 = win_hi(i, q.ch, q.out_h);
    const int x0 = win_lo(j, q.cw, q.out_w), x1 = win_hi(j, q.cw, q.out_w);
    float s = 0.f;
    for (int py = y0; py < y1; ++py)
        for (int px = x0; px < x1; ++px) s += pooled(xp, q, q.cy0 + py, q.cx0 + px, vec);
    y[idx] = s / (float)((y1 - y0) * (x1 - x0));
}

// gradient of the pooled cell (py, px) (pooled-image coordinates) from the output windows covering it
__device__ __forceinline__ float dpooled(const float* dyp, const FaceCrop& q, int py, int px) {
    const int cy = py - q.cy0, cx = px - q.cx0;
    if (cy < 0 || cy >= q.ch || cx < 0 || cx >= q.cw) return 0.f;
    // output rows whose window [lo, hi) contains cy: i in [i_lo, i_hi]
    const int i_lo = (cy * q.out_h) / q.ch > 0 ? (cy * q.out_h) / q.ch - 1 : 0;
    const int j_lo = (cx * q.out_w) / q.cw > 0 ? (cx * q.out_w) / q.cw - 1 : 0;
    float g = 0.f;
    for (int i = i_lo; i < q.out_h && win_lo(i, q.ch, q.out_h) <= cy; ++i) {
        const int y0 = win_lo(i, q.ch, q.out_h), y1 = win_hi(i, q.ch, q.out_h);
        if (cy >= y1) continue;
        for (int j = j_lo; j < q.out_w && win_lo(j, q.cw, q.out_w) <= cx; ++j) {
            const int x0 = win_lo(j, q.cw, q.out_w), x1 = win_hi(j, q.cw, q.out_w);
            if (cx >= x1) continue;
            g += dyp[(int64_t)i * q.out_w + j] / (float)((y1 - y0) * (x1 - x0));
        }
    }
    return g / (float)(q.kh * q.kw);
}

__global__ __launch_bounds__(256) void face_crop_bwd_kernel(const float* dy, float* dx, int64_t planes, FaceCrop q) {
    // one thread per kw-wide group of a row (= one pooled cell's row segment)
    const int pw = q.in_w / q.kw;
    const int64_t per = (int64_t)q.in_h * pw;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= planes * per) return;
    const int64_t pl = idx / per;
    const int rem = (int)(idx - pl * per);
    const int yy = rem / pw, px = rem - (rem / pw) * pw;
    const float g = dpooled(dy + pl * (int64_t)q.out_h * q.out_w, q, yy / q.kh, px);
    float* d = dx + pl * (int64_t)q.in_h * q.in_w + (int64_t)yy * q.in_w + (int64_t)px * q.kw;
    if (q.kw == 4 && (q.in_w & 3) == 0) {
        *reinterpret_cast<float4*>(d) = make_float4(g, g, g, g);
    } else {
        for (int b = 0; b < q.kw; ++b) d[b] = g;
    }
}

int make_q(int in_h, int in_w, int pool_h, int pool_w, int crop_y0, int crop_x0, int crop_h, int crop_w, int out_h,
           int out_w, FaceCrop* q) {
    SMC_CHECK(in_h >= 1 && in_w >= 1 && pool_h >= 1 && pool_w >= 1 && out_h >= 1 && out_w >= 1,
              "smc_face_crop: bad shape");
    if (in_h % pool_h || in_w % pool_w) {
        smc::set_error("smc_face_crop: input %dx%d is not an integer multiple of the pool %dx%d", in_h, in_w, pool_h,
                       pool_w);
        return SMC_ERR_UNSUPPORTED;
    }
    SMC_CHECK(crop_y0 >= 0 && crop_x0 >= 0 && crop_h >= 1 && crop_w >= 1 && crop_y0 + crop_h <= pool_h &&
                  crop_x0 + crop_w <= pool_w,
              "smc_face_crop: crop outside the pooled image");
    SMC_CHECK(out_h <= crop_h && out_w <= crop_w, "smc_face_crop: output larger than the crop");
    *q = FaceCrop{in_h, in_w, in_h / pool_h, in_w / pool_w, crop_y0, crop_x0, crop_h, crop_w, out_h, out_w};
    return SMC_OK;
}

}  // namespace

SMC_API int smc_face_crop_f32(const float* x, int64_t planes, int in_h, int in_w, int pool_h, int pool_w, int crop_y0,
                              int crop_x0, int crop_h, int crop_w, int out_h, int out_w, float* y, void* stream) {
    SMC_CHECK(x && y && planes >= 1, "smc_face_crop_f32: bad args");
    FaceCrop q;
    const int rc = make_q(in_h, in_w, pool_h, pool_w, crop_y0, crop_x0, crop_h, crop_w, out_h, out_w, &q);
    if (rc != SMC_OK) return rc;
    const bool vec = q.kw == 4 && (in_w & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    const int64_t total = planes * out_h * out_w;
    hipLaunchKernelGGL(face_crop_fwd_kernel, dim3((unsigned)smc::ceil_div(total, 256)), dim3(256), 0,
                       smc::as_stream(stream), x, y, planes, q, vec);
    return smc::check_launch("smc_face_crop_f32");
}

SMC_API int smc_face_crop_bwd_f32(const float* dy, int64_t planes, int in_h, int in_w, int pool_h, int pool_w,
                                  int crop_y0, int crop_x0, int crop_h, int crop_w, int out_h, int out_w, float* dx,
                                  void* stream) {
    SMC_CHECK(dy && dx && planes >= 1, "smc_face_crop_bwd_f32: bad args");
    FaceCrop q;
    const int rc = make_q(in_h, in_w, pool_h, pool_w, crop_y0, crop_x0, crop_h, crop_w, out_h, out_w, &q);
    if (rc != SMC_OK) return rc;
    SMC_CHECK(q.kw != 4 || (reinterpret_cast<uintptr_t>(dx) & 15) == 0, "smc_face_crop_bwd_f32: dx not 16-B aligned");
    const int64_t total = planes * in_h * (in_w / q.kw);
    hipLaunchKernelGGL(face_crop_bwd_kernel, dim3((unsigned)smc::ceil_div(total, 256)), dim3(256), 0,
                       smc::as_stream(stream), dy, dx, planes, q);
    return smc::check_launch("smc_face_crop_bwd_f32");
}
