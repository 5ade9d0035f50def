// Row reductions of the loss heads, batch-invariant by construction.
//
// The loss heads reduce 512-wide embedding rows: norms, cosines and dot products (clip_loss.py:28-34,
// id_loss/id_loss.py:26-39, model_irse.py:48 l2_norm).  PyTorch's row reduction picks its block shape from the
// number of rows (ATen's reduce config: block width = 512 threads / block height, and the block height follows the
// row count), so a row reduced in a batch of 2 is summed in another order than the same row in a batch of 4.  Here one
// 64-lane wave owns one row whatever the batch: lane l accumulates elements l, l + 64, ... in order (fmaf), then a
// fixed xor-butterfly combines the lanes -- the data-parallel shard of an image computes its loss terms and
// gradient bit for bit as the whole batch does (find_direction's exact N-rank parity).
#include "common.hpp"

#include <cmath>

namespace {

__device__ __forceinline__ float wave_allsum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// out[r] = sum_k a[r, k] * b[r, k]; ldb = 0 broadcasts one row of b
__global__ __launch_bounds__(256) void row_dot_kernel(const float* a, int64_t lda, const float* b, int64_t ldb,
                                                      float* out, int rows, int len) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const float* ar = a + (int64_t)r * lda;
    const float* br = b + (int64_t)r * ldb;
    float acc = 0.f;
    for (int k = lane; k < len; k += 64) acc = fmaf(ar[k], br[k], acc);
    acc = wave_allsum(acc);
    if (lane == 0) out[r] = acc;
}

// The directional CLIP head per row (clip_loss.py:28-34 with the text direction t, one row broadcast):
//   f = e - src, u = f / |f|, cos = cosine_similarity(u, t) = (u . t) / (max(|u|, eps) max(|t|, eps)),
//   loss = 1 - cos and grad = d loss / d e, the exact gradient of 1 - cos(f, t) w.r.t. f: (cos uh - th) / |f| with
//   uh = f / |f|, th = t / |t|.
constexpr int kHeadMaxPer = 16;   // len <= 64 * 16 = 1024

__global__ __launch_bounds__(256) void direction_head_kernel(const float* e, int64_t lde, const float* src,
                                                             int64_t lds, const float* t, float* loss, float* grad,
                                                             int rows, int len, float eps) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    float f[kHeadMaxPer], tv[kHeadMaxPer];
    float ff = 0.f, tt = 0.f;
#pragma unroll
    for (int j = 0; j < kHeadMaxPer; ++j) {
        const int k = lane + 64 * j;
        const bool in = k < len;
        f[j] = in ? e[(int64_t)r * lde + k] - src[(int64_t)r * lds + k] : 0.f;
        tv[j] = in ? t[k] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < kHeadMaxPer; ++j) {
        ff = fmaf(f[j], f[j], ff);
        tt = fmaf(tv[j], tv[j], tt);
    }
    ff = wave_allsum(ff);
    tt = wave_allsum(tt);
    const float nf = sqrtf(ff);
    const float inv_nf = 1.f / nf;
    // u = f / |f| (the reference normalises first, clip_loss.py:30), then cosine_similarity(u, t)
    float uu = 0.f, ut = 0.f;
#pragma unroll
    for (int j = 0; j < kHeadMaxPer; ++j) {
        f[j] *= inv_nf;
        uu = fmaf(f[j], f[j], uu);
        ut = fmaf(f[j], tv[j], ut);
    }
    uu = wave_allsum(uu);
    ut = wave_allsum(ut);
    const float nu = fmaxf(sqrtf(uu), eps), nt = fmaxf(sqrtf(tt), eps);
    const float cos = ut / (nu * nt);
    if (lane == 0) loss[r] = 1.f - cos;
    const float inv_nu = 1.f / nu, inv_nt = 1.f / nt;
#pragma unroll
    for (int j = 0; j < kHeadMaxPer; ++j) {
        const int k = lane + 64 * j;
        if (k < len) grad[(int64_t)r * len + k] = (cos * (f[j] * inv_nu) - tv[j] * inv_nt) * inv_nf;
    }
}

}  // namespace

SMC_API int smc_row_dot_f32(const float* a, int64_t lda, const float* b, int64_t ldb, float* out, int rows, int len,
                            void* stream) {
    SMC_CHECK(a && b && out && rows >= 1 && len >= 1 && lda >= len && (ldb == 0 || ldb >= len),
              "smc_row_dot_f32: bad arguments");
    hipLaunchKernelGGL(row_dot_kernel, dim3((unsigned)smc::ceil_div(rows, 4)), dim3(256), 0, smc::as_stream(stream),
                       a, lda, b, ldb, out, rows, len);
    return smc::check_launch("smc_row_dot_f32");
}

SMC_API int smc_direction_head_f32(const float* e, int64_t lde, const float* src, int64_t lds, const float* t,
                                   float* loss, float* grad, int rows, int len, float eps, void* stream) {
    SMC_CHECK(e && src && t && loss && grad && rows >= 1 && len >= 1 && lde >= len && lds >= len,
              "smc_direction_head_f32: bad arguments");
    if (len > 64 * kHeadMaxPer) {
        smc::set_error("smc_direction_head_f32: embedding width %d > %d", len, 64 * kHeadMaxPer);
        return SMC_ERR_UNSUPPORTED;
    }
    hipLaunchKernelGGL(direction_head_kernel, dim3((unsigned)smc::ceil_div(rows, 4)), dim3(256), 0,
                       smc::as_stream(stream), e, lde, src, lds, t, loss, grad, rows, len, eps);
    return smc::check_launch("smc_direction_head_f32");
}
