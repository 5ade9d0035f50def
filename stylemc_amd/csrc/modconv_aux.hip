// Memory-bound companions of the modconv GEMM for gfx950:
//   * split-K reduction + modconv epilogue            (smc_modconv_epilogue_f32)
//   * conv0's fused 4x4 blur + modconv epilogue       (smc_modconv_blur_act_f32)
//   * demodulation d = rsqrt(s^2 . Wsq + eps)         (smc_modconv_demod_f32, one wave per (n,o),
//                                                       wavefront-shuffle reduction)
//   * epilogue backward + d-gradient reduction        (smc_modconv_act_bwd_f32)
//   * per-channel dot products for style gradients    (smc_channel_dot_f32)
//   * gradient through the demodulation               (smc_modconv_demod_bwd_f32)
// The forward replaces the bias_act / upfirdn2d / fma launches the reference issues after each
// grouped conv ([upstream] SynthesisLayer.forward -> bias_act.py:153, upfirdn2d.py:237, fma.py:15).
#include "common.hpp"

namespace {

struct Epi {
    int mode;
    const float* d;
    const float* noise;
    int64_t noise_nstride;
    const float* noise_strength;
    const float* bias;
    int act;
    float alpha, gain, clamp;
    float* u_save;
    smc::EpiExt ext;
    int grad_from_y;
    float* dd_part;  // set: the act / FIR backward kernels store their per-tile dd partials here (dd_sum_kernel adds them)
};

Epi to_epi(const smc_conv_epilogue* e) {
    Epi r{};
    r.mode = SMC_EPI_STORE;
    r.act = SMC_ACT_LINEAR;
    r.gain = 1.f;
    r.clamp = -1.f;
    if (e) {
        r.mode = e->mode; r.d = e->d; r.noise = e->noise; r.noise_nstride = e->noise_nstride;
        r.noise_strength = e->noise_strength; r.bias = e->bias; r.act = e->act; r.alpha = e->alpha;
        r.gain = e->gain; r.clamp = e->clamp; r.u_save = e->u_save; r.grad_from_y = e->grad_from_y;
    }
    r.ext = smc::epi_ext(e);
    return r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Block-wide sum of 256 threads; result valid in every thread.
__device__ __forceinline__ float block_sum256(float v, float* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// ---------------------------------------------------------------------------------------------- epilogue

__global__ __launch_bounds__(256) void epilogue_kernel(const float* src, int nsplit, int64_t split_stride, float* y,
                                                       int c, int h, int w, int64_t total, Epi e) {
    const float nstr = e.noise_strength ? *e.noise_strength : 1.f;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t hw = (int64_t)h * w;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += stride) {
        // partials 8 at a time, all loads in flight before the adds (in split order, as one at a time)
        float v = src[idx];
        for (int s0 = 1; s0 < nsplit; s0 += 8) {
            float t[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = src[min(s0 + k, nsplit - 1) * split_stride + idx];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (s0 + k < nsplit) v += t[k];
        }
        if (e.mode == SMC_EPI_STORE && !e.ext.residual) {
            y[idx] = v;
            continue;
        }
        const int64_t nc = idx / hw;
        const int64_t pix = idx - nc * hw;
        const int n = (int)(nc / c), o = (int)(nc - (int64_t)n * c);
        const int yy = (int)(pix / w), xx = (int)(pix - (int64_t)yy * w);
        if (e.mode == SMC_EPI_MODACT) {
            if (e.u_save) e.u_save[idx] = v;
            const float nz = e.noise ? e.noise[n * e.noise_nstride + pix] * nstr : 0.f;
            const float dd = (e.d ? e.d[nc] : 1.f) * (e.ext.scale_c ? e.ext.scale_c[o] : 1.f);
            float r = smc::epi_y(v, dd, nz, e.bias ? e.bias[o] : 0.f, e.act, e.alpha, e.gain, e.clamp);
            if (e.ext.residual) r = smc::epi_ext_apply(SMC_EPI_STORE, r, n, o, idx, yy, xx, c, h, w, nullptr, nullptr, e.ext);
            y[idx] = r;
        } else {
            y[idx] = smc::epi_ext_apply(e.mode, v, n, o, idx, yy, xx, c, h, w, e.bias, e.u_save, e.ext);
        }
    }
}

// ---------------------------------------------------------------------------------------------- blur + act

constexpr int kBT = 32;        // output tile (kBT x kBT), 256 threads x 4 rows
constexpr int kMaxF = 8;

__global__ __launch_bounds__(256) void blur_act_kernel(const float* t, int nsplit, int64_t split_stride, float* y,
                                                       int c, int t_h, int t_w, int tp_w, int y_h, int y_w,
                                                       const float* f, int fh, int fw, int padx0, int pady0, float fgain,
                                                       int flip, Epi e) {
    __shared__ float tile[(kBT + kMaxF - 1) * (kBT + kMaxF - 1)];
    __shared__ float taps[kMaxF * kMaxF];
    const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;
    const int ox0 = blockIdx.x * kBT, oy0 = blockIdx.y * kBT;
    const int64_t nc = blockIdx.z;
    const int n = (int)(nc / c), o = (int)(nc - (int64_t)n * c);
    if (tid < fh * fw) {
        const int jy = tid / fw, jx = tid % fw;
        taps[tid] = f[(flip ? jy : fh - 1 - jy) * fw + (flip ? jx : fw - 1 - jx)] * fgain;
    }
    const int rows = kBT + fh - 1, cols = kBT + fw - 1;
    const int iy0 = oy0 - pady0, ix0 = ox0 - padx0;
    const float* tp = t + nc * (int64_t)t_h * tp_w;
    for (int i = tid; i < rows * cols; i += 256) {
        const int r = i / cols, cc = i - r * cols;
        const int iy = iy0 + r, ix = ix0 + cc;
        float v = 0.f;
        if (iy >= 0 && iy < t_h && ix >= 0 && ix < t_w) {
            const int64_t off = (int64_t)iy * tp_w + ix;
            v = tp[off];
            for (int s = 1; s < nsplit; ++s) v += tp[s * split_stride + off];
        }
        tile[i] = v;
    }
    __syncthreads();
    const float nstr = e.noise_strength ? *e.noise_strength : 1.f;
    const float dv = e.d ? e.d[nc] : 1.f;
    const float bv = e.bias ? e.bias[o] : 0.f;
    const int ox = ox0 + tx;
    if (ox >= y_w) return;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int oy = oy0 + ty + 8 * k;
        if (oy >= y_h) continue;
        const int ly = ty + 8 * k;
        float u = 0.f;
        for (int jy = 0; jy < fh; ++jy) {
            const float* trow = tile + (ly + jy) * cols + tx;
            const float* frow = taps + jy * fw;
            for (int jx = 0; jx < fw; ++jx) u += frow[jx] * trow[jx];
        }
        const int64_t pix = (int64_t)oy * y_w + ox;
        const int64_t idx = nc * (int64_t)y_h * y_w + pix;
        if (e.mode == SMC_EPI_STORE) {
            y[idx] = u;
            continue;
        }
        if (e.u_save) e.u_save[idx] = u;
        const float nz = e.noise ? e.noise[n * e.noise_nstride + pix] * nstr : 0.f;
        y[idx] = smc::epi_y(u, dv, nz, bv, e.act, e.alpha, e.gain, e.clamp);
    }
}

// ---------------------------------------------------------------------------------------------- 4x4 FIR fast path
// Output tile 32 rows x 64 columns per 256-thread workgroup; every thread produces a 4x2 block from a
// (4+FH-1) x (2+FW-1) register window of the LDS tile (35 LDS reads for 8 outputs instead of 128).

constexpr int kFH = 32, kFW = 64;
// Grids of the 4x4 FIR kernels.  The const [H, W] noise is read by every plane, so dispatch order decides whether a
// noise tile is still in an XCD's L2 when the next plane needs it (workgroup ids go round-robin over the 8 XCDs).
// Backward: (planes, column tiles, row tiles) -- one spatial tile's planes are consecutive ids, 1/8 of them per
// XCD back to back (r = 1024 HBM reads 3.0 -> 1.2 GB, 651 -> 453 us; grad_from_y 375 -> 358 us).  Forward:
// (column tiles, row tiles, planes) -- it writes two planes (y, u) and the plane-major order's write locality wins
// over the noise re-reads it saves (measured 426 us vs 464 planes-fastest, 445 with planes in the middle).
inline dim3 fir_grid_bwd(int64_t planes, int w, int h) {
    return dim3((unsigned)planes, (unsigned)smc::ceil_div(w, kFW), (unsigned)smc::ceil_div(h, kFH));
}
inline dim3 fir_grid_fwd(int64_t planes, int w, int h) {
    return dim3((unsigned)smc::ceil_div(w, kFW), (unsigned)smc::ceil_div(h, kFH), (unsigned)planes);
}

// (explicit fmaf: every kernel that shares these helpers rounds the same way whatever the compiler's contraction and
// packed-math choices in its context -- the 16-B, strip and scalar-load kernels agree bit for bit)
template <int FH, int FW>
__device__ __forceinline__ void fir_block(const float* tile, int stride, int ly0, int lx0, const float (&tp)[FH][FW],
                                          float (&out)[4][2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i][0] = out[i][1] = 0.f;
#pragma unroll
    for (int r = 0; r < 4 + FH - 1; ++r) {
        float v[2 + FW - 1];
#pragma unroll
        for (int c = 0; c < 2 + FW - 1; ++c) v[c] = tile[(ly0 + r) * stride + lx0 + c];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int jy = r - i;
            if (jy < 0 || jy >= FH) continue;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int jx = 0; jx < FW; ++jx) out[i][j] = __fmaf_rn(tp[jy][jx], v[j + jx], out[i][j]);
        }
    }
}

// As fir_block, but the thread's two output columns are lx0 and lx0 + 32: a wave's store instruction then
// covers 32 consecutive columns of two rows (two 128-B segments) instead of every other column.
template <int FH, int FW>
__device__ __forceinline__ void fir_block_split(const float* tile, int stride, int ly0, int lx0,
                                                const float (&tp)[FH][FW], float (&out)[4][2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i][0] = out[i][1] = 0.f;
#pragma unroll
    for (int r = 0; r < 4 + FH - 1; ++r) {
        float v[2][FW];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int c = 0; c < FW; ++c) v[j][c] = tile[(ly0 + r) * stride + lx0 + 32 * j + c];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int jy = r - i;
            if (jy < 0 || jy >= FH) continue;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int jx = 0; jx < FW; ++jx) out[i][j] = __fmaf_rn(tp[jy][jx], v[j][jx], out[i][j]);
        }
    }
}

template <int FH, int FW>
__device__ __forceinline__ void load_taps(const float* f, int flip, float fgain, float (&tp)[FH][FW]) {
    if (FH == 4 && FW == 4 && !f) {  // the built-in [1,3,3,1] resample filter (f = NULL): see std_taps
        constexpr float k[4] = {1.f, 3.f, 3.f, 1.f};
#pragma unroll
        for (int jy = 0; jy < FH; ++jy)
#pragma unroll
            for (int jx = 0; jx < FW; ++jx) tp[jy][jx] = k[jy] * k[jx] * (1.f / 64.f) * fgain;
        return;
    }
#pragma unroll
    for (int jy = 0; jy < FH; ++jy)
#pragma unroll
        for (int jx = 0; jx < FW; ++jx)
            tp[jy][jx] = f[(flip ? jy : FH - 1 - jy) * FW + (flip ? jx : FW - 1 - jx)] * fgain;
}

// The synthesis' resample filter, setup_filter([1,3,3,1]) = k k^T / 64, times the conv0 FIR gain 4, as compile-time
// constants k_i k_j / 16 (exact in fp32, equal bit for bit to the values load_taps reads and scales): the FMAs take
// literal operands and the 16 taps need no registers (blur_act_v4: 140 -> fewer VGPRs, more waves per SIMD for a
// memory-bound kernel).  Symmetric, so the flip does not matter.
template <int FH, int FW>
__device__ __forceinline__ void std_taps(float (&tp)[FH][FW]) {
    constexpr float k[4] = {1.f, 3.f, 3.f, 1.f};
#pragma unroll
    for (int jy = 0; jy < FH; ++jy)
#pragma unroll
        for (int jx = 0; jx < FW; ++jx) tp[jy][jx] = k[jy] * k[jx] * 0.0625f;
}

// Forward conv0 epilogue: U = FIR(T) (1:1, pad (pady0, padx0)), y = epi(U); stores y and U.
template <int FH, int FW>
__global__ __launch_bounds__(256) void blur_act_fast(const float* t, int nsplit, int64_t split_stride, float* y, int c,
                                                     int t_h, int t_w, int tp_w, int y_h, int y_w, const float* f,
                                                     int padx0, int pady0, float fgain, int flip, Epi e) {
    constexpr int ROWS = kFH + FH - 1, COLS = kFW + FW - 1, STRIDE = COLS + 1;
    __shared__ float tile[ROWS * STRIDE];
    const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;
    const int ox0 = blockIdx.x * kFW, oy0 = blockIdx.y * kFH;  // fir_grid_fwd
    const int64_t nc = blockIdx.z;
    const int n = (int)(nc / c), o = (int)(nc - (int64_t)n * c);
    float tp[FH][FW];
    load_taps<FH, FW>(f, flip, fgain, tp);
    const int iy0 = oy0 - pady0, ix0 = ox0 - padx0;
    const float* tpl = t + nc * (int64_t)t_h * tp_w;
    // Haloed tile load with a fixed, unrolled trip count: every load of the thread is in flight before
    // the first LDS store (a data-dependent loop serialises one HBM latency per element).  Out-of-range
    // elements load the plane's first float (always valid) and are zeroed by select.
    constexpr int NL = (ROWS * COLS + 255) / 256;
    float v[NL];
    int off[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        const int i = tid + 256 * l;
        const int r = i / COLS, cc = i - r * COLS;
        const int iy = iy0 + r, ix = ix0 + cc;
        const bool ok = i < ROWS * COLS && iy >= 0 && iy < t_h && ix >= 0 && ix < t_w;
        off[l] = ok ? iy * tp_w + ix : -1;
        const float a = tpl[ok ? off[l] : 0];
        v[l] = ok ? a : 0.f;
    }
    for (int s = 1; s < nsplit; ++s) {
        const float* sp = tpl + s * split_stride;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const float a = sp[off[l] >= 0 ? off[l] : 0];
            v[l] += off[l] >= 0 ? a : 0.f;
        }
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        const int i = tid + 256 * l;
        const int r = i / COLS, cc = i - r * COLS;
        if (i < ROWS * COLS) tile[r * STRIDE + cc] = v[l];
    }
    __syncthreads();
    float out[4][2];
    fir_block<FH, FW>(tile, STRIDE, 4 * ty, 2 * tx, tp, out);
    const float nstr = e.noise_strength ? *e.noise_strength : 1.f;
    const float dv = e.d ? e.d[nc] : 1.f;
    const float bv = e.bias ? e.bias[o] : 0.f;
    const int64_t plane = nc * (int64_t)y_h * y_w;
    const int ox = ox0 + 2 * tx;
    if (ox >= y_w) return;
    // y_w even (all synthesis resolutions) and ox even: the thread's two columns are one aligned float2
    const bool pair = (y_w & 1) == 0 && ((e.noise_nstride & 1) == 0) &&
                      (((uintptr_t)y | (uintptr_t)e.u_save | (uintptr_t)e.noise) & 7) == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int oy = oy0 + 4 * ty + i;
        if (oy >= y_h) continue;
        const int64_t pix = (int64_t)oy * y_w + ox;
        if (pair) {
            const float2 u2 = make_float2(out[i][0], out[i][1]);
            if (e.mode == SMC_EPI_STORE) {
                *reinterpret_cast<float2*>(y + plane + pix) = u2;
                continue;
            }
            if (e.u_save) *reinterpret_cast<float2*>(e.u_save + plane + pix) = u2;
            float2 nz = make_float2(0.f, 0.f);
            if (e.noise) {
                nz = *reinterpret_cast<const float2*>(e.noise + n * e.noise_nstride + pix);
                nz.x *= nstr;
                nz.y *= nstr;
            }
            *reinterpret_cast<float2*>(y + plane + pix) =
                make_float2(smc::epi_y(u2.x, dv, nz.x, bv, e.act, e.alpha, e.gain, e.clamp),
                            smc::epi_y(u2.y, dv, nz.y, bv, e.act, e.alpha, e.gain, e.clamp));
            continue;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (ox + j >= y_w) continue;
            const float u = out[i][j];
            if (e.mode == SMC_EPI_STORE) {
                y[plane + pix + j] = u;
                continue;
            }
            if (e.u_save) e.u_save[plane + pix + j] = u;
            const float nz = e.noise ? e.noise[n * e.noise_nstride + pix + j] * nstr : 0.f;
            y[plane + pix + j] = smc::epi_y(u, dv, nz, bv, e.act, e.alpha, e.gain, e.clamp);
        }
    }
}

// blur_act_fast with 16-B loads.  Each haloed tile row is fetched as the 16-B aligned float4 groups (aligned in the
// buffer, so any row pitch works -- the transposed conv's odd 2h + 1 width included) that cover
// [ox0 - 4, ox0 + kFW + 4): a third of the load instructions of the scalar form, every one a full 16 B; the groups'
// elements outside the tile window, the image width or the row are dropped / zeroed on the way into LDS.
// Needs a 16-B aligned t, split_stride % 4 == 0, padx0 <= 4 and FW - 1 - padx0 <= 4.
#ifndef SMC_BLUR_TPB
#define SMC_BLUR_TPB 4
#endif
#ifndef SMC_BLUR_NT
#define SMC_BLUR_NT 1
#endif
// workgroups per CU the built-in-tap FIR forward is compiled for (A/B knob; profiles/r05/fir_ab/: 4 -> 103 VGPRs, no
// spill, r = 1024 338 us; 5 -> 96 VGPRs with a 20-B spill, 372 us; runtime taps 140 VGPRs, 3 waves per SIMD, 375 us)
#ifndef SMC_BLUR_WGS
#define SMC_BLUR_WGS 4
#endif
#ifndef SMC_BLUR_STDF
#define SMC_BLUR_STDF 1
#endif
// the next row tile's loads issued before this tile's FIR and stores (A/B knob)
#ifndef SMC_BLUR_PIPE
#define SMC_BLUR_PIPE 1
#endif
template <bool NT>
__device__ __forceinline__ void st_f2(float* p, float2 v) {
    if (NT) {
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(f32x2{v.x, v.y}, reinterpret_cast<f32x2*>(p));   // one dwordx2 store
    } else {
        *reinterpret_cast<float2*>(p) = v;
    }
}

// TPB: row tiles per workgroup (grid.y = ceil(row tiles / TPB)), NT: non-temporal y / u stores (nothing reads y / u
// before the next layer's conv has streamed the whole plane set).  Measured (profiles/r04/blur_ab/, bit-identical y):
// TPB 4 + NT 712 -> 650 us over the five conv0 layers; TPB 8 / 16 no better; the same on the backward lost (dT is read
// right away by the transposed conv's data gradient).
template <int FH, int FW, int TPB, bool NT, bool STDF = false>
__global__ __launch_bounds__(256, STDF ? SMC_BLUR_WGS : 1) void blur_act_v4(const float* t, int nsplit, int64_t split_stride, float* y, int c,
                                                   int t_h, int t_w, int tp_w, int y_h, int y_w, const float* f,
                                                   int padx0, int pady0, float fgain, int flip, Epi e) {
    constexpr int ROWS = kFH + FH - 1, COLS = kFW + FW - 1, STRIDE = COLS + 1;
    constexpr int G4 = (kFW + 8) / 4 + 1;               // float4 groups per tile row (+1: row misalignment)
    constexpr int NL = (ROWS * G4 + 255) / 256;
    __shared__ float tile[ROWS * STRIDE];
    const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;
    const int ox0 = blockIdx.x * kFW;
    const int64_t nc = blockIdx.z;
    const int n = (int)(nc / c), o = (int)(nc - (int64_t)n * c);
    float tp[FH][FW];
    if constexpr (STDF) std_taps<FH, FW>(tp);
    else load_taps<FH, FW>(f, flip, fgain, tp);
    const float nstr = e.noise_strength ? *e.noise_strength : 1.f;
    const float dv = e.d ? e.d[nc] : 1.f;
    const float bv = e.bias ? e.bias[o] : 0.f;
    const int ix0 = ox0 - padx0;
    const int64_t pbase = nc * (int64_t)t_h * tp_w;
    // (16-B alignment of the groups: the plane base's offset mod 4 floats; the groups are aligned in the buffer)
    const int pmis = (int)(pbase & 3);
    const float* tpl = t + (pbase - pmis);        // 16-B aligned; plane element e sits at tpl[e + pmis]
    float4 v[NL];
    int off[NL];   // plane-relative (+ pmis) index of the group's first element, -1: no valid element
    int gx[NL];    // image column of the group's first element
    // tile tb's haloed rows into registers (issued one tile ahead: their HBM latency runs under the previous tile's
    // FIR and stores)
    auto load_tile = [&](int tb) {
        const int iy0 = (blockIdx.y * TPB + tb) * kFH - pady0;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int i = tid + 256 * l;
            const int r = i / G4, q = i - r * G4;
            const int iy = iy0 + r;
            const int row = pmis + iy * tp_w;                 // of the aligned base
            const int g0 = ((row + ox0 - 4) & ~3) + 4 * q;
            gx[l] = g0 - row;
            const bool ok = i < ROWS * G4 && iy >= 0 && iy < t_h && gx[l] + 3 >= 0 && gx[l] < t_w;
            off[l] = ok ? g0 : -1;
            v[l] = *reinterpret_cast<const float4*>(tpl + (ok ? g0 : 0));
        }
    };
    if (blockIdx.y * TPB * kFH < y_h) load_tile(0);
    for (int tb = 0; tb < TPB; ++tb) {
        const int oy0 = (blockIdx.y * TPB + tb) * kFH;
        if (oy0 >= y_h) break;
        if (tb > 0) __syncthreads();  // the previous tile's FIR reads are done
        if (!SMC_BLUR_PIPE && tb > 0) load_tile(tb);
        for (int s = 1; s < nsplit; ++s) {
            const float* sp = tpl + s * split_stride;
#pragma unroll
            for (int l = 0; l < NL; ++l) {
                const float4 a = *reinterpret_cast<const float4*>(sp + (off[l] >= 0 ? off[l] : 0));
                v[l].x += a.x; v[l].y += a.y; v[l].z += a.z; v[l].w += a.w;
            }
        }
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int i = tid + 256 * l;
            if (i >= ROWS * G4) continue;
            const int r = i / G4;
            const float a[4] = {v[l].x, v[l].y, v[l].z, v[l].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int ix = gx[l] + k;
                const int cc = ix - ix0;
                if (cc >= 0 && cc < COLS) tile[r * STRIDE + cc] = (off[l] >= 0 && ix >= 0 && ix < t_w) ? a[k] : 0.f;
            }
        }
        __syncthreads();
        if (SMC_BLUR_PIPE && tb + 1 < TPB && oy0 + kFH < y_h) load_tile(tb + 1);
        float out[4][2];
        fir_block<FH, FW>(tile, STRIDE, 4 * ty, 2 * tx, tp, out);
        const int64_t plane = nc * (int64_t)y_h * y_w;
        const int ox = ox0 + 2 * tx;
        if (ox >= y_w) continue;
        // the 4 rows' noise is loaded before the first store (loaded next to each store, every row would wait for the
        // previous row's stores: vmcnt counts both)
        float2 nz[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int oy = min(oy0 + 4 * ty + i, y_h - 1);
            nz[i] = make_float2(0.f, 0.f);
            if (e.mode != SMC_EPI_STORE && e.noise) {
                nz[i] = *reinterpret_cast<const float2*>(e.noise + n * e.noise_nstride + (int64_t)oy * y_w + ox);
                nz[i].x *= nstr;
                nz[i].y *= nstr;
            }
        }
        // the synthesis' conv0 epilogue (lrelu with 0 <= alpha <= 1, gain, clamp >= 0) with the activation fixed at
        // compile time: max / min forms, bit-identical to smc::epi_y for finite values
        const bool lrelu_clamp = e.act == SMC_ACT_LRELU && e.alpha >= 0.f && e.alpha <= 1.f && e.clamp >= 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int oy = oy0 + 4 * ty + i;
            if (oy >= y_h) continue;
            const int64_t pix = (int64_t)oy * y_w + ox;
            const float2 u2 = make_float2(out[i][0], out[i][1]);
            if (e.mode == SMC_EPI_STORE) {
                st_f2<NT>(y + plane + pix, u2);
                continue;
            }
            if (e.u_save) st_f2<NT>(e.u_save + plane + pix, u2);
            float2 q;
            if (lrelu_clamp) {
                const float zx = __fmaf_rn(u2.x, dv, nz[i].x) + bv, zy = __fmaf_rn(u2.y, dv, nz[i].y) + bv;
                q.x = smc::lrelu_gain_clamp(zx, e.alpha, e.gain, e.clamp);
                q.y = smc::lrelu_gain_clamp(zy, e.alpha, e.gain, e.clamp);
            } else {
                q = make_float2(smc::epi_y(u2.x, dv, nz[i].x, bv, e.act, e.alpha, e.gain, e.clamp),
                                smc::epi_y(u2.y, dv, nz[i].y, bv, e.act, e.alpha, e.gain, e.clamp));
            }
            st_f2<NT>(y + plane + pix, q);
        }
    }
}

// Backward of conv0's epilogue + FIR in one pass: du = act'(g; y(u)) * d (re-derived per element of the
// haloed tile), dT = FIR^T(du) (pad (pady0, padx0) of the adjoint), dd[n,o] += sum dz*u over the du
// positions this tile owns (its own 32x64 window, so every position is counted exactly once).
// FROMY (epi.grad_from_y): `u` holds the forward output y -- the mask needs nothing else; no noise read, no dd.
template <int FH, int FW, bool V2 = false, bool FROMY = false>
__global__ __launch_bounds__(256) void blur_act_bwd_fast(const float* g, const float* u, float* dt, float* dd, int c,
                                                         int u_h, int u_w, int t_h, int t_w, int tp_w, const float* f,
                                                         int padx0,
                                                         int pady0, float fgain, int flip, Epi e) {
    constexpr int ROWS = kFH + FH - 1, COLS = kFW + FW - 1, STRIDE = COLS + 1;
    __shared__ __attribute__((aligned(16))) float tile[ROWS * STRIDE];
    __shared__ float red[4];
    const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;
    const int ox0 = blockIdx.y * kFW, oy0 = blockIdx.z * kFH;  // fir_grid_bwd
    const int64_t nc = blockIdx.x;
    const int n = (int)(nc / c), o = (int)(nc - (int64_t)n * c);
    float tp[FH][FW];
    load_taps<FH, FW>(f, flip, fgain, tp);
    const float nstr = e.noise_strength ? *e.noise_strength : 1.f;
    const float dv = e.d ? e.d[nc] : 1.f;
    const float bv = e.bias ? e.bias[o] : 0.f;
    const int iy0 = oy0 - pady0, ix0 = ox0 - padx0;
    const int64_t uplane = nc * (int64_t)u_h * u_w;
    float part = 0.f;
    // fixed-trip unrolled loads (u, g, noise of every element in flight at once), then the math
    const float* up = u + uplane;
    const float* gp = g + uplane;
    const float* np_ = !FROMY && e.noise ? e.noise + n * e.noise_nstride : nullptr;
    auto elem = [&](float uu, float gg, float nn, int iy, int ix) {
        if constexpr (FROMY) return smc::act_grad_y(e.act, gg, uu, e.alpha, e.gain, e.clamp) * dv;
        const float yv = smc::epi_y(uu, dv, nn * nstr, bv, e.act, e.alpha, e.gain, e.clamp);
        const float dz = smc::act_grad_y(e.act, gg, yv, e.alpha, e.gain, e.clamp);
        if (iy >= oy0 && iy < oy0 + kFH && ix >= ox0 && ix < ox0 + kFW) part += dz * uu;
        return dz * dv;
    };
    if constexpr (V2) {
        // u_w and padx0 even: the tile row splits into aligned column pairs that are in or out together
        constexpr int C2 = (COLS + 1) / 2;  // pairs per row (the last pair's second column is the pad column)
        constexpr int NL = (ROWS * C2 + 255) / 256;
        float2 uv[NL], gv[NL], nv[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int i = tid + 256 * l;
            const int r = i / C2, c2 = i - r * C2;
            const int iy = iy0 + r, ix = ix0 + 2 * c2;
            const bool ok = i < ROWS * C2 && iy >= 0 && iy < u_h && ix >= 0 && ix < u_w;
            const int pix = ok ? iy * u_w + ix : 0;
            uv[l] = *reinterpret_cast<const float2*>(up + pix);
            gv[l] = *reinterpret_cast<const float2*>(gp + pix);
            nv[l] = np_ ? *reinterpret_cast<const float2*>(np_ + pix) : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int i = tid + 256 * l;
            const int r = i / C2, c2 = i - r * C2;
            const int iy = iy0 + r, ix = ix0 + 2 * c2;
            const bool ok = i < ROWS * C2 && iy >= 0 && iy < u_h && ix >= 0 && ix < u_w;
            float2 v = make_float2(0.f, 0.f);
            if (ok) {
                v.x = elem(uv[l].x, gv[l].x, nv[l].x, iy, ix);
                v.y = elem(uv[l].y, gv[l].y, nv[l].y, iy, ix + 1);
            }
            if (i < ROWS * C2) *reinterpret_cast<float2*>(&tile[r * STRIDE + 2 * c2]) = v;
        }
    } else {
        constexpr int NL = (ROWS * COLS + 255) / 256;
        float uv[NL], gv[NL], nv[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int i = tid + 256 * l;
            const int r = i / COLS, cc = i - r * COLS;
            const int iy = iy0 + r, ix = ix0 + cc;
            const bool ok = i < ROWS * COLS && iy >= 0 && iy < u_h && ix >= 0 && ix < u_w;
            const int pix = ok ? iy * u_w + ix : 0;
            uv[l] = up[pix];
            gv[l] = gp[pix];
            nv[l] = np_ ? np_[pix] : 0.f;
        }
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int i = tid + 256 * l;
            const int r = i / COLS, cc = i - r * COLS;
            const int iy = iy0 + r, ix = ix0 + cc;
            const bool ok = i < ROWS * COLS && iy >= 0 && iy < u_h && ix >= 0 && ix < u_w;
            const float v = ok ? elem(uv[l], gv[l], nv[l], iy, ix) : 0.f;
            if (i < ROWS * COLS) tile[r * STRIDE + cc] = v;
        }
    }
    __syncthreads();
    float out[4][2];
    fir_block_split<FH, FW>(tile, STRIDE, 4 * ty, tx, tp, out);
    const int64_t tplane = nc * (int64_t)t_h * tp_w;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int oy = oy0 + 4 * ty + i;
        if (oy >= t_h) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ox = ox0 + tx + 32 * j;
            if (ox < t_w) dt[tplane + (int64_t)oy * tp_w + ox] = out[i][j];
        }
    }
    if (dd || e.dd_part) {
        const float tot = block_sum256(part, red);
        if (tid == 0) {
            if (e.dd_part) e.dd_part[nc * (gridDim.y * gridDim.z) + blockIdx.z * gridDim.y + blockIdx.y] = tot;
            else atomicAdd(dd + nc, tot);
        }
    }
}

// blur_act_bwd_fast with 16-B loads of u / g / noise (u_w % 4 == 0, 16-B aligned planes): aligned float4 groups
// covering [ox0 - 4, ox0 + kFW + 4), elements outside the tile window dropped, outside the image zeroed.
template <int FH, int FW, bool FROMY = false, bool STDF = false>
__global__ __launch_bounds__(256) void blur_act_bwd_v4(const float* g, const float* u, float* dt, float* dd, int c,
                                                       int u_h, int u_w, int t_h, int t_w, int tp_w, const float* f,
                                                       int padx0, int pady0, float fgain, int flip, Epi e) {
    constexpr int ROWS = kFH + FH - 1, COLS = kFW + FW - 1, STRIDE = COLS + 1;
    constexpr int G4 = (kFW + 8) / 4;
    constexpr int NL = (ROWS * G4 + 255) / 256;
    __shared__ __attribute__((aligned(16))) float tile[ROWS * STRIDE];
    __shared__ float red[4];
    const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;
    const int ox0 = blockIdx.y * kFW, oy0 = blockIdx.z * kFH;  // fir_grid_bwd
    const int64_t nc = blockIdx.x;
    const int n = (int)(nc / c), o = (int)(nc - (int64_t)n * c);
    float tp[FH][FW];
    if constexpr (STDF) std_taps<FH, FW>(tp);
    else load_taps<FH, FW>(f, flip, fgain, tp);
    const float nstr = e.noise_strength ? *e.noise_strength : 1.f;
    const float dv = e.d ? e.d[nc] : 1.f;
    const float bv = e.bias ? e.bias[o] : 0.f;
    const int iy0 = oy0 - pady0, ix0 = ox0 - padx0;
    const int64_t uplane = nc * (int64_t)u_h * u_w;
    const float* up = u + uplane;
    const float* gp = g + uplane;
    const float* np_ = !FROMY && e.noise ? e.noise + n * e.noise_nstride : nullptr;
    float part = 0.f;
    float4 uv[NL], gv[NL], nv[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        const int i = tid + 256 * l;
        const int r = i / G4, q = i - r * G4;
        const int iy = iy0 + r, x = ox0 - 4 + 4 * q;
        const bool ok = i < ROWS * G4 && iy >= 0 && iy < u_h && x >= 0 && x < u_w;
        const int pix = ok ? iy * u_w + x : 0;
        uv[l] = *reinterpret_cast<const float4*>(up + pix);
        gv[l] = *reinterpret_cast<const float4*>(gp + pix);
        nv[l] = np_ ? *reinterpret_cast<const float4*>(np_ + pix) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        const int i = tid + 256 * l;
        if (i >= ROWS * G4) continue;
        const int r = i / G4, q = i - r * G4;
        const int iy = iy0 + r, x = ox0 - 4 + 4 * q;
        const bool rok = iy >= 0 && iy < u_h;
        const float ua[4] = {uv[l].x, uv[l].y, uv[l].z, uv[l].w};
        const float ga[4] = {gv[l].x, gv[l].y, gv[l].z, gv[l].w};
        const float na[4] = {nv[l].x, nv[l].y, nv[l].z, nv[l].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ix = x + k;
            const int cc = ix - ix0;
            if (cc < 0 || cc >= COLS) continue;
            float val = 0.f;
            if (rok && ix >= 0 && ix < u_w) {
                if constexpr (FROMY) {
                    val = smc::act_grad_y(e.act, ga[k], ua[k], e.alpha, e.gain, e.clamp) * dv;
                } else {
                    const float yv = smc::epi_y(ua[k], dv, na[k] * nstr, bv, e.act, e.alpha, e.gain, e.clamp);
                    const float dz = smc::act_grad_y(e.act, ga[k], yv, e.alpha, e.gain, e.clamp);
                    if (iy >= oy0 && iy < oy0 + kFH && ix >= ox0 && ix < ox0 + kFW) part += dz * ua[k];
                    val = dz * dv;
                }
            }
            tile[r * STRIDE + cc] = val;
        }
    }
    __syncthreads();
    float out[4][2];
    fir_block_split<FH, FW>(tile, STRIDE, 4 * ty, tx, tp, out);
    const int64_t tplane = nc * (int64_t)t_h * tp_w;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int oy = oy0 + 4 * ty + i;
        if (oy >= t_h) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ox = ox0 + tx + 32 * j;
            if (ox < t_w) dt[tplane + (int64_t)oy * tp_w + ox] = out[i][j];
        }
    }
    if (dd || e.dd_part) {
        const float tot = block_sum256(part, red);
        if (tid == 0) {
            if (e.dd_part) e.dd_part[nc * (gridDim.y * gridDim.z) + blockIdx.z * gridDim.y + blockIdx.y] = tot;
            else atomicAdd(dd + nc, tot);
        }
    }
}

// ---------------------------------------------------------------------------------------------- demod

__global__ __launch_bounds__(256) void demod_kernel(const float* s, const float* wsq, float* d, int n, int cin,
                                                    int cout, float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per (n, o)
    if (row >= (int64_t)n * cout) return;
    const int nn = (int)(row / cout), o = (int)(row - (int64_t)nn * cout);
    const float* sp = s + (int64_t)nn * cin;
    const float* wp = wsq + (int64_t)o * cin;
    float acc = 0.f;
    for (int i = lane; i < cin; i += 64) {
        const float sv = sp[i];
        acc += sv * sv * wp[i];
    }
    acc = wave_sum(acc);
    if (lane == 0) d[row] = rsqrtf(acc + eps);
}

// ---------------------------------------------------------------------------------------------- act bwd

template <bool FROMY>
__global__ __launch_bounds__(256) void act_bwd_kernel(const float* g, const float* u, float* du, float* dd, int c,
                                                      int64_t hw, Epi e) {
    __shared__ float red[4];
    const int64_t nc = blockIdx.y;
    const int n = (int)(nc / c), o = (int)(nc - (int64_t)n * c);
    const float nstr = e.noise_strength ? *e.noise_strength : 1.f;
    const float dv = e.d ? e.d[nc] : 1.f;
    const float bv = e.bias ? e.bias[o] : 0.f;
    const int64_t base = nc * hw;
    float part = 0.f;
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < hw; p += (int64_t)gridDim.x * 256) {
        const float uv = u[base + p];
        if constexpr (FROMY) {
            du[base + p] = smc::act_grad_y(e.act, g[base + p], uv, e.alpha, e.gain, e.clamp) * dv;
            continue;
        }
        const float nz = e.noise ? e.noise[n * e.noise_nstride + p] * nstr : 0.f;
        const float yv = smc::epi_y(uv, dv, nz, bv, e.act, e.alpha, e.gain, e.clamp);
        const float dz = smc::act_grad_y(e.act, g[base + p], yv, e.alpha, e.gain, e.clamp);
        du[base + p] = dz * dv;
        part += dz * uv;
    }
    if (dd || e.dd_part) {
        const float tot = block_sum256(part, red);
        if (threadIdx.x == 0) {
            if (e.dd_part) e.dd_part[nc * gridDim.x + blockIdx.x] = tot;
            else atomicAdd(dd + nc, tot);
        }
    }
}

// dd[n, o] += the plane's per-tile partials (the act / FIR backward kernels' block sums, Epi::dd_part), one wave per
// plane in a fixed order (lane-strided sums, then a fixed butterfly): the style gradient of the demodulation is
// bit-reproducible whatever the plane size.  The fused kernels add their partials with float atomics directly only
// while a plane has at most two dd-owning tiles (two addends onto zero commute) -- every trainable layer of
// find_direction (b8..b64); larger planes (the latent mapper's high-resolution styles) take this two-level sum.
__global__ __launch_bounds__(256) void dd_sum_kernel(const float* part, int64_t tiles, float* dd, int64_t planes) {
    const int lane = threadIdx.x & 63;
    const int64_t nc = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (nc >= planes) return;
    const float* p = part + nc * tiles;
    float acc = 0.f;
    for (int64_t t = lane; t < tiles; t += 64) acc += p[t];
    acc = wave_sum(acc);
    if (lane == 0) dd[nc] += acc;
}

// float4 form (hw % 4 == 0): each thread owns AB_V float4 groups of one plane, all loads issued first.
constexpr int AB_V = 4;
template <bool FROMY>
__global__ __launch_bounds__(256) void act_bwd_vec4_kernel(const float* g, const float* u, float* du, float* dd, int c,
                                                           int64_t hw, Epi e) {
    __shared__ float red[4];
    const int64_t nc = blockIdx.y;
    const int n = (int)(nc / c), o = (int)(nc - (int64_t)n * c);
    const float nstr = e.noise_strength ? *e.noise_strength : 1.f;
    const float dv = e.d ? e.d[nc] : 1.f;
    const float bv = e.bias ? e.bias[o] : 0.f;
    const int64_t hw4 = hw >> 2;
    const float4* g4 = reinterpret_cast<const float4*>(g + nc * hw);
    const float4* u4 = reinterpret_cast<const float4*>(u + nc * hw);
    const float4* n4 = !FROMY && e.noise ? reinterpret_cast<const float4*>(e.noise + n * e.noise_nstride) : nullptr;
    float4* du4 = reinterpret_cast<float4*>(du + nc * hw);
    float part = 0.f;
    const int64_t q0 = (int64_t)blockIdx.x * 256 * AB_V + threadIdx.x;
    float4 gv[AB_V], uv[AB_V], nv[AB_V];
#pragma unroll
    for (int k = 0; k < AB_V; ++k) {
        const int64_t q = q0 + 256 * k;
        const int64_t qq = q < hw4 ? q : 0;
        gv[k] = g4[qq];
        uv[k] = u4[qq];
        nv[k] = n4 ? n4[qq] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < AB_V; ++k) {
        const int64_t q = q0 + 256 * k;
        if (q >= hw4) continue;
        const float ua[4] = {uv[k].x, uv[k].y, uv[k].z, uv[k].w};
        const float ga[4] = {gv[k].x, gv[k].y, gv[k].z, gv[k].w};
        const float na[4] = {nv[k].x, nv[k].y, nv[k].z, nv[k].w};
        float r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (FROMY) {
                r[j] = smc::act_grad_y(e.act, ga[j], ua[j], e.alpha, e.gain, e.clamp) * dv;
                continue;
            }
            const float yv = smc::epi_y(ua[j], dv, na[j] * nstr, bv, e.act, e.alpha, e.gain, e.clamp);
            const float dz = smc::act_grad_y(e.act, ga[j], yv, e.alpha, e.gain, e.clamp);
            r[j] = dz * dv;
            part += dz * ua[j];
        }
        du4[q] = make_float4(r[0], r[1], r[2], r[3]);
    }
    if (dd || e.dd_part) {
        const float tot = block_sum256(part, red);
        if (threadIdx.x == 0) {
            if (e.dd_part) e.dd_part[nc * gridDim.x + blockIdx.x] = tot;
            else atomicAdd(dd + nc, tot);
        }
    }
}

// ---------------------------------------------------------------------------------------------- channel dot

__global__ __launch_bounds__(256) void channel_dot_kernel(const float* a, const float* b, const float* scale,
                                                          float* out, float* a_scaled, int64_t len, int accumulate) {
    __shared__ float red[4];
    const int64_t r = blockIdx.x;
    const float* ap = a + r * len;
    const float* bp = b + r * len;
    const float sc = scale ? scale[r] : 1.f;
    float acc = 0.f;
    for (int64_t p = threadIdx.x; p < len; p += 256) {
        const float av = ap[p];
        acc += av * bp[p];
        if (a_scaled) a_scaled[r * len + p] = av * sc;
    }
    const float tot = block_sum256(acc, red);
    if (threadIdx.x == 0) out[r] = accumulate ? out[r] + tot : tot;
}

// 16-B form for aligned rows with len % 4 == 0: four float4 pairs in flight per thread per trip (the scalar form keeps
// one 4-B load pair in flight and reaches ~0.6 TB/s on the 128 rows x 1 M of the r = 1024 layer).
__global__ __launch_bounds__(256) void channel_dot_v4_kernel(const float4* a, const float4* b, const float* scale,
                                                             float* out, float4* a_scaled, int64_t len4,
                                                             int accumulate) {
    __shared__ float red[4];
    const int64_t r = blockIdx.x;
    const float4* ap = a + r * len4;
    const float4* bp = b + r * len4;
    float4* sp = a_scaled ? a_scaled + r * len4 : nullptr;
    const float sc = scale ? scale[r] : 1.f;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t p = threadIdx.x;
    for (; p + 768 < len4; p += 1024) {
        float4 av[4], bv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            av[k] = ap[p + 256 * k];
            bv[k] = bp[p + 256 * k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            acc[k] += av[k].x * bv[k].x + av[k].y * bv[k].y + av[k].z * bv[k].z + av[k].w * bv[k].w;
            if (sp) sp[p + 256 * k] = make_float4(av[k].x * sc, av[k].y * sc, av[k].z * sc, av[k].w * sc);
        }
    }
    for (; p < len4; p += 256) {
        const float4 av = ap[p], bv = bp[p];
        acc[0] += av.x * bv.x + av.y * bv.y + av.z * bv.z + av.w * bv.w;
        if (sp) sp[p] = make_float4(av.x * sc, av.y * sc, av.z * sc, av.w * sc);
    }
    const float tot = block_sum256((acc[0] + acc[1]) + (acc[2] + acc[3]), red);
    if (threadIdx.x == 0) out[r] = accumulate ? out[r] + tot : tot;
}

// ---------------------------------------------------------------------------------------------- demod bwd

// 32 input channels x 8 output-channel groups per workgroup; each thread sums a strided slice of o
// (coalesced 128-B rows of Wsq), then the 8 partials are reduced through LDS.
__global__ __launch_bounds__(256) void demod_bwd_kernel(const float* s, const float* d, const float* dd,
                                                        const float* wsq, float* ds, int cin, int cout) {
    __shared__ float part[8][33];
    const int nn = blockIdx.y;
    const int il = threadIdx.x & 31, og = threadIdx.x >> 5;
    const int i = blockIdx.x * 32 + il;
    const float* dp = d + (int64_t)nn * cout;
    const float* ddp = dd + (int64_t)nn * cout;
    float acc = 0.f;
    if (i < cin) {
        // unrolled: 8 rounds of independent loads in flight instead of a 64-deep dependent chain
#pragma unroll 8
        for (int o = og; o < cout; o += 8) {
            const float dv = dp[o];
            acc += ddp[o] * dv * dv * dv * wsq[(int64_t)o * cin + i];
        }
    }
    part[og][il] = acc;
    __syncthreads();
    if (og == 0 && i < cin) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) t += part[k][il];
        ds[(int64_t)nn * cin + i] += -s[(int64_t)nn * cin + i] * t;
    }
}

int64_t grid_cap(int64_t blocks) {
    const int64_t cap = (int64_t)smc::device_cu_count() * 16;
    if (blocks > cap) blocks = cap;
    return blocks < 1 ? 1 : blocks;
}

}  // namespace

SMC_API int smc_modconv_epilogue_f32(const float* src, int nsplit, int64_t split_stride, float* y, int n, int c, int h,
                                     int w, const smc_conv_epilogue* epi, void* stream) {
    SMC_CHECK(src && y && n >= 1 && c >= 1 && h >= 1 && w >= 1 && nsplit >= 1, "smc_modconv_epilogue_f32: bad args");
    const int64_t total = (int64_t)n * c * h * w;
    hipLaunchKernelGGL(epilogue_kernel, dim3((unsigned)grid_cap(smc::ceil_div(total, 256))), dim3(256), 0,
                       smc::as_stream(stream), src, nsplit, split_stride, y, c, h, w, total, to_epi(epi));
    return smc::check_launch("smc_modconv_epilogue_f32");
}

SMC_API int smc_modconv_blur_act_f32(const float* t, int nsplit, int64_t split_stride, float* y, int n, int c,
                                     int t_h, int t_w, int t_pitch, int y_h, int y_w, const float* f, int fh, int fw,
                                     int padx0, int pady0, float fgain, int flip, const smc_conv_epilogue* epi,
                                     void* stream) {
    SMC_CHECK(t && y && (f || (fh == 4 && fw == 4)) && n >= 1 && c >= 1 && nsplit >= 1,
              "smc_modconv_blur_act_f32: bad args");
    if (fh > kMaxF || fw > kMaxF || fh < 1 || fw < 1) {
        smc::set_error("smc_modconv_blur_act_f32: filter %dx%d > %dx%d", fh, fw, kMaxF, kMaxF);
        return SMC_ERR_UNSUPPORTED;
    }
    const int tp_w = t_pitch > 0 ? t_pitch : t_w;
    SMC_CHECK(tp_w >= t_w, "smc_modconv_blur_act_f32: t_pitch < t_w");
    SMC_CHECK(y_h >= 1 && y_w >= 1 && y_h <= t_h + 2 * pady0 && y_w <= t_w + 2 * padx0,
              "smc_modconv_blur_act_f32: bad output size");
    SMC_CHECK((int64_t)n * c < 65536, "smc_modconv_blur_act_f32: too many planes");
    hipStream_t st = smc::as_stream(stream);
    if (fh == 4 && fw == 4) {
        dim3 grid = fir_grid_fwd((int64_t)n * c, y_w, y_h);
        const uintptr_t al = (uintptr_t)t | (uintptr_t)y | (uintptr_t)epi->u_save | (uintptr_t)epi->noise;
        const bool v4 = split_stride % 4 == 0 && (al & 15) == 0 && y_w % 2 == 0 &&
                        epi->noise_nstride % 2 == 0 && padx0 <= 4 && fw - 1 - padx0 <= 4;
        if (v4) {
            grid.y = (unsigned)smc::ceil_div((int)grid.y, SMC_BLUR_TPB);
            if (SMC_BLUR_STDF && !f && fgain == 4.f)   // the built-in resample filter with the conv0 gain: compile-time taps
                hipLaunchKernelGGL((blur_act_v4<4, 4, SMC_BLUR_TPB, SMC_BLUR_NT != 0, true>), grid, dim3(256), 0, st, t, nsplit,
                                   split_stride, y, c, t_h, t_w, tp_w, y_h, y_w, f, padx0, pady0, fgain, flip, to_epi(epi));
            else
                hipLaunchKernelGGL((blur_act_v4<4, 4, SMC_BLUR_TPB, SMC_BLUR_NT != 0>), grid, dim3(256), 0, st, t, nsplit,
                                   split_stride, y, c, t_h, t_w, tp_w, y_h, y_w, f, padx0, pady0, fgain, flip, to_epi(epi));
        } else {
            hipLaunchKernelGGL((blur_act_fast<4, 4>), grid, dim3(256), 0, st, t, nsplit, split_stride, y, c, t_h, t_w,
                               tp_w, y_h, y_w, f, padx0, pady0, fgain, flip, to_epi(epi));
        }
        return smc::check_launch("smc_modconv_blur_act_f32");
    }
    dim3 grid((unsigned)smc::ceil_div(y_w, kBT), (unsigned)smc::ceil_div(y_h, kBT), (unsigned)(n * c));
    hipLaunchKernelGGL(blur_act_kernel, grid, dim3(256), 0, st, t, nsplit, split_stride, y, c, t_h, t_w, tp_w, y_h, y_w,
                       f, fh, fw, padx0, pady0, fgain, flip, to_epi(epi));
    return smc::check_launch("smc_modconv_blur_act_f32");
}

SMC_API int smc_modconv_demod_f32(const float* s, const float* wsq, float* d, int n, int cin, int cout, float eps,
                                  void* stream) {
    SMC_CHECK(s && wsq && d && n >= 1 && cin >= 1 && cout >= 1, "smc_modconv_demod_f32: bad args");
    const int64_t rows = (int64_t)n * cout;
    hipLaunchKernelGGL(demod_kernel, dim3((unsigned)smc::ceil_div(rows, 4)), dim3(256), 0, smc::as_stream(stream), s,
                       wsq, d, n, cin, cout, eps);
    return smc::check_launch("smc_modconv_demod_f32");
}

// dd partials of smc_modconv_act_bwd_f32: one float per (plane, workgroup) when a plane spans more than two
// workgroups (either load form), summed per plane in a fixed order by dd_sum_kernel.
static int64_t act_bwd_blocks_per_plane(int64_t hw, bool vec4) {
    return vec4 ? smc::ceil_div(hw / 4, 256 * AB_V) : std::max<int64_t>(1, smc::ceil_div(hw, 256 * 8));
}

SMC_API int64_t smc_modconv_act_bwd_workspace_size(int n, int c, int h, int w) {
    if (n < 1 || c < 1 || h < 1 || w < 1) return 0;
    const int64_t hw = (int64_t)h * w;
    const int64_t bpp = std::max(act_bwd_blocks_per_plane(hw, hw % 4 == 0), act_bwd_blocks_per_plane(hw, false));
    return bpp > 2 ? (int64_t)sizeof(float) * n * c * bpp : 0;
}

SMC_API int smc_modconv_act_bwd_f32(const float* g, const float* u, float* du, float* dd, int n, int c, int h, int w,
                                    const smc_conv_epilogue* epi, void* workspace, int64_t workspace_bytes,
                                    void* stream) {
    SMC_CHECK(g && u && du && n >= 1 && c >= 1 && h >= 1 && w >= 1, "smc_modconv_act_bwd_f32: bad args");
    SMC_CHECK(epi && epi->mode == SMC_EPI_MODACT, "smc_modconv_act_bwd_f32: needs a MODACT epilogue");
    const bool from_y = epi->grad_from_y != 0;
    SMC_CHECK(!from_y || !dd, "smc_modconv_act_bwd_f32: dd needs u (grad_from_y set)");
    const int64_t hw = (int64_t)h * w;
    const int64_t planes = (int64_t)n * c;
    SMC_CHECK(planes < 65536, "smc_modconv_act_bwd_f32: too many planes");
    const uintptr_t align = (uintptr_t)g | (uintptr_t)u | (uintptr_t)du | (uintptr_t)(from_y ? nullptr : epi->noise);
    hipStream_t st = smc::as_stream(stream);
    const bool vec4 = hw % 4 == 0 && (from_y || !epi->noise || epi->noise_nstride % 4 == 0) && align % 16 == 0;
    const int64_t blocks_per_plane = act_bwd_blocks_per_plane(hw, vec4);
    // more than two workgroups per plane: per-workgroup dd partials in the caller's workspace, summed per plane in a
    // fixed order (two addends onto zero commute, so up to two workgroups add into dd directly)
    Epi e = to_epi(epi);
    float* ddk = dd;
    const bool two_level = dd && blocks_per_plane > 2;
    if (two_level) {
        SMC_CHECK(workspace && workspace_bytes >= (int64_t)sizeof(float) * planes * blocks_per_plane,
                  "smc_modconv_act_bwd_f32: dd needs smc_modconv_act_bwd_workspace_size() bytes of workspace");
        e.dd_part = static_cast<float*>(workspace);
        ddk = nullptr;
    }
    if (vec4) {
        const dim3 grid((unsigned)blocks_per_plane, (unsigned)planes);
        if (from_y) hipLaunchKernelGGL(act_bwd_vec4_kernel<true>, grid, dim3(256), 0, st, g, u, du, ddk, c, hw, e);
        else hipLaunchKernelGGL(act_bwd_vec4_kernel<false>, grid, dim3(256), 0, st, g, u, du, ddk, c, hw, e);
    } else {
        const dim3 grid((unsigned)blocks_per_plane, (unsigned)planes);
        if (from_y) hipLaunchKernelGGL(act_bwd_kernel<true>, grid, dim3(256), 0, st, g, u, du, ddk, c, hw, e);
        else hipLaunchKernelGGL(act_bwd_kernel<false>, grid, dim3(256), 0, st, g, u, du, ddk, c, hw, e);
    }
    int rc = smc::check_launch("smc_modconv_act_bwd_f32");
    if (two_level && rc == SMC_OK) {
        hipLaunchKernelGGL(dd_sum_kernel, dim3((unsigned)smc::ceil_div(planes, 4)), dim3(256), 0, st, e.dd_part,
                           blocks_per_plane, dd, planes);
        rc = smc::check_launch("smc_modconv_act_bwd_f32 (dd)");
    }
    return rc;
}

SMC_API int smc_channel_dot_f32(const float* a, const float* b, const float* scale, float* out, float* a_scaled,
                                int64_t rows, int64_t len, int accumulate, void* stream) {
    SMC_CHECK(a && b && out && rows >= 1 && len >= 1, "smc_channel_dot_f32: bad args");
    SMC_CHECK(!a_scaled || scale, "smc_channel_dot_f32: a_scaled needs scale");
    SMC_CHECK(rows < (1LL << 31), "smc_channel_dot_f32: too many rows");
    if (len % 4 == 0 && (((uintptr_t)a | (uintptr_t)b | (uintptr_t)a_scaled) & 15) == 0) {
        hipLaunchKernelGGL(channel_dot_v4_kernel, dim3((unsigned)rows), dim3(256), 0, smc::as_stream(stream),
                           reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(b), scale, out,
                           reinterpret_cast<float4*>(a_scaled), len / 4, accumulate);
        return smc::check_launch("smc_channel_dot_f32");
    }
    hipLaunchKernelGGL(channel_dot_kernel, dim3((unsigned)rows), dim3(256), 0, smc::as_stream(stream), a, b, scale,
                       out, a_scaled, len, accumulate);
    return smc::check_launch("smc_channel_dot_f32");
}

SMC_API int smc_modconv_demod_bwd_f32(const float* s, const float* d, const float* dd, const float* wsq, float* ds,
                                      int n, int cin, int cout, void* stream) {
    SMC_CHECK(s && d && dd && wsq && ds && n >= 1 && cin >= 1 && cout >= 1, "smc_modconv_demod_bwd_f32: bad args");
    SMC_CHECK(n < 65536, "smc_modconv_demod_bwd_f32: batch too large");
    hipLaunchKernelGGL(demod_bwd_kernel, dim3((unsigned)smc::ceil_div(cin, 32), (unsigned)n), dim3(256), 0,
                       smc::as_stream(stream), s, d, dd, wsq, ds, cin, cout);
    return smc::check_launch("smc_modconv_demod_bwd_f32");
}

// dd partials of smc_modconv_blur_act_bwd_f32: one float per (plane, FIR tile) when more than two tiles of a plane own
// a part of its u window.
static int64_t blur_bwd_dd_tiles(int u_h, int u_w, int t_h, int t_w) {
    if (smc::ceil_div(u_h, kFH) * smc::ceil_div(u_w, kFW) <= 2) return 0;
    const dim3 grid = fir_grid_bwd(1, t_w, t_h);
    return (int64_t)grid.y * grid.z;
}

SMC_API int64_t smc_modconv_blur_act_bwd_workspace_size(int n, int c, int u_h, int u_w, int t_h, int t_w) {
    if (n < 1 || c < 1 || u_h < 1 || u_w < 1 || t_h < 1 || t_w < 1) return 0;
    return (int64_t)sizeof(float) * n * c * blur_bwd_dd_tiles(u_h, u_w, t_h, t_w);
}

SMC_API int smc_modconv_blur_act_bwd_f32(const float* g, const float* u, float* dt, float* dd, int n, int c, int u_h,
                                         int u_w, int t_h, int t_w, int t_pitch, const float* f, int fh, int fw,
                                         int padx0, int pady0, float fgain, int flip, const smc_conv_epilogue* epi,
                                         void* workspace, int64_t workspace_bytes, void* stream) {
    SMC_CHECK(g && u && dt && (f || (fh == 4 && fw == 4)) && n >= 1 && c >= 1 && u_h >= 1 && u_w >= 1,
              "smc_modconv_blur_act_bwd_f32: bad args");
    SMC_CHECK(epi && epi->mode == SMC_EPI_MODACT, "smc_modconv_blur_act_bwd_f32: needs a MODACT epilogue");
    SMC_CHECK(t_h == u_h + 2 * pady0 - fh + 1 && t_w == u_w + 2 * padx0 - fw + 1,
              "smc_modconv_blur_act_bwd_f32: t shape does not match the adjoint FIR");
    const int tp_w = t_pitch > 0 ? t_pitch : t_w;
    SMC_CHECK(tp_w >= t_w, "smc_modconv_blur_act_bwd_f32: t_pitch < t_w");
    SMC_CHECK((int64_t)n * c < 65536, "smc_modconv_blur_act_bwd_f32: too many planes");
    if (fh != 4 || fw != 4) {
        smc::set_error("smc_modconv_blur_act_bwd_f32: only the 4x4 FIR has a fused kernel (got %dx%d)", fh, fw);
        return SMC_ERR_UNSUPPORTED;
    }
    const bool from_y = epi->grad_from_y != 0;
    SMC_CHECK(!from_y || !dd, "smc_modconv_blur_act_bwd_f32: dd needs u (grad_from_y set)");
    hipStream_t st = smc::as_stream(stream);
    const dim3 grid = fir_grid_bwd((int64_t)n * c, t_w, t_h);
    Epi e = to_epi(epi);
    // dd-owning tiles per plane (each tile owns its 32 x 64 window of the u plane): more than two -> per-tile partials
    // in the caller's workspace, summed per plane in a fixed order after the fused kernel
    const int64_t planes = (int64_t)n * c, tiles = blur_bwd_dd_tiles(u_h, u_w, t_h, t_w);
    float* const dd_out = dd;
    const bool two_level = dd && tiles > 0;
    if (two_level) {
        SMC_CHECK(workspace && workspace_bytes >= (int64_t)sizeof(float) * planes * tiles,
                  "smc_modconv_blur_act_bwd_f32: dd needs smc_modconv_blur_act_bwd_workspace_size() bytes of workspace");
        e.dd_part = static_cast<float*>(workspace);
        dd = nullptr;
    }
    const uintptr_t al = (uintptr_t)g | (uintptr_t)u | (uintptr_t)(from_y ? nullptr : epi->noise);
    const int64_t nstr = from_y ? 0 : epi->noise_nstride;
#define SMC_BLUR_BWD(KERNEL)                                                                                       \
    hipLaunchKernelGGL(KERNEL, grid, dim3(256), 0, st, g, u, dt, dd, c, u_h, u_w, t_h, t_w, tp_w, f, padx0, pady0, \
                       fgain, flip, e)
    const bool stdf = SMC_BLUR_STDF && !f && fgain == 4.f;   // built-in [1,3,3,1] taps as constants
    if (u_w % 4 == 0 && nstr % 4 == 0 && (al & 15) == 0 && padx0 <= 4 && fw - 1 - padx0 <= 4) {
        if (from_y && stdf) SMC_BLUR_BWD((blur_act_bwd_v4<4, 4, true, true>));
        else if (from_y) SMC_BLUR_BWD((blur_act_bwd_v4<4, 4, true>));
        else if (stdf) SMC_BLUR_BWD((blur_act_bwd_v4<4, 4, false, true>));
        else SMC_BLUR_BWD((blur_act_bwd_v4<4, 4, false>));
    } else if (u_w % 2 == 0 && padx0 % 2 == 0 && nstr % 2 == 0 && ((al & 7) == 0)) {
        if (from_y) SMC_BLUR_BWD((blur_act_bwd_fast<4, 4, true, true>));
        else SMC_BLUR_BWD((blur_act_bwd_fast<4, 4, true, false>));
    } else {
        if (from_y) SMC_BLUR_BWD((blur_act_bwd_fast<4, 4, false, true>));
        else SMC_BLUR_BWD((blur_act_bwd_fast<4, 4, false, false>));
    }
#undef SMC_BLUR_BWD
    int rc = smc::check_launch("smc_modconv_blur_act_bwd_f32");
    if (two_level && rc == SMC_OK) {
        hipLaunchKernelGGL(dd_sum_kernel, dim3((unsigned)smc::ceil_div(planes, 4)), dim3(256), 0, st, e.dd_part,
                           tiles, dd_out, planes);
        rc = smc::check_launch("smc_modconv_blur_act_bwd_f32 (dd)");
    }
    return rc;
}
