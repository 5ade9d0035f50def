// upfirdn2d for gfx950: zero-insert upsample -> pad/crop -> 2-D FIR -> decimate, fp32.
//
// Replaces the reference's `_plugin.upfirdn2d` (torch_utils/ops/upfirdn2d.cpp:16-94; kernels
// upfirdn2d.cu:29-200).  HBM-bound: each 256-thread workgroup stages the input footprint of a
// (8R x 32) output tile of one plane in LDS once (coalesced row loads, zero fill outside the image),
// the taps in LDS, and every thread evaluates R outputs with the polyphase tap walk (only the taps
// that land on non-inserted samples are visited: fh/up x fw/up multiply-adds per output).
#include "common.hpp"

namespace {

constexpr int kTileW = 32;        // output columns per workgroup
constexpr int kMaxLdsIn = 9216;   // input-tile floats (36 KiB)
constexpr int kMaxTaps = 256;

struct UFDParams {
    const float* x;
    const float* f;
    float* y;
    int64_t major;
    int in_h, in_w, out_h, out_w;
    int fh, fw, upx, upy, downx, downy, padx0, pady0;
    int flip;
    float gain;
};

__device__ __forceinline__ int floor_div(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }
__device__ __forceinline__ int pos_mod(int a, int b) { int r = a % b; return r < 0 ? r + b : r; }

// UP / DN / F > 0: compile-time up (both axes), down (both axes) and square filter size -- the
// upsample2d / downsample2d shapes of the synthesis skip path and its adjoint (integer divisions become
// shifts, the tap walk unrolls, the tile load has a fixed unrolled trip count so all of a thread's loads
// are in flight together); 0 = runtime values (generic upfirdn2d).
template <int R, int UP = 0, int DN = 0, int F = 0>
__global__ __launch_bounds__(256) void ufd_tiled(UFDParams p) {
    __shared__ float tile[kMaxLdsIn];
    __shared__ float taps[kMaxTaps];
    const int upx = UP ? UP : p.upx, upy = UP ? UP : p.upy;
    const int downx = DN ? DN : p.downx, downy = DN ? DN : p.downy;
    const int fh = F ? F : p.fh, fw = F ? F : p.fw;
    const int tid = threadIdx.x;
    const int tx = tid & 31, ty = tid >> 5;
    const int ox0 = blockIdx.x * kTileW;
    const int oy0 = blockIdx.y * (8 * R);

    for (int i = tid; i < fh * fw; i += 256) {
        // store the taps in "correlation order": tap (jy, jx) multiplies upsampled sample u0 + j.
        int jy = i / fw, jx = i % fw;
        int sy = p.flip ? jy : fh - 1 - jy;
        int sx = p.flip ? jx : fw - 1 - jx;
        taps[i] = p.f[sy * fw + sx] * p.gain;
    }

    // input footprint of this output tile
    const int uy_lo = oy0 * downy - p.pady0;
    const int ux_lo = ox0 * downx - p.padx0;
    const int iy_lo = -floor_div(-uy_lo, upy);   // ceil(uy_lo / upy)
    const int ix_lo = -floor_div(-ux_lo, upx);
    const int uy_hi = (oy0 + 8 * R - 1) * downy - p.pady0 + fh - 1;
    const int ux_hi = (ox0 + kTileW - 1) * downx - p.padx0 + fw - 1;
    const int rows = floor_div(uy_hi, upy) - iy_lo + 1;
    const int cols = floor_div(ux_hi, upx) - ix_lo + 1;

    for (int64_t mj = blockIdx.z; mj < p.major; mj += gridDim.z) {
        const float* xp = p.x + mj * (int64_t)p.in_h * p.in_w;
        __syncthreads();
        if constexpr (UP > 0) {
            constexpr int MAXR = ((8 * R - 1) * (DN > 0 ? DN : 1) + F - 1) / UP + 2;
            constexpr int MAXC = ((kTileW - 1) * (DN > 0 ? DN : 1) + F - 1) / UP + 2;
            constexpr int NL = (MAXR * MAXC + 255) / 256;
            float v[NL];
#pragma unroll
            for (int l = 0; l < NL; ++l) {
                const int i = tid + 256 * l;
                const int r = i / cols, c = i - r * cols;
                const int iy = iy_lo + r, ix = ix_lo + c;
                const bool ok = i < rows * cols && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w;
                const float a = xp[ok ? (int64_t)iy * p.in_w + ix : 0];
                v[l] = ok ? a : 0.f;
            }
#pragma unroll
            for (int l = 0; l < NL; ++l)
                if (tid + 256 * l < rows * cols) tile[tid + 256 * l] = v[l];
        } else {
            for (int i = tid; i < rows * cols; i += 256) {
                int r = i / cols, c = i - r * cols;
                int iy = iy_lo + r, ix = ix_lo + c;
                float v = 0.f;
                if (iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w) v = xp[(int64_t)iy * p.in_w + ix];
                tile[i] = v;
            }
        }
        __syncthreads();
        float* yp = p.y + mj * (int64_t)p.out_h * p.out_w;
        const int ox = ox0 + tx;
        const int ux0 = ox * downx - p.padx0;
        const int jx0 = pos_mod(-ux0, upx);
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int oy = oy0 + ty + 8 * k;
            if (oy >= p.out_h || ox >= p.out_w) continue;
            const int uy0 = oy * downy - p.pady0;
            const int jy0 = pos_mod(-uy0, upy);
            float acc = 0.f;
            for (int jy = jy0; jy < fh; jy += upy) {
                const int ly = (uy0 + jy) / upy - iy_lo;
                const float* trow = tile + ly * cols - ix_lo;
                const float* frow = taps + jy * fw;
                for (int jx = jx0; jx < fw; jx += upx) acc += frow[jx] * trow[(ux0 + jx) / upx];
            }
            yp[(int64_t)oy * p.out_w + ox] = acc;
        }
    }
}

// Fallback for footprints that do not fit the LDS tile: one output per thread, direct gathers.
__global__ __launch_bounds__(256) void ufd_direct(UFDParams p) {
    const int64_t total = p.major * (int64_t)p.out_h * p.out_w;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += stride) {
        const int ox = (int)(idx % p.out_w);
        const int oy = (int)((idx / p.out_w) % p.out_h);
        const int64_t mj = idx / ((int64_t)p.out_w * p.out_h);
        const float* xp = p.x + mj * (int64_t)p.in_h * p.in_w;
        const int uy0 = oy * p.downy - p.pady0, ux0 = ox * p.downx - p.padx0;
        float acc = 0.f;
        for (int jy = pos_mod(-uy0, p.upy); jy < p.fh; jy += p.upy) {
            const int iy = (uy0 + jy) / p.upy;
            if (iy < 0 || iy >= p.in_h) continue;
            const int sy = p.flip ? jy : p.fh - 1 - jy;
            for (int jx = pos_mod(-ux0, p.upx); jx < p.fw; jx += p.upx) {
                const int ix = (ux0 + jx) / p.upx;
                if (ix < 0 || ix >= p.in_w) continue;
                const int sx = p.flip ? jx : p.fw - 1 - jx;
                acc += p.f[sy * p.fw + sx] * xp[(int64_t)iy * p.in_w + ix];
            }
        }
        p.y[idx] = acc * p.gain;
    }
}

int tile_cols(const UFDParams& p) { return ((kTileW - 1) * p.downx + p.fw - 1) / p.upx + 2; }
int tile_rows(const UFDParams& p, int R) { return ((8 * R - 1) * p.downy + p.fh - 1) / p.upy + 2; }

}  // namespace

SMC_API int smc_upfirdn2d_f32(const float* x, const float* f, float* y, int64_t major, int in_h, int in_w,
                              int out_h, int out_w, int fh, int fw, int upx, int upy, int downx, int downy,
                              int padx0, int padx1, int pady0, int pady1, int flip, float gain, void* stream) {
    SMC_CHECK(major >= 0 && in_h >= 1 && in_w >= 1, "smc_upfirdn2d_f32: bad input shape");
    SMC_CHECK(fh >= 1 && fw >= 1, "smc_upfirdn2d_f32: bad filter shape");
    SMC_CHECK(upx >= 1 && upy >= 1 && downx >= 1 && downy >= 1, "smc_upfirdn2d_f32: bad up/down");
    const int eh = (in_h * upy + pady0 + pady1 - fh + downy) / downy;
    const int ew = (in_w * upx + padx0 + padx1 - fw + downx) / downx;
    SMC_CHECK(eh >= 1 && ew >= 1, "smc_upfirdn2d_f32: output would be empty");
    SMC_CHECK(out_h == eh && out_w == ew, "smc_upfirdn2d_f32: out shape %dx%d != expected %dx%d", out_h, out_w, eh,
              ew);
    if (major == 0) return SMC_OK;
    UFDParams p{x, f, y, major, in_h, in_w, out_h, out_w, fh, fw, upx, upy, downx, downy, padx0, pady0, flip, gain};
    hipStream_t st = smc::as_stream(stream);
    int R = 0;
    if (fh * fw <= kMaxTaps) {
        for (int r : {4, 2, 1}) {
            if (tile_rows(p, r) * tile_cols(p) <= kMaxLdsIn) { R = r; break; }
        }
    }
    if (R > 0) {
        // keep enough workgroups in flight for 256 CUs; planes beyond grid.z are looped in-kernel
        const int gx = (int)smc::ceil_div(out_w, kTileW);
        const int gy = (int)smc::ceil_div(out_h, 8 * R);
        int64_t gz = major < 65535 ? major : 65535;
        dim3 grid(gx, gy, (unsigned)gz);
        const bool sq = upx == upy && downx == downy && fh == 4 && fw == 4;
        if (R == 4 && sq && upx == 2 && downx == 1) hipLaunchKernelGGL((ufd_tiled<4, 2, 1, 4>), grid, dim3(256), 0, st, p);
        else if (R == 4 && sq && upx == 1 && downx == 2) hipLaunchKernelGGL((ufd_tiled<4, 1, 2, 4>), grid, dim3(256), 0, st, p);
        else if (R == 4) hipLaunchKernelGGL(ufd_tiled<4>, grid, dim3(256), 0, st, p);
        else if (R == 2) hipLaunchKernelGGL(ufd_tiled<2>, grid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL(ufd_tiled<1>, grid, dim3(256), 0, st, p);
    } else {
        int64_t total = major * (int64_t)out_h * out_w;
        int64_t blocks = smc::ceil_div(total, 256);
        const int64_t cap = (int64_t)smc::device_cu_count() * 16;
        if (blocks > cap) blocks = cap;
        hipLaunchKernelGGL(ufd_direct, dim3((unsigned)blocks), dim3(256), 0, st, p);
    }
    return smc::check_launch("smc_upfirdn2d_f32");
}
