// Winograd F(4x4, 3x3) convolution on fp32 MFMA for gfx950 (v_mfma_f32_16x16x4_f32).
//
// The same 3x3 stride-1 'same' convolutions as wino.hip (SynthesisLayer conv1 forward and data gradient,
// conv2d_resample.py:147-154), with 4x4 output tiles: each tile comes from a 6x6 input patch with 36 multiplies per
// (input, output) channel pair instead of 144 (4x fewer MFMA FLOPs; F(2x2) saves 2.25x):
//     V = B^T d B   (6x6)        U = G g G^T   (6x6, frozen: smc_wino4_weights_f32, computed in fp64)
//     M[xi] = sum_c U[xi][c][o] * V[xi][c][t]      (36 independent GEMMs on the matrix core)
//     Y = A^T M A   (4x4)
// with the interpolation points 0, 1, -1, 2, -2 (Lavin & Gray):
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   G   = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
// Index xi = 6 b + a for the element (row a, column b) of the 6x6 transform domain.
//
// Work decomposition (one 768-thread workgroup per CU, roles below the W4Cfg definition):
//   * a work item is 64 output channels x 32 tiles (2 tile rows x 16 tile columns = 8 x 64 outputs of one image);
//     each of the 8 MFMA waves owns 16 channels x 16 tiles, all 36 xi = 36 accumulators of the 16x16x4 MFMA (144
//     registers).  A lane holds one tile and 4 channels of each, so the 36 M values of a (channel, tile) sit in one
//     lane and the output transform + modconv epilogue are lane-local.
//   * K steps of 4 input channels (the MFMA's k).  V is computed ONCE per workgroup by two transform waves and shared
//     through LDS by the 4 channel groups; two DMA waves stage the operands (buffer_load ... lds): the U slab
//     [4][9][64][4] one step ahead, the raw input rows of the block's 10 x 72 patch two steps ahead (16-B chunks from
//     column 4 tx0 - 4; the buffer range check zero-fills the image border).  LDS: 2 x (U + patch + V) = 132 KiB;
//     one barrier per step.
#include <algorithm>
#include <type_traits>

#include "common.hpp"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int W4K = 4;       // input channels per K step (= the MFMA's k)
constexpr int NXQ = 9;       // xi quads (36 / 4)
constexpr int PCH = 18;      // 16-B chunks per staged patch row
constexpr int PPITCH = 72;   // floats per staged patch row (columns 4 tx0 - 4 .. 4 tx0 + 67)
constexpr int SENTINEL = 0x7ffffff0;

struct Wino4Params {
    const float* x;
    int n, cin, h, w;
    float* y;
    int cout;
    const float* uw;  // [cin][9][cout][4]
    const float* s;   // [n][cin] or NULL
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
    int gx, gy;  // tile blocks per image along x / y
    int ntn;     // output-channel blocks (cout / 64)
};

template <int CG, int TG>
struct W4Cfg {
    static_assert(CG * TG == 8, "8 waves");
    static constexpr int OB = 16 * CG;                 // output channels per work item
    static constexpr int TB = 16 * TG;                 // tiles per work item
    static constexpr int ROWS = 4 * TG + 2;            // staged input rows
    static constexpr int SLAB = ROWS * PPITCH;         // patch floats per channel
    static constexpr int UJ = W4K * NXQ * OB / 64;     // U DMA wave-instructions per step (16 B per lane)
    static constexpr int PL = W4K * ROWS * PCH;        // patch DMA lanes per step
    static constexpr int PJ = (PL + 63) / 64;
    static constexpr int UF = UJ * 256;                // floats
    static constexpr int PF = PJ * 256;                // floats (whole instructions)
    static constexpr int VF = W4K * NXQ * TB * 4;      // floats
    static constexpr int STAGE = UF + PF + VF;
    static constexpr int UJW = (UJ + 7) / 8;
    static constexpr int PJW = (PJ + 7) / 8;
    static_assert(W4K * TB == 64 * TG, "one patch per lane of TG waves");
};

template <int N>
__device__ __forceinline__ void w4_wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// six-point input transform y = B^T x (14 VALU)
__device__ __forceinline__ void bt6(const float (&x)[6], float (&y)[6]) {
    y[0] = __fmaf_rn(4.f, x[0], __fmaf_rn(-5.f, x[2], x[4]));
    const float p = x[1] + x[2], q = x[3] + x[4];
    y[1] = __fmaf_rn(-4.f, p, q);
    const float r = x[1] - x[2], s = x[4] - x[3];
    y[2] = __fmaf_rn(4.f, r, s);
    const float u = x[3] - x[1], w = x[4] - x[2];
    y[3] = __fmaf_rn(2.f, u, w);
    y[4] = __fmaf_rn(-2.f, u, w);
    y[5] = __fmaf_rn(4.f, x[1], __fmaf_rn(-5.f, x[3], x[5]));
}

// six-point output transform z = A^T m (4 outputs)
__device__ __forceinline__ void at6(const float (&m)[6], float (&z)[4]) {
    const float s12 = m[1] + m[2], d12 = m[1] - m[2], s34 = m[3] + m[4], d34 = m[3] - m[4];
    z[0] = m[0] + s12 + s34;
    z[1] = __fmaf_rn(2.f, d34, d12);
    z[2] = __fmaf_rn(4.f, s34, s12);
    z[3] = __fmaf_rn(8.f, d34, d12) + m[5];
}

struct W4Item {
    int nn, ty0, tx0, o0;
};

// Wave roles (12 waves = 768 threads, 3 per SIMD, one workgroup per CU; the roles run concurrently, one s_barrier
// per K step for all of them):
//   waves 0-7   consumers: only MFMAs (A fragments from the U slot, B fragments from the V slot of step k) and, after
//               the K loop, the output transform + epilogue.  Wave w owns channel group w % 4 and tile row w / 4.
//   waves 8-9   transform: V(k + 1) from the patch of step k + 1 (64 patches each: 18 LDS reads, 2 x 6 six-point
//               transforms, x s[n, c], 9 ds_write_b128).
//   waves 10-11 DMA: U(k + 1) and the patch of step k + 2 into their LDS slots (24 LDS-DMAs each), then their wait.
// Measured (tools/probes/wino4_probe.hip, r = 64, profiles/r03_wino4/): with the transform and the DMAs issued by the
// MFMA waves themselves a launch took 338 us (196 without the transform, 250 without the DMAs) -- a wave that
// serialises LDS reads, VALU and DMA issue between its own MFMAs starves the matrix pipe of its SIMD; with these
// roles 232 us (178 without the transform).  Four producer waves (one per SIMD, two lanes per patch with a DPP swap
// between the row and column pass, a quarter of the DMAs each) measured 243 us: VALU on every SIMD's issue port.
// SM: style scale s[n, c] (1: present, 2: absent).  EK: epilogue body (1: MODACT lrelu + gain + clamp, 2: MODACT
// linear, 0: any mode through smc::epi_y / epi_ext_apply).  PROBE (0 in the library; tools/probes/wino4_probe.hip)
// removes pieces for timing: 1 the U DMAs after step 0, 2 the patch DMAs after step 1, 4 the transform after step 0.
constexpr int W4_THREADS = 768;
#ifndef W4_TPRIO
#define W4_TPRIO 2
#endif

template <int SM, int EK, int PROBE = 0>
__global__ __launch_bounds__(W4_THREADS) __attribute__((amdgpu_waves_per_eu(3, 3)))
void wino4_kernel(Wino4Params p) {
    using C = W4Cfg<4, 2>;
    constexpr int OB = C::OB, TB = C::TB, SLAB = C::SLAB, STAGE = C::STAGE, ROWS = C::ROWS;
    constexpr int UJ = C::UJ, PJ = C::PJ;
    // + the MODACT epilogue operands of the work item, staged once by the DMA waves: the noise block (8 rows x
    // 64 columns, x strength) and per output channel d * scale_c and the bias (read by the consumers' epilogue from
    // LDS, so its loads neither stall behind its own stores nor hold registers across the output transform)
    constexpr int EPI_F = 8 * 64 + 2 * 64;
    __shared__ __attribute__((aligned(16))) float smem[2 * STAGE + EPI_F];
    float* epi_s = smem + 2 * STAGE;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = p.h, W = p.w;
    const int64_t plane = (int64_t)H * W;
    const int nsteps = p.cin / W4K;
    const int total = p.n * p.gx * p.gy * p.ntn;

    const int v = blockIdx.x;
    if (v >= total) return;
    // work item -> (image, tile block, output-channel block) in the XCD-aware bijective order of wino.hip
    // (output-channel blocks fastest: the workgroups that stage the same input patch share an L2)
    W4Item it;
    {
        const int xcd = v % 8, q8 = total / 8, r8 = total % 8;
        const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + v / 8;
        const int ob = id % p.ntn, tgi = id / p.ntn;
        const int per_img = p.gx * p.gy;
        it.nn = tgi / per_img;
        const int rem = tgi - it.nn * per_img;
        it.ty0 = (rem / p.gx) * 2;
        it.tx0 = (rem % p.gx) * 16;
        it.o0 = ob * OB;
    }

    if (wave >= 10) {
        // ---- DMA waves: U instructions j = d, d + 2, ... (run j of the slab: 64 output channels x 16 B), patch
        // instructions jj = d, d + 2, ... (16-B lane L = (c * ROWS + r) * PCH + ch)
        constexpr int UPW = UJ / 2, PPW = (PJ + 1) / 2;
        const int d = wave - 10;
        const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
            (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * plane * 4), 0x00020000);
        const __amdgpu_buffer_rsrc_t ursrc =
            __builtin_amdgcn_make_buffer_rsrc((void*)p.uw, (short)0, p.cin * 36 * p.cout * 4, 0x00020000);
        const int uv0 = (it.o0 + lane) * 16;
        int pv[PPW];
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int L = (d + 2 * i) * 64 + lane;
            const int c = L / (ROWS * PCH);
            const int r2 = L - c * (ROWS * PCH);
            const int r = r2 / PCH, ch = r2 - r * PCH;
            const int gyy = 4 * it.ty0 - 1 + r, gxx = 4 * it.tx0 - 4 + 4 * ch;
            const bool ok = c < W4K && gyy >= 0 && gyy < H && gxx >= 0 && gxx < W;
            pv[i] = ok ? (int)((((int64_t)(it.nn * p.cin + c) * H + gyy) * W + gxx) * 4) : SENTINEL;
        }
        const int ustep = NXQ * W4K * p.cout * 16;
        const int urun = p.cout * 16;
        const int pstep = W4K * (int)plane * 4;
        auto issue_u = [&](int ks, int slot) {
            if constexpr ((PROBE & 1) != 0)
                if (ks > 0) return;
            float* us = smem + slot * STAGE;
#pragma unroll
            for (int i = 0; i < UPW; ++i) {
                const int j = d + 2 * i;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    ursrc, (__attribute__((address_space(3))) void*)(us + j * 256), 16, uv0, ks * ustep + j * urun, 0, 0);
            }
        };
        auto issue_p = [&](int ks, int slot) {
            if constexpr ((PROBE & 2) != 0)
                if (ks > 1) return;
            float* ps = smem + slot * STAGE + C::UF;
#pragma unroll
            for (int i = 0; i < PPW; ++i) {
                const int jj = d + 2 * i;
                if (jj < PJ) {
                    const int vo = pv[i];
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        xrsrc, (__attribute__((address_space(3))) void*)(ps + jj * 256), 16, vo, ks * pstep, 0, 0);
                }
            }
        };
        issue_u(0, 0);
        issue_p(0, 0);
        if (nsteps > 1) issue_p(1, 1);
        if (p.mode == SMC_EPI_MODACT) {
            const int pt = d * 64 + lane;  // 128 lanes: noise floats 4 pt .. 4 pt + 3; channel pt < 64
            const int yy = 4 * it.ty0 + (4 * pt) / 64, xx = 4 * it.tx0 + (4 * pt) % 64;
            const float nstr = p.noise ? (p.noise_strength ? *p.noise_strength : 1.f) : 0.f;
            const f32x4 nz = p.noise ? *reinterpret_cast<const f32x4*>(p.noise + it.nn * p.noise_nstride +
                                                                        (int64_t)yy * W + xx)
                                     : f32x4{0.f, 0.f, 0.f, 0.f};
            float dv = 0.f, bv = 0.f;
            if (pt < 64) {
                const int o = it.o0 + pt;
                dv = (p.d ? p.d[(int64_t)it.nn * p.cout + o] : 1.f) * (p.ext.scale_c ? p.ext.scale_c[o] : 1.f);
                bv = p.bias ? p.bias[o] : 0.f;
            }
            *reinterpret_cast<f32x4*>(epi_s + 4 * pt) = nz * nstr;
            if (pt < 64) {
                epi_s[512 + pt] = dv;
                epi_s[576 + pt] = bv;
            }
        }
        w4_wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        for (int ks = 0; ks < nsteps; ++ks) {
            __builtin_amdgcn_s_barrier();  // step ks: its U slot and the patch of ks + 1 have landed everywhere
            asm volatile("" ::: "memory");
            if (ks + 1 < nsteps) issue_u(ks + 1, (ks + 1) & 1);
            if (ks + 2 < nsteps) issue_p(ks + 2, ks & 1);
            w4_wait_vmcnt<0>();
        }
        return;
    }

    if (wave >= 8) {
        // ---- transform waves: lane -> patch pi = (wave - 8) 64 + lane = (channel, tile) of the step
        const int pi = (wave - 8) * 64 + lane;
        const int tc_ch = pi / TB, tc_t = pi - tc_ch * TB;
        const int p_off = tc_ch * SLAB + 4 * (tc_t / 16) * PPITCH + 4 * (tc_t % 16) + 3;
        const int v_off = (tc_ch * NXQ * TB + tc_t) * 4;
        const float* srow = SM == 1 ? p.s + (int64_t)it.nn * p.cin + tc_ch : nullptr;
        // the transform is the step's long pole: its VALU goes ahead of the consumers' (their MFMAs queue on the
        // matrix pipe anyway) -- issue arbitration is by priority, then age, and these waves are the youngest
        __builtin_amdgcn_s_setprio(W4_TPRIO);
        auto transform = [&](int slot, float sc) {
            const float* pp = smem + slot * STAGE + C::UF + p_off;
            float d[6][6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                d[i][0] = pp[i * PPITCH];
                const f32x4 m = *reinterpret_cast<const f32x4*>(pp + i * PPITCH + 1);
                d[i][1] = m[0]; d[i][2] = m[1]; d[i][3] = m[2]; d[i][4] = m[3];
                d[i][5] = pp[i * PPITCH + 5];
            }
            float rt[6][6];  // rt[i][b] = (d B)[i][b]
#pragma unroll
            for (int i = 0; i < 6; ++i) bt6(d[i], rt[i]);
            float* vs = smem + slot * STAGE + C::UF + C::PF + v_off;
            float vv[36];   // xi = 6 b + a
#pragma unroll
            for (int b = 0; b < 6; ++b) {
                float x[6], y[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) x[i] = rt[i][b];
                bt6(x, y);
#pragma unroll
                for (int a = 0; a < 6; ++a) vv[6 * b + a] = SM == 1 ? y[a] * sc : y[a];
            }
#pragma unroll
            for (int q = 0; q < NXQ; ++q)
                *reinterpret_cast<f32x4*>(vs + q * TB * 4) = f32x4{vv[4 * q], vv[4 * q + 1], vv[4 * q + 2], vv[4 * q + 3]};
        };
        // style scale for V(k + 1) loaded during step k - 1
        float s_nx = SM == 1 && nsteps > 1 ? srow[W4K] : 1.f;
        const float s0 = SM == 1 ? srow[0] : 1.f;
        __builtin_amdgcn_s_barrier();
        transform(0, s0);
        for (int ks = 0; ks < nsteps; ++ks) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // V(ks) visible; the V slot of ks - 1 is free
            asm volatile("" ::: "memory");
            if (ks + 1 < nsteps && ((PROBE & 4) == 0 || ks == 0)) {
                const float sc = s_nx;
                if (SM == 1 && ks + 2 < nsteps) s_nx = srow[(ks + 2) * W4K];
                transform((ks + 1) & 1, sc);
            }
        }
        return;
    }

    // ---- consumer waves
    const int cg = wave & 3, tg = wave >> 2;
    const int kq_lane = lane >> 4;
    const int fa_off = (kq_lane * NXQ * OB + 16 * cg + (lane & 15)) * 4;   // A fragment (xq 0) in a U slot
    const int fb_off = (kq_lane * NXQ * TB + 16 * tg + (lane & 15)) * 4;   // B fragment (xq 0) in a V slot
    f32x4 acc[36];
#pragma unroll
    for (int xi = 0; xi < 36; ++xi) acc[xi] = f32x4{0.f, 0.f, 0.f, 0.f};
    __builtin_amdgcn_s_barrier();
    for (int ks = 0; ks < nsteps; ++ks) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of step ks - 1 are done
        __builtin_amdgcn_s_barrier();  // U(ks), V(ks) in LDS
        asm volatile("" ::: "memory");
        const int sl = ks & 1;
        const float* us = smem + sl * STAGE + fa_off;
        const float* vs = smem + sl * STAGE + C::UF + C::PF + fb_off;
        f32x4 fa[2], fb[2];
        fa[0] = *reinterpret_cast<const f32x4*>(us);
        fb[0] = *reinterpret_cast<const f32x4*>(vs);
#pragma unroll
        for (int xq = 0; xq < NXQ; ++xq) {
            if (xq + 1 < NXQ) {
                fa[(xq + 1) & 1] = *reinterpret_cast<const f32x4*>(us + (xq + 1) * OB * 4);
                fb[(xq + 1) & 1] = *reinterpret_cast<const f32x4*>(vs + (xq + 1) * TB * 4);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[4 * xq + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[xq & 1][j], fb[xq & 1][j], acc[4 * xq + j], 0, 0, 0);
        }
    }

    // ---- epilogue: Y = A^T M A per (channel, tile), then the conv epilogue
    const int nn = it.nn;
    const int yy0 = 4 * (it.ty0 + tg), xx0 = 4 * (it.tx0 + (lane & 15));
    const bool modact = p.mode == SMC_EPI_MODACT;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int o = it.o0 + 16 * cg + 4 * kq_lane + r;
        float zc[4][6];  // A^T M: zc[p][b]
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            float m[6], z[4];
#pragma unroll
            for (int a = 0; a < 6; ++a) m[a] = acc[6 * b + a][r];
            at6(m, z);
#pragma unroll
            for (int q = 0; q < 4; ++q) zc[q][b] = z[q];
        }
        const int64_t obase = ((int64_t)nn * p.cout + o) * plane;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float out[4];
            at6(zc[i], out);
            const int64_t idx = obase + (int64_t)(yy0 + i) * W + xx0;
            float q[4];
            if (EK != 0 || modact) {
                if (p.u_save) *reinterpret_cast<f32x4*>(p.u_save + idx) = f32x4{out[0], out[1], out[2], out[3]};
                const int ol = 16 * cg + 4 * kq_lane + r;
                const float dsc = epi_s[512 + ol], bo = epi_s[576 + ol];
                const f32x4 nq = *reinterpret_cast<const f32x4*>(epi_s + (4 * tg + i) * 64 + 4 * (lane & 15));
                const float nz[4] = {nq[0], nq[1], nq[2], nq[3]};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if constexpr (EK == 1) {
                        const float z = __fmaf_rn(out[j], dsc, nz[j]) + bo;
                        q[j] = smc::lrelu_gain_clamp(z, p.alpha, p.gain, p.clamp);
                    } else if constexpr (EK == 2) {
                        q[j] = (__fmaf_rn(out[j], dsc, nz[j]) + bo) * p.gain;
                    } else {
                        q[j] = smc::epi_y(out[j], dsc, nz[j], bo, p.act, p.alpha, p.gain, p.clamp);
                        if (p.ext.residual)
                            q[j] = smc::epi_ext_apply(SMC_EPI_STORE, q[j], nn, o, idx + j, yy0 + i, xx0 + j, p.cout, H,
                                                      W, nullptr, nullptr, p.ext);
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    q[j] = smc::epi_ext_apply(p.mode, out[j], nn, o, idx + j, yy0 + i, xx0 + j, p.cout, H, W, p.bias,
                                              p.u_save, p.ext);
            }
            *reinterpret_cast<f32x4*>(p.y + idx) = f32x4{q[0], q[1], q[2], q[3]};
        }
    }
}

// U = G g G^T per (k, n) in fp64, rounded once: flip = 0: g = w[n][k] (k = cin, n = cout: the forward
// correlation); flip = 1: g = w[k][n] rotated by 180 degrees (k = cout, n = cin: the data gradient).
// Out: [K][9][N][4], element xi = 6 b + a of the 6x6 U at [k][xi / 4][n][xi % 4].
__global__ __launch_bounds__(256) void wino4_weights_kernel(const float* w, int cout, int cin, int flip, float* uw) {
    const int K = flip ? cout : cin, N = flip ? cin : cout;
    const int64_t total = (int64_t)K * N;
    const double Gm[6][3] = {{0.25, 0., 0.},
                             {-1. / 6., -1. / 6., -1. / 6.},
                             {-1. / 6., 1. / 6., -1. / 6.},
                             {1. / 24., 1. / 12., 1. / 6.},
                             {1. / 24., -1. / 12., 1. / 6.},
                             {0., 0., 1.}};
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(e / N), nidx = (int)(e - (int64_t)k * N);
        double g[3][3];
        const float* src = flip ? w + ((int64_t)k * cin + nidx) * 9 : w + ((int64_t)nidx * cin + k) * 9;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) g[i][j] = flip ? src[(2 - i) * 3 + (2 - j)] : src[i * 3 + j];
        double gg[6][3];  // G g
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int j = 0; j < 3; ++j) gg[a][j] = Gm[a][0] * g[0][j] + Gm[a][1] * g[1][j] + Gm[a][2] * g[2][j];
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int b = 0; b < 6; ++b) {
                const double u = gg[a][0] * Gm[b][0] + gg[a][1] * Gm[b][1] + gg[a][2] * Gm[b][2];
                const int xi = 6 * b + a;
                uw[(((int64_t)k * NXQ + (xi >> 2)) * N + nidx) * 4 + (xi & 3)] = (float)u;
            }
    }
}

template <int SM, int EK>
void launch_w4(const Wino4Params& p, int64_t items, hipStream_t st) {
    hipLaunchKernelGGL((wino4_kernel<SM, EK>), dim3((unsigned)items), dim3(W4_THREADS), 0, st, p);
}

template <int EK>
void launch_w4_s(bool has_s, const Wino4Params& p, int64_t items, hipStream_t st) {
    if (has_s) launch_w4<1, EK>(p, items, st);
    else launch_w4<2, EK>(p, items, st);
}

// work item = 64 output channels x 32 tiles (2 tile rows x 16 tile columns = 8 x 64 outputs)
bool w4_shape_ok(int cout, int h, int w) { return w % 64 == 0 && w >= 64 && h % 8 == 0 && cout % 64 == 0; }

}  // namespace

SMC_API int smc_conv3x3_wino4_supported(int n, int cin, int cout, int h, int w) {
    if (n < 1 || cin < W4K || cin % W4K) return 0;
    if ((int64_t)n * cin * h * w * 4 >= (1LL << 31)) return 0;  // raw buffer offsets are 32-bit
    if ((int64_t)cin * 36 * cout * 4 >= (1LL << 31)) return 0;
    return w4_shape_ok(cout, h, w);
}

SMC_API int smc_wino4_weights_f32(const float* w, int cout, int cin, int flip, float* uw, void* stream) {
    SMC_CHECK(w && uw && cout >= 1 && cin >= 1, "smc_wino4_weights_f32: bad arguments");
    SMC_CHECK((reinterpret_cast<uintptr_t>(uw) & 15) == 0, "smc_wino4_weights_f32: uw must be 16-B aligned");
    const int64_t total = (int64_t)cout * cin;
    hipLaunchKernelGGL(wino4_weights_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(total, 256), 4096)),
                       dim3(256), 0, smc::as_stream(stream), w, cout, cin, flip, uw);
    return smc::check_launch("smc_wino4_weights_f32");
}

SMC_API int smc_conv3x3_wino4_f32(const float* x, int n, int cin, int h, int w, float* y, int cout, const float* uw,
                                  const float* s_in, const smc_conv_epilogue* epi, void* stream) {
    SMC_CHECK(x && y && uw, "smc_conv3x3_wino4_f32: null pointer");
    if (!smc_conv3x3_wino4_supported(n, cin, cout, h, w)) {
        smc::set_error("smc_conv3x3_wino4_f32: no Winograd F(4x4) kernel for n=%d cin=%d cout=%d %dx%d", n, cin, cout,
                       h, w);
        return SMC_ERR_UNSUPPORTED;
    }
    SMC_CHECK((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(uw) & 15) == 0,
              "smc_conv3x3_wino4_f32: x / y / uw must be 16-B aligned");
    smc_conv_epilogue e{};
    e.mode = SMC_EPI_STORE; e.act = SMC_ACT_LINEAR; e.gain = 1.f; e.clamp = -1.f;
    if (epi) e = *epi;
    SMC_CHECK(e.mode >= SMC_EPI_STORE && e.mode <= SMC_EPI_AFFINE, "smc_conv3x3_wino4_f32: bad epilogue mode %d", e.mode);
    SMC_CHECK((e.mode != SMC_EPI_PRELU && e.mode != SMC_EPI_PRELU_GRAD) || e.alpha_c,
              "smc_conv3x3_wino4_f32: PReLU epilogue needs alpha_c");
    SMC_CHECK(e.mode != SMC_EPI_PRELU_GRAD || e.act_ref, "smc_conv3x3_wino4_f32: PRELU_GRAD needs act_ref");
    SMC_CHECK(!e.u_save || (reinterpret_cast<uintptr_t>(e.u_save) & 15) == 0, "smc_conv3x3_wino4_f32: u_save alignment");
    SMC_CHECK(!e.noise || ((reinterpret_cast<uintptr_t>(e.noise) & 15) == 0 && e.noise_nstride % 4 == 0),
              "smc_conv3x3_wino4_f32: noise must be 16-B aligned");
    Wino4Params p{};
    p.x = x; p.n = n; p.cin = cin; p.h = h; p.w = w; p.y = y; p.cout = cout; p.uw = uw; p.s = s_in;
    p.mode = e.mode; p.d = e.d; p.noise = e.noise; p.noise_nstride = e.noise_nstride;
    p.noise_strength = e.noise_strength; p.bias = e.bias; p.act = e.act; p.alpha = e.alpha; p.gain = e.gain;
    p.clamp = e.clamp; p.u_save = e.u_save;
    p.ext = smc::epi_ext(epi);
    p.gx = w / 64;
    p.gy = h / 8;
    p.ntn = cout / 64;
    const int64_t items = (int64_t)n * p.gx * p.gy * p.ntn;
    SMC_CHECK(items < (1LL << 31), "smc_conv3x3_wino4_f32: grid too large");
    hipStream_t st = smc::as_stream(stream);
    const bool modact_plain = p.mode == SMC_EPI_MODACT && !p.ext.residual;
    if (modact_plain && p.act == SMC_ACT_LRELU && p.alpha >= 0.f && p.alpha <= 1.f && p.clamp >= 0.f)
        launch_w4_s<1>(s_in != nullptr, p, items, st);
    else if (modact_plain && p.act == SMC_ACT_LINEAR && p.clamp < 0.f)
        launch_w4_s<2>(s_in != nullptr, p, items, st);
    else
        launch_w4_s<0>(s_in != nullptr, p, items, st);
    return smc::check_launch("smc_conv3x3_wino4_f32");
}
