// Winograd F(2x2, 3x3) convolution on fp32 MFMA for gfx950 (v_mfma_f32_16x16x4_f32).
//
// The 3x3 stride-1 'same' convolutions of the synthesis (every SynthesisLayer conv1 forward and its data
// gradient, conv2d_resample.py:147-154 with groups = batch in the reference) are the largest GEMM family
// of a find_direction step.  F(2x2, 3x3) computes each 2x2 output tile from a 4x4 input patch with 16
// multiplies per (input, output) channel pair instead of 36 (2.25x fewer MFMA FLOPs):
//     V = B^T d B   (input patch d, 4x4)          U = G g G^T   (3x3 taps g, frozen: smc_wino_weights_f32)
//     M[xi] = sum_c U[xi][c][o] * V[xi][c][t]      (16 independent GEMMs, xi = 4a + b, on the matrix core)
//     Y = A^T M A   (2x2 outputs)
// B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1], A^T = [1 1 1 0; 0 1 -1 -1].
// Everything stays fp32 (transforms on the VALU, products and sums on the f32-input MFMA); the transforms
// add a few ulps next to the direct conv (tests/test_gpu_wino.py states the tolerance against fp64).
//
// Work decomposition (256 threads = 4 waves, 2 workgroups per CU):
//   * a workgroup owns 32 output channels x 64 tiles (a TR x TC block of one image, TC = min(64, W/2)),
//     each wave 32 channels x 16 tiles, all 16 xi: 16 x 2 accumulators of the 16x16x4 MFMA (128 registers).
//     In the MFMA C layout a lane holds column j = tile and rows i = channels, so the 16 M values of one
//     (channel, tile) sit in ONE lane (the same register of the 16 xi accumulators): the output transform
//     and the modconv epilogue are lane-local.
//   * K steps of 8 input channels; per step both operands go global -> LDS by DMA into a 2-stage ring (one
//     barrier per step): the raw input rows of the block's (2TR+2) x (2TC+2) patch, staged from column
//     2*tx0 - 4 as 16-B chunks (the buffer range check zero-fills the image border), and the U slab
//     [8][4][32][4] (channel, xi group, out channel, xi % 4) by global_load_lds_dwordx4.
//   * per k-quad (4 channels: MFMA k = lane >> 4) every lane reads ITS tile's 4x4 patch of ITS channel from
//     LDS, transforms it in registers (32 adds; x s[n, c] for the style-scaled forward) and that is its B
//     fragment for all 16 xi -- V never goes through LDS.  A fragments: 8 ds_read_b128 (bank-conflict free).
#include <algorithm>
#include <type_traits>

#include "common.hpp"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int WBK = 8;    // input channels per K step
constexpr int WBO = 32;   // output channels per workgroup
constexpr int WBT = 64;   // tiles per workgroup (4 waves x 16)
constexpr int WOBW = 2;   // the library's waves-per-workgroup variant (wino_kernel OBW)

struct WinoParams {
    const float* x;
    int n, cin, h, w;
    float* y;
    int cout;
    const float* uw;  // [cin][4][cout][4]
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
    int gx, gy;  // tile groups per image along x / y
    int ntn;     // output-channel blocks (cout / 32)
};

// RD selects how a lane reads its 4x4 patch from LDS.  0: 16 ds_read_b32 from the lane-linear DMA image (the 4
// channels a half-wave reads sit SLAB apart, SLAB = 0 mod 32 floats: a 2-way bank conflict on every read).
// 1: rows padded to CHP chunks so that SLAB = 32 mod 64 floats, and the image shifted by one float so the patch's
// first column is 8-B aligned: 8 ds_read_b64 per patch, the 32 lanes of a group on 64 distinct banks.
template <int TC, int RD = 0, int WT = WBT>
struct WinoCfg {
    static constexpr int TR = WT / TC;              // tile rows of the block
    static constexpr int ROWS = 2 * TR + 2;         // staged input rows
    static constexpr int CH = TC / 2 + 2;           // 16-B chunks per staged row (2 TC + 8 floats)
    static constexpr int chp(int c) { return (ROWS * 4 * c) % 64 == 32 ? c : chp(c + 1); }
    static constexpr int CHP = RD == 0 ? CH : chp(CH);  // chunks per row in LDS (>= CH)
    static constexpr int SHIFT = RD == 0 ? 0 : 1;   // floats the patch image is shifted by
    static constexpr int PITCH = 4 * CHP;
    static constexpr int SLAB = ROWS * PITCH;       // floats per channel
    static constexpr int PL = WBK * ROWS * CHP;     // DMA lanes of the patch
    static constexpr int PJ = (PL + 63) / 64;       // patch DMA wave-instructions per step
    static constexpr int PF = PJ * 256 + 4 * SHIFT; // floats reserved for the patch (whole instructions)
    static constexpr int UF = WBK * 16 * WBO;       // floats of the U slab
    static constexpr int UJ = UF / 256;             // U DMA wave-instructions per step (16 B per lane)
    static constexpr int STAGE = UF + PF;
    static_assert(UJ % 4 == 0, "U slab splits evenly over the 4 waves");
    static_assert(RD == 0 || SLAB % 64 == 32, "padded slab");
};

template <int N>
__device__ __forceinline__ void wino_wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// PROBE (0 in the library) removes pieces for the timing probe tools/probes/wino_probe.hip: 1 the U DMAs after the
// first step, 2 the patch DMAs after the first step, 4 the per-step wait + barrier, 8 the epilogue, 16 the transform,
// 32 the LDS fragment reads.
// OBW: 16-channel output blocks per wave (2: 4 waves of 32 channels x 16 tiles, 2 waves / SIMD; 1: 8 waves of
// 16 channels x 16 tiles, 4 waves / SIMD -- both o-waves of a tile row transform the same patch).
// WPE: waves per SIMD the register allocation targets (0: the OBW default, 2 for OBW 2).
// WT: tiles per workgroup (64: 4 waves of 16 tiles; 128: 8 waves -- one U slab per step for twice the tiles, and
// 2 TR + 2 staged rows for 2 TR output-tile rows, at one workgroup per CU).
template <int TC, int OBW, int PROBE = 0, int RD = 0, int WPE = 0, int WT = WBT>
__global__ __launch_bounds__(64 * 8 / OBW * WT / WBT)
__attribute__((amdgpu_waves_per_eu(WPE ? WPE : 8 / (2 * OBW), WPE ? WPE : 8 / (2 * OBW))))
void wino_kernel(WinoParams p) {
    using C = WinoCfg<TC, RD, WT>;
    constexpr int NW = 8 / OBW * WT / WBT;  // waves per workgroup
    constexpr int OW = 2 / OBW;             // o-waves per tile row of waves
    constexpr int TR = C::TR, ROWS = C::ROWS, CH = C::CH, PITCH = C::PITCH, SLAB = C::SLAB, STAGE = C::STAGE;
    __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = p.h, W = p.w;

    // XCD-aware bijective order (conv_gemm.hip): consecutive ids land on one XCD, output-channel blocks fastest,
    // so the workgroups that stage the same input patch share an L2.
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const int ob = wgid % p.ntn;
    const int tg = wgid / p.ntn;
    const int per_img = p.gx * p.gy;
    const int nn = tg / per_img;
    if (nn >= p.n) return;
    const int rem = tg - nn * per_img;
    const int ty0 = (rem / p.gx) * TR, tx0 = (rem % p.gx) * TC;
    const int o0 = ob * WBO;

    const int64_t plane = (int64_t)H * W;
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * plane * 4), 0x00020000);
    const int nsteps = p.cin / WBK;

    auto issue = [&](int ks, int slot) {
        const int ci0 = ks * WBK;
        float* us = smem + slot * STAGE;
        // U slab: wave-instruction q covers runs 2q, 2q + 1 (run = channel * 4 + xi group: 32 x 16 B)
#pragma unroll
        for (int j = 0; j < ((PROBE & 1) != 0 && ks > 0 ? 0 : C::UJ / NW); ++j) {
            const int q = wave + NW * j;
            const int run = 2 * q + (lane >> 5);
            const float* src = p.uw + (((int64_t)(ci0 + (run >> 2)) * 4 + (run & 3)) * p.cout + o0 + (lane & 31)) * 4;
            __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(us + q * 256),
                                             16, 0, 0);
        }
        if constexpr ((PROBE & 2) != 0)
            if (ks > 0) return;
        float* ps = us + C::UF + C::SHIFT;
#pragma unroll
        for (int j = wave; j < C::PJ; j += NW) {
            const int L = j * 64 + lane;
            const int c = L / (ROWS * C::CHP);
            const int r2 = L - c * (ROWS * C::CHP);
            const int r = r2 / C::CHP, ch = r2 - r * C::CHP;
            const int gyy = 2 * ty0 - 1 + r, gxx = 2 * tx0 - 4 + 4 * ch;
            const bool ok = c < WBK && ch < CH && gyy >= 0 && gyy < H && gxx >= 0 && gxx < W;
            const int v = (int)((((int64_t)(nn * p.cin + ci0 + c) * H + gyy) * W + gxx) * 4);
            const int msk = -(int)ok;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, (__attribute__((address_space(3))) void*)(ps + j * 256),
                                                     16, (v & msk) | (0x7ffffff0 & ~msk), 0, 0, 0);
        }
    };

    f32x4 acc[16][OBW];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi)
#pragma unroll
        for (int b = 0; b < OBW; ++b) acc[xi][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int kq_lane = lane >> 4;   // MFMA k (channel within a k-quad)
    const int wo = wave % OW, wt = wave / OW;
    const int ob16 = wo * OBW;       // first 16-channel block of this wave
    const int tl = 16 * wt + (lane & 15);
    const int tr = tl / TC, tc = tl - tr * TC;
    const int poff = kq_lane * SLAB + 2 * tr * PITCH + 2 * tc + 3 + C::SHIFT;
    const int uoff = (kq_lane * 4 * WBO + 16 * ob16 + (lane & 15)) * 4;
    const int yy0 = 2 * (ty0 + tr), xx0 = 2 * (tx0 + tc);
    // The MODACT epilogue's per-channel / per-pixel operands, loaded before the K loop: issued after the epilogue's
    // first stores (which may alias them) they would cost one global round trip per output channel.
    float e_d[OBW][4], e_b[OBW][4], nz[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
    if (p.mode == SMC_EPI_MODACT) {
#pragma unroll
        for (int b = 0; b < OBW; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = o0 + 16 * (ob16 + b) + 4 * kq_lane + r;
                e_d[b][r] = (p.d ? p.d[(int64_t)nn * p.cout + o] : 1.f) * (p.ext.scale_c ? p.ext.scale_c[o] : 1.f);
                e_b[b][r] = p.bias ? p.bias[o] : 0.f;
            }
        if (p.noise) {
            const float nstr = p.noise_strength ? *p.noise_strength : 1.f;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    nz[i][j] = p.noise[nn * p.noise_nstride + (int64_t)(yy0 + i) * W + xx0 + j] * nstr;
        }
    }
    const bool has_s = p.s != nullptr;
    const float* srow = has_s ? p.s + (int64_t)nn * p.cin + kq_lane : p.x;
    float sv[2] = {1.f, 1.f}, sn[2] = {1.f, 1.f};

    // Fragment pipeline.  A step's 8 MFMA groups gi = 4 kq + g (k-quad kq, xi group g: 8 MFMAs each) read their A
    // fragments from a 2-deep register ring loaded one group ahead; the k-quad-1 patch is read under group 0 and
    // transformed under group 3.  The last group of a step is deferred past the next step's barrier, so its MFMAs
    // cover the LDS latency of the next step's first patch / A reads (it needs only registers).
    float pd[16], va[16], vb[16];
    f32x4 ar[2][OBW];
    bool pend = false;
    auto load_patch = [&](const float* ps, int kq) {
        if constexpr ((PROBE & 32) != 0) return;
        const float* pp = ps + kq * 4 * SLAB + poff;
        if constexpr (RD == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) pd[4 * i + j] = pp[i * PITCH + j];
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; j += 2) {
                    const float2 v = *reinterpret_cast<const float2*>(pp + i * PITCH + j);
                    pd[4 * i + j] = v.x;
                    pd[4 * i + j + 1] = v.y;
                }
        }
    };
    auto load_a = [&](const float* us, int gi, f32x4 (&a)[OBW]) {
        if constexpr ((PROBE & 32) != 0) {
#pragma unroll
            for (int b = 0; b < OBW; ++b) a[b] = f32x4{pd[gi], pd[gi + 1], pd[gi + 2], pd[b]};
            return;
        }
        const float* up = us + (gi >> 2) * 4 * 4 * WBO * 4 + uoff + (gi & 3) * WBO * 4;
#pragma unroll
        for (int b = 0; b < OBW; ++b) a[b] = *reinterpret_cast<const f32x4*>(up + 16 * 4 * b);
    };
    // V = B^T d B (rows, then columns), scaled by s[n, c]
    auto transform = [&](float sc, float (&v)[16]) {
        if constexpr ((PROBE & 16) != 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = pd[i];
            return;
        }
        float t[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            t[0][j] = pd[j] - pd[8 + j];
            t[1][j] = pd[4 + j] + pd[8 + j];
            t[2][j] = pd[8 + j] - pd[4 + j];
            t[3][j] = pd[4 + j] - pd[12 + j];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[4 * i + 0] = (t[i][0] - t[i][2]) * sc;
            v[4 * i + 1] = (t[i][1] + t[i][2]) * sc;
            v[4 * i + 2] = (t[i][2] - t[i][1]) * sc;
            v[4 * i + 3] = (t[i][1] - t[i][3]) * sc;
        }
    };
    auto mma_group = [&](int g, const f32x4 (&a)[OBW], const float (&v)[16]) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int b = 0; b < OBW; ++b)
                acc[4 * g + j][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[b][j], v[4 * g + j], acc[4 * g + j][b], 0, 0, 0);
    };

    if (nsteps > 0) {
        issue(0, 0);
        if (has_s) { sn[0] = srow[0]; sn[1] = srow[4]; }
    }
    for (int ks = 0; ks < nsteps; ++ks) {
        if constexpr ((PROBE & 4) == 0) {
            wino_wait_vmcnt<0>();
            __builtin_amdgcn_s_barrier();  // step ks landed for every wave; slot (ks + 1) & 1 is no longer read
        }
        asm volatile("" ::: "memory");
        sv[0] = sn[0]; sv[1] = sn[1];
        if (ks + 1 < nsteps) {
            issue(ks + 1, (ks + 1) & 1);
            if (has_s) { sn[0] = srow[(ks + 1) * WBK]; sn[1] = srow[(ks + 1) * WBK + 4]; }
        }
        const float* us = smem + (ks & 1) * STAGE;
        const float* ps = us + C::UF;   // (the patch image starts C::SHIFT floats further; poff includes it)
        // (sched_barrier fences keep each phase where it is written: the compiler would otherwise sink the
        // prefetches next to their use to save registers and wait on them with lgkmcnt(0))
        load_patch(ps, 0);
        load_a(us, 0, ar[0]);
        __builtin_amdgcn_sched_barrier(0);
        if (pend) mma_group(3, ar[1], vb);  // the previous step's last group
        __builtin_amdgcn_sched_barrier(0);
        transform(sv[0], va);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int gi = 0; gi < 8; ++gi) {
            if (gi + 1 < 8) load_a(us, gi + 1, ar[(gi + 1) & 1]);
            if (gi == 0) load_patch(ps, 1);
            __builtin_amdgcn_sched_barrier(0);
            if (gi < 7) {
                mma_group(gi & 3, ar[gi & 1], gi < 4 ? va : vb);
            } else {
                pend = ks + 1 < nsteps;
                if (!pend) mma_group(3, ar[1], vb);
            }
            if (gi == 3) {
                transform(sv[1], vb);
                // the transform's VALU ops between this group's MFMAs (the MFMA pipe stays fed)
#pragma unroll
                for (int q = 0; q < 4 * OBW; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 12 / OBW, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this slot's reads are done before the next barrier
    }

    // ---- epilogue: Y = A^T M A per (channel, tile), then the conv epilogue (smc::epi_y / epi_ext_apply)
    if constexpr ((PROBE & 8) != 0) {
        float sum = 0.f;
#pragma unroll
        for (int xi = 0; xi < 16; ++xi)
#pragma unroll
            for (int b = 0; b < OBW; ++b) sum += acc[xi][b][0] + acc[xi][b][1] + acc[xi][b][2] + acc[xi][b][3];
        if (sum == 12345.f) p.y[tid] = sum;
        return;
    }
    // The synthesis' two MODACT forms get a body with the activation fixed at compile time (KIND 1: lrelu with
    // 0 <= alpha <= 1, gain, clamp -- the conv1 forward; KIND 2: linear, no clamp -- the data gradient's x s[n, i]):
    // lrelu(z) = max(z, alpha z) and clamp = min / max, bit-identical to smc::epi_y for every finite value, without
    // the per-element tests of the runtime activation.  KIND 0: any epilogue through smc::epi_y / epi_ext_apply.
    auto body = [&](auto kind_c) {
        constexpr int KIND = decltype(kind_c)::value;
#pragma unroll
        for (int b = 0; b < OBW; ++b) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = o0 + 16 * (ob16 + b) + 4 * kq_lane + r;
                float m[4][4];
#pragma unroll
                for (int xi = 0; xi < 16; ++xi) m[xi >> 2][xi & 3] = acc[xi][b][r];
                float rr[2][4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    rr[0][j] = m[0][j] + m[1][j] + m[2][j];
                    rr[1][j] = m[1][j] - m[2][j] - m[3][j];
                }
                float out[2][2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    out[i][0] = rr[i][0] + rr[i][1] + rr[i][2];
                    out[i][1] = rr[i][1] - rr[i][2] - rr[i][3];
                }
                const int64_t obase = ((int64_t)nn * p.cout + o) * plane;
                if (KIND != 0 || p.mode == SMC_EPI_MODACT) {
                    const float dsc = e_d[b][r], bo = e_b[b][r];
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const int64_t idx = obase + (int64_t)(yy0 + i) * W + xx0;
                        if (p.u_save) *reinterpret_cast<float2*>(p.u_save + idx) = make_float2(out[i][0], out[i][1]);
                        float q[2];
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            if constexpr (KIND == 1) {
                                const float z = __fmaf_rn(out[i][j], dsc, nz[i][j]) + bo;
                                q[j] = fmaxf(fminf(fmaxf(z, z * p.alpha) * p.gain, p.clamp), -p.clamp);
                            } else if constexpr (KIND == 2) {
                                q[j] = (__fmaf_rn(out[i][j], dsc, nz[i][j]) + bo) * p.gain;
                            } else {
                                q[j] = smc::epi_y(out[i][j], dsc, nz[i][j], bo, p.act, p.alpha, p.gain, p.clamp);
                                if (p.ext.residual)
                                    q[j] = smc::epi_ext_apply(SMC_EPI_STORE, q[j], nn, o, idx + j, yy0 + i, xx0 + j, p.cout,
                                                              H, W, nullptr, nullptr, p.ext);
                            }
                        }
                        *reinterpret_cast<float2*>(p.y + idx) = make_float2(q[0], q[1]);
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const int64_t idx = obase + (int64_t)(yy0 + i) * W + xx0;
                        float q[2];
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            q[j] = smc::epi_ext_apply(p.mode, out[i][j], nn, o, idx + j, yy0 + i, xx0 + j, p.cout, H, W,
                                                      p.bias, p.u_save, p.ext);
                        *reinterpret_cast<float2*>(p.y + idx) = make_float2(q[0], q[1]);
                    }
                }
            }
        }
    };
    const bool modact_plain = p.mode == SMC_EPI_MODACT && !p.ext.residual;
    if (modact_plain && p.act == SMC_ACT_LRELU && p.alpha >= 0.f && p.alpha <= 1.f && p.clamp >= 0.f)
        body(std::integral_constant<int, 1>{});
    else if (modact_plain && p.act == SMC_ACT_LINEAR && p.clamp < 0.f)
        body(std::integral_constant<int, 2>{});
    else
        body(std::integral_constant<int, 0>{});
}

// U = G g G^T per (k, n): flip = 0: g = w[n][k] (k = cin, n = cout: the forward correlation);
// flip = 1: g = w[k][n] rotated by 180 degrees (k = cout, n = cin: the data gradient).  Out: [K][4][N][4].
__global__ __launch_bounds__(256) void wino_weights_kernel(const float* w, int cout, int cin, int flip, float* uw) {
    const int K = flip ? cout : cin, N = flip ? cin : cout;
    const int64_t total = (int64_t)K * N;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(e / N), nidx = (int)(e - (int64_t)k * N);
        float g[3][3];
        const float* src = flip ? w + ((int64_t)k * cin + nidx) * 9 : w + ((int64_t)nidx * cin + k) * 9;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) g[i][j] = flip ? src[(2 - i) * 3 + (2 - j)] : src[i * 3 + j];
        float gg[4][3];  // G g
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            gg[0][j] = g[0][j];
            gg[1][j] = 0.5f * (g[0][j] + g[1][j] + g[2][j]);
            gg[2][j] = 0.5f * (g[0][j] - g[1][j] + g[2][j]);
            gg[3][j] = g[2][j];
        }
        float u[4][4];   // (G g) G^T
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            u[i][0] = gg[i][0];
            u[i][1] = 0.5f * (gg[i][0] + gg[i][1] + gg[i][2]);
            u[i][2] = 0.5f * (gg[i][0] - gg[i][1] + gg[i][2]);
            u[i][3] = gg[i][2];
        }
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) uw[(((int64_t)k * 4 + (xi >> 2)) * N + nidx) * 4 + (xi & 3)] = u[xi >> 2][xi & 3];
    }
}

// tile columns of a workgroup's block: 64, 32 or 16 (the kernel's instantiations), dividing the tile grid
int wino_tc(int h, int w, int wt = WBT) {
    if (h % 2 || w % 4 || w < 32) return 0;
    for (int tc = 64; tc >= 16; tc /= 2)
        if ((w / 2) % tc == 0 && (h / 2) % (wt / tc) == 0) return tc;
    return 0;
}

}  // namespace

SMC_API int smc_conv3x3_wino_supported(int n, int cin, int cout, int h, int w) {
    if (n < 1 || cin < WBK || cin % WBK || cout < WBO || cout % WBO) return 0;
    if ((int64_t)n * cin * h * w * 4 >= (1LL << 31)) return 0;  // raw buffer offsets are 32-bit
    return wino_tc(h, w) != 0;
}

SMC_API int smc_wino_weights_f32(const float* w, int cout, int cin, int flip, float* uw, void* stream) {
    SMC_CHECK(w && uw && cout >= 1 && cin >= 1, "smc_wino_weights_f32: bad arguments");
    SMC_CHECK((reinterpret_cast<uintptr_t>(uw) & 15) == 0, "smc_wino_weights_f32: uw must be 16-B aligned");
    const int64_t total = (int64_t)cout * cin;
    hipLaunchKernelGGL(wino_weights_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(total, 256), 4096)),
                       dim3(256), 0, smc::as_stream(stream), w, cout, cin, flip, uw);
    return smc::check_launch("smc_wino_weights_f32");
}

SMC_API int smc_conv3x3_wino_f32(const float* x, int n, int cin, int h, int w, float* y, int cout, const float* uw,
                                 const float* s_in, const smc_conv_epilogue* epi, void* stream) {
    SMC_CHECK(x && y && uw, "smc_conv3x3_wino_f32: null pointer");
    if (!smc_conv3x3_wino_supported(n, cin, cout, h, w)) {
        smc::set_error("smc_conv3x3_wino_f32: no Winograd kernel for n=%d cin=%d cout=%d %dx%d", n, cin, cout, h, w);
        return SMC_ERR_UNSUPPORTED;
    }
    SMC_CHECK((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 7) == 0 &&
                  (reinterpret_cast<uintptr_t>(uw) & 15) == 0,
              "smc_conv3x3_wino_f32: x / uw must be 16-B and y 8-B aligned");
    smc_conv_epilogue e{};
    e.mode = SMC_EPI_STORE; e.act = SMC_ACT_LINEAR; e.gain = 1.f; e.clamp = -1.f;
    if (epi) e = *epi;
    SMC_CHECK(e.mode >= SMC_EPI_STORE && e.mode <= SMC_EPI_AFFINE, "smc_conv3x3_wino_f32: bad epilogue mode %d", e.mode);
    SMC_CHECK((e.mode != SMC_EPI_PRELU && e.mode != SMC_EPI_PRELU_GRAD) || e.alpha_c,
              "smc_conv3x3_wino_f32: PReLU epilogue needs alpha_c");
    SMC_CHECK(e.mode != SMC_EPI_PRELU_GRAD || e.act_ref, "smc_conv3x3_wino_f32: PRELU_GRAD needs act_ref");
    SMC_CHECK(!e.u_save || (reinterpret_cast<uintptr_t>(e.u_save) & 7) == 0, "smc_conv3x3_wino_f32: u_save alignment");
    WinoParams p{};
    p.x = x; p.n = n; p.cin = cin; p.h = h; p.w = w; p.y = y; p.cout = cout; p.uw = uw; p.s = s_in;
    p.mode = e.mode; p.d = e.d; p.noise = e.noise; p.noise_nstride = e.noise_nstride;
    p.noise_strength = e.noise_strength; p.bias = e.bias; p.act = e.act; p.alpha = e.alpha; p.gain = e.gain;
    p.clamp = e.clamp; p.u_save = e.u_save;
    p.ext = smc::epi_ext(epi);
    const int tc = wino_tc(h, w);
    p.gx = (w / 2) / tc;
    p.gy = (h / 2) / (WBT / tc);
    p.ntn = cout / WBO;
    const int64_t wgs = (int64_t)n * p.gx * p.gy * p.ntn;
    SMC_CHECK(wgs < (1LL << 31), "smc_conv3x3_wino_f32: grid too large");
    hipStream_t st = smc::as_stream(stream);
    if (tc == 64) hipLaunchKernelGGL((wino_kernel<64, WOBW>), dim3((unsigned)wgs), dim3(64 * 8 / WOBW), 0, st, p);
    else if (tc == 32) hipLaunchKernelGGL((wino_kernel<32, WOBW>), dim3((unsigned)wgs), dim3(64 * 8 / WOBW), 0, st, p);
    else hipLaunchKernelGGL((wino_kernel<16, WOBW>), dim3((unsigned)wgs), dim3(64 * 8 / WOBW), 0, st, p);
    return smc::check_launch("smc_conv3x3_wino_f32");
}
