// Implicit-GEMM "gather convolution" on fp32 MFMA for gfx950 (v_mfma_f32_32x32x2_f32).
//
// Replaces the cuDNN grouped convolutions the reference issues through
// torch_utils/ops/conv2d_resample.py:29-54 (F.conv2d / F.conv_transpose2d, groups = batch) for the
// fused modulated_conv2d.  The build computes the mathematically identical non-fused form:
//     acc[n,o,p] = sum_{t,i} W[t][i][o] * (s[n,i] * x[n,i,tap_t(p)])        (shared weights)
// so one GEMM serves the whole batch: M = batch x positions, N = out channels, K = taps x in channels.
//
// Layout of the GEMM on the matrix core: C^T[o][m] = Wt[k][o]^T . X[k][m]; the MFMA's lane index
// (column) runs over positions m, so every epilogue store of one accumulator register is 32
// consecutive pixels of one channel plane (128-B coalesced) -- the reference layout is NCHW.
//
// Tiling (256 threads = 4 waves of 64): the workgroup owns BO output channels x BM positions, each
// wave TO x TM MFMA blocks of 32x32.  K advances in steps of 16 input channels of ONE tap
// (K is ordered tap-major), so a step's input tile is a contiguous 16-channel slab at one shift:
// the per-thread position decode is done once, the per-tap bounds once per step.  Next step's tiles
// are prefetched into registers while the MFMAs consume the LDS copy (register staging, one LDS
// buffer, two barriers per step).  Low-parallelism shapes (the 4..16 px blocks) split K across
// workgroups into a workspace that the epilogue kernel reduces.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace {

constexpr int BK = 16;   // K-step granularity the host requires (cin % 16 == 0)
constexpr int NT = 256;
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct PhaseDev {
    int ntaps;
    int dy[9];
    int dx[9];
    int in_stride;
    int out_h, out_w, out_oy, out_ox, out_sy, out_sx;
    const float* wk;
    int64_t wstride;  // LDS-DMA kernel: floats between two samples' weights (0 = shared weights)
    const short* wx3;    // split-bf16 kernel: the three-term bf16 planes of wk (x3_weights_kernel layout)
    int64_t wx3_stride;  // bf16 elements between two samples' planes (0 = shared weights)
};

struct GemmParams {
    const float* x;
    int n, cin, in_h, in_w;
    float* y;
    int cout, y_h, y_w;
    PhaseDev ph[4];
    int nphases;
    const float* s;
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
    int nsplit;
    int64_t split_stride;
    int per_sample;  // LDS-DMA kernel: blockIdx.x -> (sample, tile of that sample): no tile straddles two images
    int ntn;         // LDS-DMA kernel: column tiles; grid.x = row tiles x ntn, XCD-swizzled (0: 2-D grid)
};

// Epilogue shared by the gather-GEMM kernels: lane owns column m, registers walk output channels.
// The per-channel operands of the tile's BO channels (d[n, o] * scale_c[o] / scale_c[o], bias[o], alpha_c[o]) are
// staged through LDS first (one global round trip per workgroup; `lds` must hold 3 * BO floats and is free once the
// K loop is done), and the per-element ones (act_ref, residual) are gathered 16 at a time ahead of their stores:
// loaded next to each store, every output channel would wait a global round trip behind the previous stores.
template <int WO, int WM, int TO, int TM>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, const PhaseDev& ph, const f32x16 (&acc)[TO][TM],
                                              int m0, int o0, int M, int hw_out, int split, int wo, int wm, int kh,
                                              int l32, float* lds) {
    constexpr int BO = WO * TO * 32;
    constexpr int BM = WM * TM * 32;
    const int64_t plane = (int64_t)p.y_h * p.y_w;
    if (p.nsplit > 1) {  // raw partial sums of this split
        float* dst = p.y + (int64_t)split * p.split_stride;
#pragma unroll
        for (int j = 0; j < TM; ++j) {
            const int mc = m0 + wm * TM * 32 + j * 32 + l32;
            if (mc >= M) continue;
            const int en = mc / hw_out;
            const int erem = mc - en * hw_out;
            const int ea = erem / ph.out_w;
            const int64_t pix = (int64_t)(ph.out_oy + ph.out_sy * ea) * p.y_w + ph.out_ox + ph.out_sx * (erem - ea * ph.out_w);
#pragma unroll
            for (int i = 0; i < TO; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int o = o0 + wo * TO * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                    if (o < p.cout) dst[((int64_t)en * p.cout + o) * plane + pix] = acc[i][j][r];
                }
        }
        return;
    }
    const int tid = threadIdx.x;
    const int en0 = m0 / hw_out;
    const bool one_img = (min(m0 + BM, M) - 1) / hw_out == en0;
    const int mode = p.mode;
    __syncthreads();  // every wave is done with the last K step's operand tiles
    for (int t = tid; t < BO; t += NT) {
        const int o = o0 + t;
        float mul = 1.f, add = 0.f, al = 0.f;
        if (o < p.cout) {
            if (mode == SMC_EPI_MODACT) {
                mul = (p.d && one_img ? p.d[(int64_t)en0 * p.cout + o] : 1.f) * (p.ext.scale_c ? p.ext.scale_c[o] : 1.f);
                add = p.bias ? p.bias[o] : 0.f;
            } else if (mode == SMC_EPI_PRELU || mode == SMC_EPI_AFFINE) {
                mul = p.ext.scale_c ? p.ext.scale_c[o] : 1.f;
                add = p.bias ? p.bias[o] : 0.f;
            }
            if ((mode == SMC_EPI_PRELU || mode == SMC_EPI_PRELU_GRAD) && p.ext.alpha_c) al = p.ext.alpha_c[o];
        }
        lds[t] = mul;
        lds[BO + t] = add;
        lds[2 * BO + t] = al;
    }
    __syncthreads();
    const float nstr = p.noise_strength ? *p.noise_strength : 1.f;
    const int rs = p.ext.rs;
    const int rh = p.y_h / rs, rw = p.y_w / rs;
    // One straight-line body per epilogue mode (MODE is a compile-time constant inside it): with the mode tested per
    // element every output would be its own branch region, and the loads of the next one would wait for the
    // previous stores (vmcnt counts both).
    auto body = [&](auto mode_c, auto kind_c) {
        constexpr int MODE = decltype(mode_c)::value;
        constexpr int KIND = decltype(kind_c)::value;  // MODACT: 1 lrelu (0 <= alpha <= 1) + clamp, 2 linear, 0 any
        constexpr bool EX_REF = MODE == SMC_EPI_PRELU_GRAD;  // per-element operand: act_ref (else the residual)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
            const int mc = m0 + wm * TM * 32 + j * 32 + l32;
            if (mc >= M) continue;
            const int en = mc / hw_out;
            const int erem = mc - en * hw_out;
            const int ea = erem / ph.out_w;
            const int eb = erem - ea * ph.out_w;
            const int yy = ph.out_oy + ph.out_sy * ea;
            const int xx = ph.out_ox + ph.out_sx * eb;
            const int64_t pix = (int64_t)yy * p.y_w + xx;
            const bool res_here = p.ext.residual && yy % rs == 0 && xx % rs == 0;
            const bool need_ex = EX_REF || p.ext.residual;
            float nz = 0.f;
            if (MODE == SMC_EPI_MODACT && p.noise) nz = p.noise[en * p.noise_nstride + pix] * nstr;
#pragma unroll
            for (int i = 0; i < TO; ++i) {
                const int ol0 = wo * TO * 32 + i * 32 + 4 * kh;  // tile-local channel of register r: ol0 + (r&3) + 8(r>>2)
                float ex[16];
                if (need_ex) {  // gathered before this row's stores
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int o = min(o0 + ol0 + (r & 3) + 8 * (r >> 2), p.cout - 1);
                        if (EX_REF) ex[r] = p.ext.act_ref[((int64_t)en * p.cout + o) * plane + pix];
                        else ex[r] = res_here ? p.ext.residual[(((int64_t)en * p.cout + o) * rh + yy / rs) * rw + xx / rs] : 0.f;
                    }
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int ol = ol0 + (r & 3) + 8 * (r >> 2);
                    const int o = o0 + ol;
                    if (o >= p.cout) continue;
                    const int64_t idx = ((int64_t)en * p.cout + o) * plane + pix;
                    const float v = acc[i][j][r];
                    float q;
                    if constexpr (MODE == SMC_EPI_MODACT) {
                        if (p.u_save) p.u_save[idx] = v;
                        const float dd = one_img ? lds[ol]
                                                 : (p.d ? p.d[(int64_t)en * p.cout + o] : 1.f) *
                                                       (p.ext.scale_c ? p.ext.scale_c[o] : 1.f);
                        if constexpr (KIND == 1) {  // max / min forms: bit-identical to epi_y for finite values
                            const float z = __fmaf_rn(v, dd, nz) + lds[BO + ol];
                            q = smc::lrelu_gain_clamp(z, p.alpha, p.gain, p.clamp);
                        } else if constexpr (KIND == 2) {
                            q = (__fmaf_rn(v, dd, nz) + lds[BO + ol]) * p.gain;
                        } else {
                            q = smc::epi_y(v, dd, nz, lds[BO + ol], p.act, p.alpha, p.gain, p.clamp);
                        }
                    } else if constexpr (MODE == SMC_EPI_PRELU) {
                        const float z = v * lds[ol] + lds[BO + ol];
                        if (p.u_save) p.u_save[idx] = z;
                        q = z >= 0.f ? z : z * lds[2 * BO + ol];
                    } else if constexpr (MODE == SMC_EPI_PRELU_GRAD) {
                        q = ex[r] >= 0.f ? v : v * lds[2 * BO + ol];
                        if (res_here)  // (no caller combines the two)
                            q += p.ext.residual[(((int64_t)en * p.cout + o) * rh + yy / rs) * rw + xx / rs];
                    } else if constexpr (MODE == SMC_EPI_AFFINE) {
                        q = v * lds[ol] + lds[BO + ol];
                    } else {
                        q = v;
                    }
                    if (!EX_REF && need_ex) q += ex[r];  // the residual (0 off its stride grid)
                    p.y[idx] = q;
                }
            }
        }
    };
    using K0 = std::integral_constant<int, 0>;
    switch (mode) {
        case SMC_EPI_MODACT:
            if (p.act == SMC_ACT_LRELU && p.alpha >= 0.f && p.alpha <= 1.f && p.clamp >= 0.f)
                body(std::integral_constant<int, SMC_EPI_MODACT>{}, std::integral_constant<int, 1>{});
            else if (p.act == SMC_ACT_LINEAR && p.clamp < 0.f)
                body(std::integral_constant<int, SMC_EPI_MODACT>{}, std::integral_constant<int, 2>{});
            else
                body(std::integral_constant<int, SMC_EPI_MODACT>{}, K0{});
            break;
        case SMC_EPI_PRELU: body(std::integral_constant<int, SMC_EPI_PRELU>{}, K0{}); break;
        case SMC_EPI_PRELU_GRAD: body(std::integral_constant<int, SMC_EPI_PRELU_GRAD>{}, K0{}); break;
        case SMC_EPI_AFFINE: body(std::integral_constant<int, SMC_EPI_AFFINE>{}, K0{}); break;
        default: body(std::integral_constant<int, SMC_EPI_STORE>{}, K0{}); break;
    }
}

// TAG only renames the instantiation (0: the synthesis modconv, 1: the IR-SE50 executor), so profiles can
// tell the two GEMM families apart.
template <int WO, int WM, int TO, int TM, int BKT, bool BUF, int TAG = 0>
__global__ __launch_bounds__(NT, 2) void conv_gemm_kernel(GemmParams p) {
    static_assert(WO * WM == 4, "4 waves");
    constexpr int BO = WO * TO * 32;
    constexpr int BM = WM * TM * 32;
    constexpr int XR = BKT * BM / NT;        // input-tile rows (channels) loaded per thread
    constexpr int WV = BKT * BO / 4;         // float4 vectors in the weight tile
    constexpr int WPT = (WV + NT - 1) / NT;  // float4 weight vectors per thread
    constexpr int TILE = BKT * (BO + BM);    // floats per LDS stage
    static_assert(NT % BM == 0 && XR % 4 == 0, "thread->position map");

    // One LDS array, two stages: [stage][ Ws[BKT][BO] | Xs[BKT][BM] ]
    __shared__ float smem[2 * TILE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wo = wave / WM, wm = wave % WM;

    const int phase = blockIdx.z / p.nsplit;
    const int split = blockIdx.z - phase * p.nsplit;
    const PhaseDev& ph = p.ph[phase];
    const int hw_out = ph.out_h * ph.out_w;
    const int M = p.n * hw_out;
    const int m0 = blockIdx.x * BM;
    if (m0 >= M) return;  // uniform: grid is sized for the largest phase
    const int o0 = blockIdx.y * BO;

    const int cpk = p.cin / BKT;  // channel chunks per tap
    const int ks_total = ph.ntaps * cpk;
    const int ks_begin = (int)((int64_t)ks_total * split / p.nsplit);
    const int ks_end = (int)((int64_t)ks_total * (split + 1) / p.nsplit);

    // ---- per-thread input position (fixed for the whole K loop)
    const int ml = tid % BM;
    const int kr0 = (tid / BM) * XR;
    const int m = m0 + ml;
    const bool mvalid = m < M;
    int nn = 0, a = 0, b = 0;
    if (mvalid) {
        nn = m / hw_out;
        const int rem = m - nn * hw_out;
        a = rem / ph.out_w;
        b = rem - a * ph.out_w;
    }
    const int64_t in_hw = (int64_t)p.in_h * p.in_w;
    const float* xbase = p.x + (int64_t)nn * p.cin * in_hw + (int64_t)kr0 * in_hw;
    const float* sbase = p.s ? p.s + (int64_t)nn * p.cin + kr0 : nullptr;
    const int ay = a * ph.in_stride, bx = b * ph.in_stride;

    // Prefetch registers.  Loads are unconditional and nothing consumes a loaded value before the
    // next barrier, so the loads overlap the whole step's MFMAs; the style scale is applied when the
    // tile is written to LDS.
    //  * input tile: raw buffer loads -- per-thread 32-bit voffset (position) + wave-uniform soffset
    //    (channel row), so each load costs no VALU address math; an out-of-image tap gets a voffset
    //    beyond the buffer and the hardware range check returns 0 (no select, no branch).
    //  * style scale: when a workgroup's positions lie in one image (hw_out % BM == 0) s[n, i] scales
    //    the BKT x BO weight tile (BO/BM of the multiplies of scaling the input tile).
    float xr[XR];
    float4 sr[XR / 4];
    float4 wr[WPT];
    float ws_[WPT];
    bool xok = false;
    const bool has_s = p.s != nullptr;
    const bool s_on_w = has_s && hw_out % BM == 0;
    const bool s_on_x = has_s && !s_on_w;
    const float* swhere = s_on_x ? sbase : p.x;  // any valid address when unused
    const float* sblk = s_on_w ? p.s + (int64_t)(m0 / hw_out) * p.cin : p.x;
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)(BUF ? (int64_t)p.n * p.cin * in_hw * 4 : 0), 0x00020000);
    const int xvbase = (int)(((int64_t)nn * p.cin + kr0) * in_hw) * 4;

    auto load_step = [&](int ks) {
        const int t = ks / cpk;
        const int ci0 = (ks - t * cpk) * BKT;
        const int iy = ay + ph.dy[t], ix = bx + ph.dx[t];
        xok = mvalid && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w;
        if constexpr (BUF) {
            const int voff = xok ? xvbase + (iy * p.in_w + ix) * 4 : 0x7ffffff0;
            const int srow = ci0 * (int)in_hw * 4;
#pragma unroll
            for (int r = 0; r < XR; ++r)
                xr[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                      xrsrc, voff, srow + r * (int)in_hw * 4, 0));
        } else {
            const float* src = xbase + (int64_t)ci0 * in_hw + (xok ? (int64_t)iy * p.in_w + ix : 0);
#pragma unroll
            for (int r = 0; r < XR; ++r) xr[r] = src[r * in_hw];
        }
        if (s_on_x) {
#pragma unroll
            for (int r = 0; r < XR; r += 4) sr[r / 4] = *reinterpret_cast<const float4*>(swhere + ci0 + r);
        }
#pragma unroll
        for (int q = 0; q < WPT; ++q) {
            int v = tid + q * NT;
            v = v < WV ? v : v - WV;  // surplus threads re-read a valid vector; the store skips them
            const int wkk = v / (BO / 4), wc4 = v - wkk * (BO / 4);
            const int o = o0 + wc4 * 4;
            wr[q] = *reinterpret_cast<const float4*>(ph.wk + ((int64_t)t * p.cin + ci0 + wkk) * p.cout +
                                                     (o < p.cout ? o : 0));
            ws_[q] = s_on_w ? sblk[ci0 + wkk] : 1.f;
        }
    };
    auto store_step = [&](int stage) {
        float* Ws = smem + stage * TILE;
        float* Xs = Ws + BKT * BO;
#pragma unroll
        for (int r = 0; r < XR; ++r) {
            float v = xr[r];
            if (s_on_x) {
                const float4 sv = sr[r / 4];
                v *= (r & 3) == 0 ? sv.x : (r & 3) == 1 ? sv.y : (r & 3) == 2 ? sv.z : sv.w;
            }
            if constexpr (!BUF) v = xok ? v : 0.f;
            Xs[(kr0 + r) * BM + ml] = v;
        }
#pragma unroll
        for (int q = 0; q < WPT; ++q) {
            const int v = tid + q * NT;
            const int wkk = v / (BO / 4), wc4 = v - wkk * (BO / 4);
            float4 w = wr[q];
            const float sc = (o0 + wc4 * 4 >= p.cout) ? 0.f : ws_[q];  // 0: cout = 16 in a 32-wide tile
            w.x *= sc; w.y *= sc; w.z *= sc; w.w *= sc;
            if (v < WV) *reinterpret_cast<float4*>(&Ws[wkk * BO + wc4 * 4]) = w;
        }
    };

    f32x16 acc[TO][TM];
#pragma unroll
    for (int i = 0; i < TO; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int kh = lane >> 5, l32 = lane & 31;
    int stage = 0;
    if (ks_begin < ks_end) {
        load_step(ks_begin);
        store_step(0);
    }
    __syncthreads();
    for (int ks = ks_begin; ks < ks_end; ++ks) {
        const bool more = ks + 1 < ks_end;
        if (more) load_step(ks + 1);  // global loads stay in flight under the MFMAs below
        const float* Ws = smem + stage * TILE;
        const float* Xs = Ws + BKT * BO;
        // All fragments of a 16-deep chunk are read first, pinned ahead of the MFMAs by a scheduling
        // barrier: the LDS latency is then paid once per chunk (counted lgkmcnt waits), not per k-pair.
        const float* wrow = Ws + kh * BO + wo * TO * 32 + l32;
        const float* xrow = Xs + kh * BM + wm * TM * 32 + l32;
#pragma unroll
        for (int k0 = 0; k0 < BKT; k0 += 16) {
            float af[8][TO], bf[8][TM];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
#pragma unroll
                for (int i = 0; i < TO; ++i) af[q][i] = wrow[(k0 + 2 * q) * BO + i * 32];
#pragma unroll
                for (int j = 0; j < TM; ++j) bf[q][j] = xrow[(k0 + 2 * q) * BM + j * 32];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int i = 0; i < TO; ++i)
#pragma unroll
                    for (int j = 0; j < TM; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q][i], bf[q][j], acc[i][j], 0, 0, 0);
        }
        if (more) store_step(stage ^ 1);  // the other stage was last read before the previous barrier
        __syncthreads();
        stage ^= 1;
    }

    gemm_epilogue<WO, WM, TO, TM>(p, ph, acc, m0, o0, M, hw_out, split, wo, wm, kh, l32, smem);
}

// ---------------------------------------------------------------------------------------------------
// LDS-DMA variant (the default where it applies): both operand tiles go global -> LDS with no VGPR
// staging -- the input slab by `buffer_load_dword ... lds` (lane = position, 4 B, the buffer range check
// zero-fills out-of-image taps), the weight slab by `global_load_lds_dword[x4]` -- into an NST-deep LDS
// ring.  Loads run NST-1 K steps ahead; each step waits with a counted vmcnt (never 0 in steady state)
// and a raw s_barrier (a __syncthreads would drain the in-flight DMA, cdna_hip_programming.md section 5
// "Pipelining across barriers").  Nothing is transformed in transit, so the style scale s[n,i] lives in
// per-sample weights W[t][i][o]*s[n,i] prepared by wscale_kernel (a workgroup's positions lie in one
// image); s == NULL (data gradients, IR-SE50) reads the shared weights.

template <int WF>
struct WeightDma {
    static constexpr int ww = WF % 1024 == 0 ? 4 : 1;  // floats per lane of one weight DMA
    static constexpr int bytes = ww * 4;
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int WO, int WM, int TO, int TM, int BKT, int NST, int TAG = 0>
__global__ __launch_bounds__(NT, 2) void conv_gemm_lds_kernel(GemmParams p) {
    static_assert(WO * WM == 4, "4 waves");
    constexpr int BO = WO * TO * 32;
    constexpr int BM = WM * TM * 32;
    constexpr int TILE = BKT * (BO + BM);
    constexpr int NCH = BM / 64;                 // 64-position chunks per input row
    static_assert(NCH >= 1 && NCH <= 4 && 4 % NCH == 0, "BM in {64,128,256}");
    constexpr int RSTEP = 4 / NCH;               // rows between one wave's consecutive input DMAs
    constexpr int XI = BKT * NCH / 4;            // input DMAs per wave per step
    constexpr int WF = BKT * BO;                 // floats in the weight slab
    constexpr int WW = WeightDma<WF>::ww;         // floats per lane of a weight DMA
    static_assert(WF % (256 * WW) == 0, "weight slab must split evenly over the 4 waves");
    constexpr int WI = WF / (256 * WW);          // weight DMAs per wave per step
    constexpr int PER = XI + WI;
    static_assert(NST >= 2 && NST <= 4 && PER * (NST - 2) <= 63, "vmcnt range");
    __shared__ __attribute__((aligned(16))) float smem[NST * TILE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: DMA bases / M0 need SGPRs
    const int wo = wave / WM, wm = wave % WM;
    const int phase = blockIdx.z / p.nsplit;
    const int split = blockIdx.z - phase * p.nsplit;
    const PhaseDev& ph = p.ph[phase];
    const int hw_out = ph.out_h * ph.out_w;
    // XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs (private L2 each), so the
    // bijective remap below gives every XCD a contiguous run of tiles, column tiles fastest: the workgroups
    // that share an input tile (all column tiles of one row tile) and the row-neighbour tiles the 3x3 taps
    // re-read run on the same L2.
    int tm = blockIdx.x, tn = blockIdx.y;
    if (p.ntn) {
        const int nwg = gridDim.x, orig = blockIdx.x;
        const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
        const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
        tm = wgid / p.ntn;
        tn = wgid - tm * p.ntn;
    }
    int M = p.n * hw_out;
    int m0 = tm * BM;
    if (p.per_sample) {
        // per-sample weights with hw_out % BM != 0: tiles restart at every image (M = that image's end)
        const int tps = (hw_out + BM - 1) / BM;
        const int nb = tm / tps;
        if (nb >= p.n) return;
        m0 = nb * hw_out + (tm - nb * tps) * BM;
        M = (nb + 1) * hw_out;
    }
    if (m0 >= M) return;
    const int o0 = tn * BO;
    const int cpk = p.cin / BKT;
    const int ks_total = ph.ntaps * cpk;
    const int ks_begin = (int)((int64_t)ks_total * split / p.nsplit);
    const int ks_end = (int)((int64_t)ks_total * (split + 1) / p.nsplit);

    // input DMAs: wave -> chunk cw (64 positions), rows r0 + RSTEP*j; lane -> one position
    const int cw = wave % NCH, r0 = wave / NCH;
    const int m = m0 + cw * 64 + lane;
    const bool mvalid = m < M;
    int nn = 0, a = 0, b = 0;
    if (mvalid) {
        nn = m / hw_out;
        const int rem = m - nn * hw_out;
        a = rem / ph.out_w;
        b = rem - a * ph.out_w;
    }
    const int in_hw = p.in_h * p.in_w;
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * in_hw * 4), 0x00020000);
    const int xvbase = nn * p.cin * in_hw * 4;
    const int ay = a * ph.in_stride, bx = b * ph.in_stride;
    // weight DMAs: this workgroup's sample (s != NULL) or the shared weights
    const float* wk = ph.wk + (ph.wstride ? (int64_t)(m0 / hw_out) * ph.wstride : 0);

    auto issue = [&](int ks, int slot) {
        const int t = ks / cpk;
        const int ci0 = (ks - t * cpk) * BKT;
        const int iy = ay + ph.dy[t], ix = bx + ph.dx[t];
        const bool ok = mvalid && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w;
        const int voff = ok ? xvbase + (iy * p.in_w + ix) * 4 : 0x7ffffff0;
        float* xs = smem + slot * TILE + BKT * BO;
#pragma unroll
        for (int j = 0; j < XI; ++j) {
            const int row = r0 + RSTEP * j;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                xrsrc, (__attribute__((address_space(3))) void*)(xs + row * BM + cw * 64), 4, voff,
                (ci0 + row) * in_hw * 4, 0, 0);
        }
        float* ws = smem + slot * TILE;
        const float* wrow = wk + ((int64_t)t * p.cin + ci0) * p.cout + o0;
#pragma unroll
        for (int j = 0; j < WI; ++j) {
            const int f0 = (wave + 4 * j) * 64 * WW;          // first float of this DMA in the slab
            const int f = f0 + lane * WW;
            const int row = f / BO, col = f - row * BO;
            const void* src = (const void*)(wrow + (int64_t)row * p.cout + col);
            auto* dst = (__attribute__((address_space(3))) void*)(ws + f0);
            if constexpr (WW == 4) __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
            else __builtin_amdgcn_global_load_lds(src, dst, 4, 0, 0);
        }
    };

    f32x16 acc[TO][TM];
#pragma unroll
    for (int i = 0; i < TO; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int kh = lane >> 5, l32 = lane & 31;
    int issued = ks_begin;
#pragma unroll
    for (int q = 0; q < NST - 1; ++q) {
        if (issued < ks_end) {
            issue(issued, (issued - ks_begin) % NST);
            ++issued;
        }
    }
    for (int ks = ks_begin; ks < ks_end; ++ks) {
        // this wave's DMAs for step ks are done once at most (issued - ks - 1) later steps remain in flight
        const int ahead = issued - ks - 1;
        if constexpr (NST == 2) {
            wait_vmcnt<0>();
        } else if constexpr (NST == 3) {
            if (ahead >= 1) wait_vmcnt<PER>();
            else wait_vmcnt<0>();
        } else {
            if (ahead >= 2) wait_vmcnt<2 * PER>();
            else if (ahead == 1) wait_vmcnt<PER>();
            else wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();  // every wave's DMAs for step ks have landed; slot ks-1 is free
        asm volatile("" ::: "memory");
        const int slot = (ks - ks_begin) % NST;
        const float* Ws = smem + slot * TILE;
        const float* Xs = Ws + BKT * BO;
        const float* wrow = Ws + kh * BO + wo * TO * 32 + l32;
        const float* xrow = Xs + kh * BM + wm * TM * 32 + l32;
        // Step schedule: the workgroups sharing a CU run in near lockstep, so whatever a wave does between
        // the barrier and its first MFMA leaves the SIMD's MFMA pipe idle for every wave at once.  Only the
        // first half-chunk of fragment reads precedes the first MFMAs; the DMA issue for a later step and
        // the second half of the reads are issued under the executing MFMAs.
#pragma unroll
        for (int k0 = 0; k0 < BKT; k0 += 16) {
            float af[8][TO], bf[8][TM];
            auto frag = [&](int q) {
#pragma unroll
                for (int i = 0; i < TO; ++i) af[q][i] = wrow[(k0 + 2 * q) * BO + i * 32];
#pragma unroll
                for (int j = 0; j < TM; ++j) bf[q][j] = xrow[(k0 + 2 * q) * BM + j * 32];
            };
            // software pipeline over the 8 K-pairs: fragments of pair q+2 are read under pair q's MFMAs
            frag(0);
            frag(1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
#pragma unroll
                for (int i = 0; i < TO; ++i)
#pragma unroll
                    for (int j = 0; j < TM; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q][i], bf[q][j], acc[i][j], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (q == 0 && k0 == 0 && issued < ks_end) {
                    issue(issued, (issued - ks_begin) % NST);
                    ++issued;
                }
                if (q + 2 < 8) frag(q + 2);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // fragment reads of this slot done before the next barrier
    }
    gemm_epilogue<WO, WM, TO, TM>(p, ph, acc, m0, o0, M, hw_out, split, wo, wm, kh, l32, smem);
}

// ---------------------------------------------------------------------------------------------------
// Split-bf16 form of conv_gemm_lds_kernel: the same tiles, K steps, DMA ring and epilogue, the fp32 products on the
// bf16 matrix core (v_mfma_f32_32x32x16_bf16) as three-term splits.  Every fp32 operand is split exactly into
// three bf16 terms, a = a0 + a1 + a2 (truncation: a0 = the top 8 significant bits, a1 the next 8 of a - a0, a2 the
// last 8), and a * b is accumulated as the six products a_i b_j with i + j <= 2 -- smallest first -- leaving out
// a1 b2 + a2 b1 + a2 b2 <= 2^-23 |a b|: the error of one fp32 rounding, per product.  The bf16 MFMA runs 16x the
// fp32 MFMA's FLOP rate, so six of them cost 6/16 of one fp32 product (tools/probes/bx6_probe.hip, LDS-fed tile
// loop: 146 TF/s fp32 MFMA, 251 TF/s split with the input split in registers; max error vs fp64 9.3e-6 against
// 1.4e-5 for the fp32 MFMA on the same sums).
//   * weights (frozen, or the per-sample W * s): split once into planes [taps][cin/16][3][2][cout][8] bf16
//     (x3_weights_kernel) that the DMA copies as they are: an A fragment (8 consecutive k of one output channel)
//     is one conflict-free ds_read_b128 per term;
//   * input: the fp32 slab [BKT][BM] of conv_gemm_lds_kernel; a B fragment (8 consecutive k of one position) is 8
//     ds_read_b32, split in registers (4 VALU per value + 3 v_perm per pair) and reused by the wave's TO blocks.
// The C/D layout of the 32x32x16 bf16 MFMA is that of the fp32 32x32x2 one, so gemm_epilogue is shared.

typedef short bf16x8 __attribute__((ext_vector_type(8)));

// a = t0 + t1 + t2 for each of 8 values, as three bf16x8 fragments (the high halves of a, a - t0, a - t0 - t1)
__device__ __forceinline__ void x3_split8(const float (&x)[8], bf16x8 (&t)[3]) {
    unsigned u0[8], u1[8], u2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const unsigned u = __float_as_uint(x[j]);
        const float r1 = x[j] - __uint_as_float(u & 0xffff0000u);
        const unsigned v = __float_as_uint(r1);
        const float r2 = r1 - __uint_as_float(v & 0xffff0000u);
        u0[j] = u;
        u1[j] = v;
        u2[j] = __float_as_uint(r2);
    }
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 w0, w1, w2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // (high half of element 2j) | (high half of element 2j + 1) << 16
        w0[j] = __builtin_amdgcn_perm(u0[2 * j + 1], u0[2 * j], 0x07060302u);
        w1[j] = __builtin_amdgcn_perm(u1[2 * j + 1], u1[2 * j], 0x07060302u);
        w2[j] = __builtin_amdgcn_perm(u2[2 * j + 1], u2[2 * j], 0x07060302u);
    }
    t[0] = __builtin_bit_cast(bf16x8, w0);
    t[1] = __builtin_bit_cast(bf16x8, w1);
    t[2] = __builtin_bit_cast(bf16x8, w2);
}

// acc += a * b over the six split products, smallest first
__device__ __forceinline__ f32x16 x3_mma(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
}

// out[nn][t][ci / 16][s][(ci % 16) / 8][o][ci % 8] = term s of wk[t][ci][o] * (s_in ? s_in[nn][ci] : 1)
__global__ __launch_bounds__(256) void x3_weights_kernel(const float* wk, const float* s_in, short* out, int ntaps,
                                                         int cin, int cout, int n) {
    const int64_t per = (int64_t)ntaps * cin * cout;
    const int64_t total = per * n;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        // e -> (nn, t, c16, kq, o, ee): ee fastest (the 16-B runs the kernel's DMA reads)
        const int ee = (int)(e & 7);
        int64_t r = e >> 3;
        const int o = (int)(r % cout);
        r /= cout;
        const int kq = (int)(r & 1);
        r >>= 1;
        const int c16 = (int)(r % (cin / 16));
        r /= cin / 16;
        const int t = (int)(r % ntaps);
        const int nn = (int)(r / ntaps);
        const int ci = c16 * 16 + kq * 8 + ee;
        const float v = wk[((int64_t)t * cin + ci) * cout + o] * (s_in ? s_in[(int64_t)nn * cin + ci] : 1.f);
        const unsigned u = __float_as_uint(v);
        const float r1 = v - __uint_as_float(u & 0xffff0000u);
        const unsigned w = __float_as_uint(r1);
        const float r2 = r1 - __uint_as_float(w & 0xffff0000u);
        const unsigned term[3] = {u >> 16, w >> 16, __float_as_uint(r2) >> 16};
        short* dst = out + nn * per * 3;
#pragma unroll
        for (int sidx = 0; sidx < 3; ++sidx)
            dst[((((int64_t)t * (cin / 16) + c16) * 3 + sidx) * 2 + kq) * ((int64_t)cout * 8) + (int64_t)o * 8 + ee] =
                (short)term[sidx];
    }
}

// Ring depth of the split-bf16 kernel (A/B knob: SMC_AB_DEFINES=-DSMC_X3_NST=n builds a variant library).  Its K step
// holds 2.67x fewer MFMA cycles than the fp32 kernel's, so the DMA latency a 2-stage ring leaves exposed is larger.
#ifndef SMC_X3_NST
#define SMC_X3_NST 2
#endif
#ifndef SMC_X3_K32_SMALL
#define SMC_X3_K32_SMALL 1
#endif
// Tiles whose waves each own all of the tile's output channels (WO = 1: 128 x 32 or 64 x 32 per wave instead of
// 64 x 64 / 32 x 64): a B fragment is split once per workgroup instead of once per wave pair (A/B knob)
#ifndef SMC_X3_WO1
#define SMC_X3_WO1 1
#endif
// ... with 16-channel K steps (half the LDS per stage: 3 workgroups per CU instead of 2; A/B knob).  Measured
// (profiles/r05/ab5/, two interleaved rounds on one box): 468.96 / 467.66 against 467.77 / 466.56 images/s.
#ifndef SMC_X3_WO1_K16
#define SMC_X3_WO1_K16 1
#endif
// Timing probes only (0 in the library; tools/ builds a variant with SMC_AB_DEFINES): 1 drops the input DMAs after
// the first K step, 2 the weight DMAs after the first, 4 the register split (the fp32 bits reused as the three terms)
#ifndef SMC_X3_PROBE
#define SMC_X3_PROBE 0
#endif

// Wide tiles (AS: 256 output channels x 128 positions, each wave 256 x 32): the K step's input DMAs and its B split
// are amortised over twice the MFMAs of the 128-channel tile (per wave and step: 8 input + 6 weight DMAs, 44 split
// VALU for 48 MFMAs, against 8 + 3 and 44 for 24), the issue budget the 128-channel tile overruns.  The A fragments
// are read one output block ahead of its MFMAs instead of all at once (128 accumulator registers leave no room for
// 8 x 3 fragments).  Only where the 256-channel grid needs no split-K, for shared weights (A/B knob SMC_X3_WIDE).
// Measured it gains less than the issue count suggests (-5 % on the r = 256 data gradient, +2 % on the style-scaled
// r = 128 forward): the 128-channel tile is not bound by its DMA + split issue alone.
#ifndef SMC_X3_WIDE
#define SMC_X3_WIDE 1
#endif

template <int WO, int WM, int TO, int TM, int BKT, int NST = SMC_X3_NST, int TAG = 0, bool AS = false>
__global__ __launch_bounds__(NT, 2) void conv_gemm_x3_kernel(GemmParams p) {
    static_assert(WO * WM == 4, "4 waves");
    static_assert(BKT % 16 == 0, "16-channel chunks");
    static_assert(!AS || (BKT == 16 && TM == 1 && NST == 2), "streamed A fragments: one 16-channel chunk per step");
    constexpr int BO = WO * TO * 32;
    constexpr int BM = WM * TM * 32;
    constexpr int NKC = BKT / 16;                // 16-channel chunks per K step (one bf16 MFMA K each)
    constexpr int WB = NKC * 6 * BO * 16;         // bytes of the step's weight planes [NKC][3][2][BO][8] bf16
    constexpr int XB = BKT * BM * 4;              // bytes of the step's input slab [BKT][BM] fp32
    constexpr int STAGE = WB + XB;
    constexpr int NCH = BM / 64;                 // 64-position chunks per input row
    static_assert(NCH >= 1 && NCH <= 4 && 4 % NCH == 0, "BM in {64,128,256}");
    constexpr int RSTEP = 4 / NCH;
    constexpr int XI = BKT * NCH / 4;            // input DMAs per wave per step
    static_assert(WB % 1024 == 0, "weight planes split into whole 1-KB DMAs");
    constexpr int WLI = WB / 1024;               // weight DMAs per step (whole workgroup)
    constexpr int WIW = (WLI + 3) / 4;           // ... per wave (the last round re-issues early ones: same bytes, same
                                                 // place), so every wave counts the same DMAs per step
    constexpr int PER = XI + WIW;
    static_assert(NST >= 2 && NST <= 4 && PER * (NST - 2) <= 63, "vmcnt range");
    __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wo = wave / WM, wm = wave % WM;
    const int phase = blockIdx.z / p.nsplit;
    const int split = blockIdx.z - phase * p.nsplit;
    const PhaseDev& ph = p.ph[phase];
    const int hw_out = ph.out_h * ph.out_w;
    int tm = blockIdx.x, tn = blockIdx.y;
    if (p.ntn) {  // XCD-aware bijective tile order (conv_gemm_lds_kernel)
        const int nwg = gridDim.x, orig = blockIdx.x;
        const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
        const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
        tm = wgid / p.ntn;
        tn = wgid - tm * p.ntn;
    }
    int M = p.n * hw_out;
    int m0 = tm * BM;
    if (p.per_sample) {
        const int tps = (hw_out + BM - 1) / BM;
        const int nb = tm / tps;
        if (nb >= p.n) return;
        m0 = nb * hw_out + (tm - nb * tps) * BM;
        M = (nb + 1) * hw_out;
    }
    if (m0 >= M) return;
    const int o0 = tn * BO;
    const int cpk = p.cin / BKT;
    const int ks_total = ph.ntaps * cpk;
    const int ks_begin = (int)((int64_t)ks_total * split / p.nsplit);
    const int ks_end = (int)((int64_t)ks_total * (split + 1) / p.nsplit);

    const int cw = wave % NCH, r0 = wave / NCH;
    const int m = m0 + cw * 64 + lane;
    const bool mvalid = m < M;
    int nn = 0, a = 0, b = 0;
    if (mvalid) {
        nn = m / hw_out;
        const int rem = m - nn * hw_out;
        a = rem / ph.out_w;
        b = rem - a * ph.out_w;
    }
    const int in_hw = p.in_h * p.in_w;
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * in_hw * 4), 0x00020000);
    const int xvbase = nn * p.cin * in_hw * 4;
    const int ay = a * ph.in_stride, bx = b * ph.in_stride;
    const short* wx = ph.wx3 + (ph.wx3_stride ? (int64_t)(m0 / hw_out) * ph.wx3_stride : 0);
    const int c16n = p.cin / 16;
    // weight-plane DMAs through a buffer resource: each lane's byte offset within a step's planes is fixed (computed
    // once here), the step's part is wave-uniform (soffset) -- no per-DMA 64-bit address VALU in the K loop
    const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)wx, (short)0, 0x7ffffff0, 0x00020000);
    int woff[WIW];
#pragma unroll
    for (int jw = 0; jw < WIW; ++jw) {
        int j = wave + 4 * jw;
        if (j >= WLI) j -= WLI;  // wave-uniform
        const int L = j * 64 + lane;
        const int run = L / BO, o = L - run * BO;   // run = chunk * 6 + term * 2 + octet
        woff[jw] = (run * p.cout + o0 + o) * 16;
    }

    auto issue = [&](int ks, int slot) {
        const int t = ks / cpk;
        const int ci0 = (ks - t * cpk) * BKT;
        const int iy = ay + ph.dy[t], ix = bx + ph.dx[t];
        const bool ok = mvalid && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w;
        const int voff = ok ? xvbase + (iy * p.in_w + ix) * 4 : 0x7ffffff0;
        char* st = smem + slot * STAGE;
        float* xs = reinterpret_cast<float*>(st + WB);
#pragma unroll
        for (int j = 0; j < ((SMC_X3_PROBE & 1) && ks > ks_begin ? 0 : XI); ++j) {
            const int row = r0 + RSTEP * j;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                xrsrc, (__attribute__((address_space(3))) void*)(xs + row * BM + cw * 64), 4, voff,
                (ci0 + row) * in_hw * 4, 0, 0);
        }
        // weight planes: 16-B lanes over [NKC][6 = term x octet][BO] (each (term, octet) run of BO lanes contiguous
        // in global memory at (((t * cin / 16 + chunk) * 6 + run) * cout + o0 + o) * 8 bf16)
        const int wsoff = ((t * c16n + ci0 / 16) * 6) * p.cout * 16;
#pragma unroll
        for (int jw = 0; jw < ((SMC_X3_PROBE & 2) && ks > ks_begin ? 0 : WIW); ++jw) {
            int j = wave + 4 * jw;
            if (j >= WLI) j -= WLI;  // wave-uniform
            const int vo = woff[jw];  // (through a local: hipcc drops the kernel's host stub when the array is passed)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wrsrc, (__attribute__((address_space(3))) void*)(st + j * 1024), 16,
                                                     vo, wsoff, 0, 0);
        }
    };

    f32x16 acc[TO][TM];
#pragma unroll
    for (int i = 0; i < TO; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int kh = lane >> 5, l32 = lane & 31;
    int issued = ks_begin;
#pragma unroll
    for (int q = 0; q < NST - 1; ++q) {
        if (issued < ks_end) {
            issue(issued, (issued - ks_begin) % NST);
            ++issued;
        }
    }
    for (int ks = ks_begin; ks < ks_end; ++ks) {
        // this wave's DMAs for step ks are done once at most (issued - ks - 1) later steps remain in flight
        const int ahead = issued - ks - 1;
        if constexpr (NST == 2) {
            wait_vmcnt<0>();
        } else if constexpr (NST == 3) {
            if (ahead >= 1) wait_vmcnt<PER>();
            else wait_vmcnt<0>();
        } else {
            if (ahead >= 2) wait_vmcnt<2 * PER>();
            else if (ahead == 1) wait_vmcnt<PER>();
            else wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();  // every wave's DMAs for step ks have landed; slot ks-1 is free
        asm volatile("" ::: "memory");
        const int slot = (ks - ks_begin) % NST;
        const char* st = smem + slot * STAGE;
        const short* Wp = reinterpret_cast<const short*>(st);
        const float* Xs = reinterpret_cast<const float*>(st + WB);
        const float* xcol = Xs + wm * TM * 32 + l32;
        if constexpr (AS) {
            float xw[8];
            bf16x8 ar[2][3];
#pragma unroll
            for (int e = 0; e < 8; ++e) xw[e] = xcol[(8 * kh + e) * BM];
            auto read_a = [&](int i, int b) {
#pragma unroll
                for (int s = 0; s < 3; ++s)
                    ar[b][s] = *reinterpret_cast<const bf16x8*>(Wp + (((s * 2 + kh) * BO) + wo * TO * 32 + i * 32 + l32) * 8);
            };
            read_a(0, 0);
            if (issued < ks_end) {  // the next step's DMAs under this step's first reads
                issue(issued, (issued - ks_begin) % NST);
                ++issued;
            }
            bf16x8 bw[3];
            x3_split8(xw, bw);
#pragma unroll
            for (int i = 0; i < TO; ++i) {
                if (i + 1 < TO) read_a(i + 1, (i + 1) & 1);
                acc[i][0] = x3_mma(ar[i & 1], bw, acc[i][0]);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            continue;
        }
        // Chunk pipeline: chunk kc + 1's fragment reads and input split are issued in the same region as chunk kc's
        // MFMAs (no scheduling fence between them), so the LDS latency and the split VALU fill the MFMA issue gaps.
        float xv[2][TM][8];
        bf16x8 at[2][TO][3];
        auto read_frags = [&](int kc, int b) {
#pragma unroll
            for (int j = 0; j < TM; ++j)
#pragma unroll
                for (int e = 0; e < 8; ++e) xv[b][j][e] = xcol[(kc * 16 + 8 * kh + e) * BM + j * 32];
#pragma unroll
            for (int i = 0; i < TO; ++i)
#pragma unroll
                for (int s = 0; s < 3; ++s)
                    at[b][i][s] = *reinterpret_cast<const bf16x8*>(
                        Wp + ((((kc * 3 + s) * 2 + kh) * BO) + wo * TO * 32 + i * 32 + l32) * 8);
        };
        read_frags(0, 0);
        if (issued < ks_end) {  // a later step's DMAs, issued while this step's first reads are in flight
            issue(issued, (issued - ks_begin) % NST);
            ++issued;
        }
        bf16x8 bt[TM][3];
#pragma unroll
        for (int j = 0; j < TM; ++j) {
            if constexpr ((SMC_X3_PROBE & 4) != 0) {
                typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 w = {__float_as_uint(xv[0][j][0]), __float_as_uint(xv[0][j][2]),
                                 __float_as_uint(xv[0][j][4]), __float_as_uint(xv[0][j][6])};
                bt[j][0] = bt[j][1] = bt[j][2] = __builtin_bit_cast(bf16x8, w);
            } else {
                x3_split8(xv[0][j], bt[j]);
            }
        }
#pragma unroll
        for (int kc = 0; kc < NKC; ++kc) {
            const int b = kc & 1;
            if (kc + 1 < NKC) read_frags(kc + 1, b ^ 1);
            bf16x8 btn[TM][3];
#pragma unroll
            for (int i = 0; i < TO; ++i)
#pragma unroll
                for (int j = 0; j < TM; ++j) acc[i][j] = x3_mma(at[b][i], bt[j], acc[i][j]);
            if (kc + 1 < NKC) {
#pragma unroll
                for (int j = 0; j < TM; ++j) {
                    if constexpr ((SMC_X3_PROBE & 4) != 0) {
                        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                        const u32x4 w = {__float_as_uint(xv[b ^ 1][j][0]), __float_as_uint(xv[b ^ 1][j][2]),
                                         __float_as_uint(xv[b ^ 1][j][4]), __float_as_uint(xv[b ^ 1][j][6])};
                        btn[j][0] = btn[j][1] = btn[j][2] = __builtin_bit_cast(bf16x8, w);
                    } else {
                        x3_split8(xv[b ^ 1][j], btn[j]);
                    }
                }
#pragma unroll
                for (int j = 0; j < TM; ++j)
#pragma unroll
                    for (int s = 0; s < 3; ++s) bt[j][s] = btn[j][s];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // fragment reads of this slot done before the next barrier
    }
    if constexpr (AS) {
        // two 128-channel halves (the 8-block body is not unrolled by the compiler: the accumulators would go to
        // scratch for a dynamically indexed epilogue)
        static_assert(WO == 1 && TO % 2 == 0, "halves");
        f32x16 lo[TO / 2][TM], hi[TO / 2][TM];
#pragma unroll
        for (int i = 0; i < TO / 2; ++i) {
            lo[i][0] = acc[i][0];
            hi[i][0] = acc[TO / 2 + i][0];
        }
        gemm_epilogue<WO, WM, TO / 2, TM>(p, ph, lo, m0, o0, M, hw_out, split, wo, wm, kh, l32,
                                          reinterpret_cast<float*>(smem));
        gemm_epilogue<WO, WM, TO / 2, TM>(p, ph, hi, m0, o0 + (TO / 2) * 32, M, hw_out, split, wo, wm, kh, l32,
                                          reinterpret_cast<float*>(smem));
        return;
    }
    gemm_epilogue<WO, WM, TO, TM>(p, ph, acc, m0, o0, M, hw_out, split, wo, wm, kh, l32,
                                  reinterpret_cast<float*>(smem));
}

// Row-halo variant for the 3x3 stride-1 'same' convs whose position tiles are row segments (W % BM == 0: the
// r >= 128 conv1 forward and data gradient).  The tap-major kernel above stages one BKT x BM input slab per tap,
// so every input pixel crosses L2 -> LDS nine times.  Here a K step is (tap row dy, BKT channels): the slab is
// the input row a + dy over [b0 - 4, b0 + BM + 4) -- one 16-B DMA lane per 4 pixels, aligned because W and b0
// are multiples of 4 -- and the three taps dx = -1, 0, 1 of that row read it at offsets 3, 4, 5.  Input staging
// per FLOP drops 3x and the DMA instruction count ~3x; weights for the three taps ride in the same step.
// Out-of-image pixels (row ends, rows -1 and H) come back as zeros from the buffer range check.
struct RowTaps {
    int t[3][3];  // packed-weight tap index of (dy + 1, dx + 1)
};

template <int WO, int WM, int TO, int TM, int BKT>
struct RowCfg {
    static constexpr int BO = WO * TO * 32;
    static constexpr int BM = WM * TM * 32;
    static constexpr int CHK = (BM + 8) / 4;               // 16-B chunks of one halo'd row
    // floats per staged row: the smallest >= CHK * 4 that is 32 mod 64 (the two half-waves' B reads, rows k and
    // k + 1, fall on disjoint LDS banks)
    static constexpr int PITCH = ((CHK * 4 - 32 + 63) / 64) * 64 + 32;
    static constexpr int XL = BKT * PITCH / 4;               // DMA lanes of the X slab (pitch padding included)
    static constexpr int XJ = (XL + 63) / 64;                // X DMA wave-instructions per step
    static constexpr int XF = XJ * 64 * 4;                   // floats reserved for X (whole instructions)
    static constexpr int WF = 3 * BKT * BO;                  // floats of the three taps' weight slabs
    static constexpr int WJ = WF / 256;                      // weight DMA wave-instructions per step (16 B/lane)
    static constexpr int STAGE = XF + WF;
    static_assert(WF % 256 == 0, "weight slabs split into whole 1-KB DMAs");
    static_assert(PITCH % 64 == 32 && PITCH >= CHK * 4, "row pitch");
};

template <int WO, int WM, int TO, int TM, int BKT>
__global__ __launch_bounds__(NT, 2) void conv_row_kernel(GemmParams p, RowTaps rt) {
    using C = RowCfg<WO, WM, TO, TM, BKT>;
    constexpr int BO = C::BO, BM = C::BM, PITCH = C::PITCH, STAGE = C::STAGE;
    constexpr int RCH = PITCH / 4;                           // DMA lanes per staged row
    static_assert(WO * WM == 4, "4 waves");
    __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wo = wave / WM, wm = wave % WM;
    const PhaseDev& ph = p.ph[0];
    const int H = p.in_h, W = p.in_w, hw = H * W;
    int tm = blockIdx.x, tn = blockIdx.y;
    if (p.ntn) {  // XCD-aware bijective tile order (see conv_gemm_lds_kernel)
        const int nwg = gridDim.x, orig = blockIdx.x;
        const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
        const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
        tm = wgid / p.ntn;
        tn = wgid - tm * p.ntn;
    }
    const int m0 = tm * BM;
    if (m0 >= p.n * hw) return;
    const int nn = m0 / hw;
    const int rem = m0 - nn * hw;
    const int a = rem / W, b0 = rem - a * W;
    const int o0 = tn * BO;
    const int cpk = p.cin / BKT;
    const int ks_total = 3 * cpk;
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * hw * 4), 0x00020000);
    const float* wk = ph.wk + (ph.wstride ? (int64_t)nn * ph.wstride : 0);

    auto issue = [&](int ks, int slot) {
        const int dyi = ks / cpk;
        const int ci0 = (ks - dyi * cpk) * BKT;
        const int iy = a + dyi - 1;
        const bool rowok = iy >= 0 && iy < H;
        float* xs = smem + slot * STAGE;
        // X slab: lane L -> (row L / RCH, 16-B chunk L % RCH) at pixel b0 - 4 + 4 * chunk
#pragma unroll
        for (int j = wave; j < C::XJ; j += 4) {
            const int L = j * 64 + lane;
            const int row = L / RCH, ch = L - row * RCH;
            const int x = b0 - 4 + 4 * ch;
            const bool ok = rowok && row < BKT && ch < C::CHK && x >= 0 && x < W;
            const int v = ((((nn * p.cin + ci0 + row) * H + iy) * W) + x) * 4;
            const int msk = -(int)ok;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, (__attribute__((address_space(3))) void*)(xs + j * 256), 16,
                                                     (v & msk) | (0x7ffffff0 & ~msk), 0, 0, 0);
        }
        // weights of the three taps of row dy: [tt][ci][o] slabs, 4 floats per lane
        float* ws = xs + C::XF;
#pragma unroll
        for (int j = wave; j < C::WJ; j += 4) {
            const int f = (j * 64 + lane) * 4;
            const int tt = f / (BKT * BO);
            const int r2 = f - tt * (BKT * BO);
            const int ci = r2 / BO, o = r2 - ci * BO;
            const float* src = wk + ((int64_t)rt.t[dyi][tt] * p.cin + ci0 + ci) * p.cout + o0 + o;
            __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(ws + j * 256),
                                             16, 0, 0);
        }
    };

    f32x16 acc[TO][TM];
#pragma unroll
    for (int i = 0; i < TO; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int kh = lane >> 5, l32 = lane & 31;
    if (ks_total > 0) issue(0, 0);
    for (int ks = 0; ks < ks_total; ++ks) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // step ks landed for every wave; the other slot is free
        asm volatile("" ::: "memory");
        const int slot = ks & 1;
        const float* Xs = smem + slot * STAGE + kh * PITCH + 3 + wm * TM * 32 + l32;
        const float* Ws = smem + slot * STAGE + C::XF + kh * BO + wo * TO * 32 + l32;
#pragma unroll
        for (int tt = 0; tt < 3; ++tt) {
#pragma unroll
            for (int k0 = 0; k0 < BKT; k0 += 8) {
                float af[4][TO], bf[4][TM];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
#pragma unroll
                    for (int i = 0; i < TO; ++i) af[q][i] = Ws[(tt * BKT + k0 + 2 * q) * BO + i * 32];
#pragma unroll
                    for (int j = 0; j < TM; ++j) bf[q][j] = Xs[(k0 + 2 * q) * PITCH + tt + j * 32];
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int i = 0; i < TO; ++i)
#pragma unroll
                        for (int j = 0; j < TM; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q][i], bf[q][j], acc[i][j], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (tt == 0 && k0 == 0 && ks + 1 < ks_total) issue(ks + 1, slot ^ 1);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    gemm_epilogue<WO, WM, TO, TM>(p, ph, acc, m0, o0, p.n * hw, hw, 0, wo, wm, kh, l32, smem);
}

// Style-scaled input for the low-resolution layers: out[n][i][p] = x[n][i][p] * s[n][i] (float4 when hw % 4 == 0).
__global__ __launch_bounds__(256) void xscale_kernel(const float* x, const float* s, float* out, int64_t hw,
                                                     int64_t planes) {
    const int64_t per = hw / 4;
    const int64_t total = per * planes;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < total; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t pl = v / per;
        const float sc = s[pl];
        float4 a = reinterpret_cast<const float4*>(x)[v];
        a.x *= sc; a.y *= sc; a.z *= sc; a.w *= sc;
        reinterpret_cast<float4*>(out)[v] = a;
    }
}

// Per-sample weights for the LDS-DMA kernel: out[n][row][o] = wk[row][o] * s[n][row % cin].
__global__ __launch_bounds__(256) void wscale_kernel(const float* wk, const float* s, float* out, int rows, int cin,
                                                     int cout, int n) {
    const int64_t per = (int64_t)rows * cout / 4;
    const int64_t total = per * n;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < total; v += (int64_t)gridDim.x * blockDim.x) {
        const int64_t nn = v / per;
        const int64_t e = (v - nn * per) * 4;
        const int row = (int)(e / cout);
        float4 w = *reinterpret_cast<const float4*>(wk + e);
        const float sc = s[nn * cin + row % cin];
        w.x *= sc; w.y *= sc; w.z *= sc; w.w *= sc;
        *reinterpret_cast<float4*>(out + nn * (int64_t)rows * cout + e) = w;
    }
}

// ---------------------------------------------------------------------------------------------------
// Phase-fused stride-2 transposed 3x3 conv (the up=2 layers' conv, conv2d_resample.py:125-138).
// T[o, 2a+py, 2b+px] = sum over the taps of phase (py,px) of W[o,i,ky,kx] * x[i, a-(ky-py)/2, b-(kx-px)/2].
// All 4 phases read x at one of 4 shifts {(0,0), (-1,0), (0,-1), (-1,-1)}; a workgroup owns a tile of
// super-pixels (a,b) in [0,H]x[0,W] and all 4 phases, so every shifted input tile is staged ONCE and
// feeds every phase that uses it (shift 0: 4 phases, shifts 1/2: 2, shift 3: 1 -> the 9 taps).
// K steps are (channel chunk, shift); accumulators: 4 phases x TO x TM blocks (128 registers).

struct ConvTParams {
    const float* w[4][4];  // [shift][phase] -> [cin][cout] weight slice (nullptr: phase unused)
};

template <int S>
struct ShiftPhases;  // phases (py*2+px) that read input shift S
template <> struct ShiftPhases<0> { static constexpr int n = 4; static constexpr int p[4] = {0, 1, 2, 3}; };
template <> struct ShiftPhases<1> { static constexpr int n = 2; static constexpr int p[4] = {0, 1, 0, 0}; };
template <> struct ShiftPhases<2> { static constexpr int n = 2; static constexpr int p[4] = {0, 2, 0, 0}; };
template <> struct ShiftPhases<3> { static constexpr int n = 1; static constexpr int p[4] = {0, 0, 0, 0}; };

__host__ __device__ constexpr int shift_nph(int s) { return s == 0 ? 4 : (s == 3 ? 1 : 2); }

template <int S, int TO, int TM, int BKT, int BO, int BM>
__device__ __forceinline__ void convt_mma(const float* Ws, const float* Xs, int wo, int wm, int kh, int l32,
                                          f32x16 (&acc)[4][TO][TM]) {
    constexpr int NP = ShiftPhases<S>::n;
#pragma unroll
    for (int k0 = 0; k0 < BKT; k0 += 4) {
        float af[2][NP][TO], bf[2][TM];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int kk = k0 + 2 * q + kh;
#pragma unroll
            for (int j = 0; j < TM; ++j) bf[q][j] = Xs[kk * BM + wm * TM * 32 + j * 32 + l32];
#pragma unroll
            for (int ph = 0; ph < NP; ++ph)
#pragma unroll
                for (int i = 0; i < TO; ++i) af[q][ph][i] = Ws[(ph * BKT + kk) * BO + wo * TO * 32 + i * 32 + l32];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int ph = 0; ph < NP; ++ph)
#pragma unroll
                for (int i = 0; i < TO; ++i)
#pragma unroll
                    for (int j = 0; j < TM; ++j)
                        acc[ShiftPhases<S>::p[ph]][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                            af[q][ph][i], bf[q][j], acc[ShiftPhases<S>::p[ph]][i][j], 0, 0, 0);
    }
}

template <int WO, int WM, int TO, int TM, int BKT>
__global__ __launch_bounds__(NT, 1) void convt_gemm_kernel(GemmParams p, ConvTParams q) {
    static_assert(WO * WM == 4, "4 waves");
    constexpr int BO = WO * TO * 32;
    constexpr int BM = WM * TM * 32;
    constexpr int XR = BKT * BM / NT;
    constexpr int WV = BKT * BO / 4;         // float4 vectors per phase weight tile
    constexpr int WPT = (WV + NT - 1) / NT;
    constexpr int TILE = BKT * (4 * BO + BM);
    static_assert(NT % BM == 0 && XR % 4 == 0, "thread->position map");
    __shared__ float smem[2 * TILE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wo = wave / WM, wm = wave % WM;
    const int gh = p.in_h + 1, gw = p.in_w + 1, hw_g = gh * gw;
    const int M = p.n * hw_g;
    const int m0 = blockIdx.x * BM;
    const int o0 = blockIdx.y * BO;
    const int split = blockIdx.z;
    const int cpk = p.cin / BKT;
    const int ks_total = 4 * cpk;
    const int ks_begin = (int)((int64_t)ks_total * split / p.nsplit);
    const int ks_end = (int)((int64_t)ks_total * (split + 1) / p.nsplit);

    const int ml = tid % BM, kr0 = (tid / BM) * XR;
    const int m = m0 + ml;
    const bool mvalid = m < M;
    int nn = 0, a = 0, b = 0;
    if (mvalid) {
        nn = m / hw_g;
        const int rem = m - nn * hw_g;
        a = rem / gw;
        b = rem - a * gw;
    }
    const int64_t in_hw = (int64_t)p.in_h * p.in_w;
    const float* xbase = p.x + (int64_t)nn * p.cin * in_hw + (int64_t)kr0 * in_hw;
    const bool has_s = p.s != nullptr;
    const float* swhere = has_s ? p.s + (int64_t)nn * p.cin + kr0 : p.x;

    float xr[XR];
    float4 sr[XR / 4];
    float4 wr[4][WPT];
    bool xok = false;

    auto load_step = [&](int ks) {
        const int c = ks >> 2, sh = ks & 3;
        const int ci0 = c * BKT;
        const int iy = a - (sh & 1), ix = b - ((sh >> 1) & 1);
        xok = mvalid && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w;
        const float* src = xbase + (int64_t)ci0 * in_hw + (xok ? (int64_t)iy * p.in_w + ix : 0);
#pragma unroll
        for (int r = 0; r < XR; ++r) xr[r] = src[r * in_hw];
#pragma unroll
        for (int r = 0; r < XR; r += 4) sr[r / 4] = *reinterpret_cast<const float4*>(swhere + (has_s ? ci0 + r : 0));
        const int nph = shift_nph(sh);
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {
            if (ph >= nph) break;  // uniform
            const int phase = sh == 0 ? ph : (sh == 1 ? (ph ? 1 : 0) : (sh == 2 ? (ph ? 2 : 0) : 0));
            const float* wbase = q.w[sh][phase];
#pragma unroll
            for (int t = 0; t < WPT; ++t) {
                int v = tid + t * NT;
                v = v < WV ? v : v - WV;
                const int wkk = v / (BO / 4), wc4 = v - wkk * (BO / 4);
                const int o = o0 + wc4 * 4;
                wr[ph][t] = *reinterpret_cast<const float4*>(wbase + (int64_t)(ci0 + wkk) * p.cout + (o < p.cout ? o : 0));
            }
        }
    };
    auto store_step = [&](int stage, int sh) {
        float* Ws = smem + stage * TILE;
        float* Xs = Ws + 4 * BKT * BO;
#pragma unroll
        for (int r = 0; r < XR; ++r) {
            const float4 sv = sr[r / 4];
            const float sc = has_s ? ((r & 3) == 0 ? sv.x : (r & 3) == 1 ? sv.y : (r & 3) == 2 ? sv.z : sv.w) : 1.f;
            Xs[(kr0 + r) * BM + ml] = xok ? xr[r] * sc : 0.f;
        }
        const int nph = shift_nph(sh);
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) {
            if (ph >= nph) break;
#pragma unroll
            for (int t = 0; t < WPT; ++t) {
                const int v = tid + t * NT;
                const int wkk = v / (BO / 4), wc4 = v - wkk * (BO / 4);
                float4 w = wr[ph][t];
                if (o0 + wc4 * 4 >= p.cout) w = make_float4(0.f, 0.f, 0.f, 0.f);
                if (v < WV) *reinterpret_cast<float4*>(&Ws[(ph * BKT + wkk) * BO + wc4 * 4]) = w;
            }
        }
    };

    f32x16 acc[4][TO][TM];
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int i = 0; i < TO; ++i)
#pragma unroll
            for (int j = 0; j < TM; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[ph][i][j][r] = 0.f;

    const int kh = lane >> 5, l32 = lane & 31;
    int stage = 0;
    if (ks_begin < ks_end) {
        load_step(ks_begin);
        store_step(0, ks_begin & 3);
    }
    __syncthreads();
    for (int ks = ks_begin; ks < ks_end; ++ks) {
        const bool more = ks + 1 < ks_end;
        if (more) load_step(ks + 1);
        const float* Ws = smem + stage * TILE;
        const float* Xs = Ws + 4 * BKT * BO;
        switch (ks & 3) {
            case 0: convt_mma<0, TO, TM, BKT, BO, BM>(Ws, Xs, wo, wm, kh, l32, acc); break;
            case 1: convt_mma<1, TO, TM, BKT, BO, BM>(Ws, Xs, wo, wm, kh, l32, acc); break;
            case 2: convt_mma<2, TO, TM, BKT, BO, BM>(Ws, Xs, wo, wm, kh, l32, acc); break;
            default: convt_mma<3, TO, TM, BKT, BO, BM>(Ws, Xs, wo, wm, kh, l32, acc); break;
        }
        if (more) store_step(stage ^ 1, (ks + 1) & 3);
        __syncthreads();
        stage ^= 1;
    }

    // epilogue: raw T (mode STORE) or this split's partial plane
    float* dst = p.nsplit > 1 ? p.y + (int64_t)split * p.split_stride : p.y;
    const int64_t plane = (int64_t)p.y_h * p.y_w;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
        const int mc = m0 + wm * TM * 32 + j * 32 + l32;
        if (mc >= M) continue;
        const int en = mc / hw_g;
        const int erem = mc - en * hw_g;
        const int ea = erem / gw;
        const int eb = erem - ea * gw;
#pragma unroll
        for (int i = 0; i < TO; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = o0 + wo * TO * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                if (o >= p.cout) continue;
                float* row0 = dst + ((int64_t)en * p.cout + o) * plane + (int64_t)(2 * ea) * p.y_w + 2 * eb;
                row0[0] = acc[0][i][j][r];
                if (eb < p.in_w) row0[1] = acc[1][i][j][r];
                if (ea < p.in_h) {
                    row0[p.y_w] = acc[2][i][j][r];
                    if (eb < p.in_w) row0[p.y_w + 1] = acc[3][i][j][r];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// Phase-fused stride-2 transposed 3x3 conv on LDS-DMA operands (the default for the up = 2 layers' conv).
// Same decomposition as convt_gemm_kernel -- a workgroup owns BM super-pixels (a, b) of the (H+1) x (W+1)
// grid and all 4 output phases, K steps are (channel chunk, input shift), and each staged shift tile feeds
// every phase that reads it (shift 0: 4 phases, shifts 1 / 2: 2, shift 3: 1 -> the 9 taps) -- but both
// operands go global -> LDS by DMA into a 2-stage ring as in conv_gemm_lds_kernel (no register staging, one
// barrier per step): the input slab by `buffer_load_dword ... lds` (lane = super-pixel, the buffer range check
// zero-fills the out-of-image shifts), the phases' weight slabs by `global_load_lds_dwordx4`.  Style scaling
// comes in the per-sample weights (wscale_kernel) or a prescaled input, as for the other LDS-DMA launches.
struct ConvTTaps {
    int tap[4][4];  // [shift][phase] -> tap index in phase `phase`'s packed weights (-1: phase unused)
};

template <int S>
__host__ __device__ constexpr int shift_phase(int j) {
    // j-th phase reading shift S (the ShiftPhases table as a constexpr function)
    return S == 0 ? j : (S == 1 ? (j ? 1 : 0) : (S == 2 ? (j ? 2 : 0) : 0));
}

template <int S, int TO, int TM, int BKT, int BO, int BM>
__device__ __forceinline__ void convt_lds_mma(const float* Ws, const float* Xs, int wo, int wm, int kh, int l32,
                                              f32x16 (&acc)[4][TO][TM]) {
    constexpr int NP = shift_nph(S);
    const float* wrow = Ws + kh * BO + wo * TO * 32 + l32;
    const float* xrow = Xs + kh * BM + wm * TM * 32 + l32;
    // software pipeline over the BKT / 2 K-pairs: the fragments of pair q + 1 are read under pair q's MFMAs
    float af[2][NP][TO], bf[2][TM];
    auto frag = [&](int q, int b) {
#pragma unroll
        for (int j = 0; j < TM; ++j) bf[b][j] = xrow[(2 * q) * BM + j * 32];
#pragma unroll
        for (int ph = 0; ph < NP; ++ph)
#pragma unroll
            for (int i = 0; i < TO; ++i) af[b][ph][i] = wrow[(ph * BKT + 2 * q) * BO + i * 32];
    };
    frag(0, 0);
#pragma unroll
    for (int q = 0; q < BKT / 2; ++q) {
        if (q + 1 < BKT / 2) frag(q + 1, (q + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ph = 0; ph < NP; ++ph)
#pragma unroll
            for (int i = 0; i < TO; ++i)
#pragma unroll
                for (int j = 0; j < TM; ++j)
                    acc[shift_phase<S>(ph)][i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                        af[q & 1][ph][i], bf[q & 1][j], acc[shift_phase<S>(ph)][i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int WO, int WM, int TO, int TM, int BKT>
__global__ __launch_bounds__(NT, 2) void convt_lds_kernel(GemmParams p, ConvTTaps tt) {
    static_assert(WO * WM == 4, "4 waves");
    constexpr int BO = WO * TO * 32;
    constexpr int BM = WM * TM * 32;
    constexpr int NCH = BM / 64;                 // 64-position chunks per input row
    static_assert(NCH >= 1 && NCH <= 4 && 4 % NCH == 0, "BM in {64,128,256}");
    constexpr int RSTEP = 4 / NCH;
    constexpr int XI = BKT * NCH / 4;            // input DMAs per wave per step
    constexpr int WSL = BKT * BO;                // floats of one phase's weight slab
    static_assert(WSL % 256 == 0, "weight slabs split into whole 1-KB DMAs");
    constexpr int TILE = BKT * BM + 4 * WSL;     // X slab + up to 4 phase slabs
    __shared__ __attribute__((aligned(16))) float smem[2 * TILE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wo = wave / WM, wm = wave % WM;
    const int gh = p.in_h + 1, gw = p.in_w + 1, hw_g = gh * gw;
    int tm = blockIdx.x, tn = blockIdx.y;
    if (p.ntn) {  // XCD-aware bijective tile order (see conv_gemm_lds_kernel)
        const int nwg = gridDim.x, orig = blockIdx.x;
        const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
        const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
        tm = wgid / p.ntn;
        tn = wgid - tm * p.ntn;
    }
    int M = p.n * hw_g;
    int m0 = tm * BM;
    if (p.per_sample) {  // per-sample weights: tiles restart at every image
        const int tps = (hw_g + BM - 1) / BM;
        const int nb = tm / tps;
        if (nb >= p.n) return;
        m0 = nb * hw_g + (tm - nb * tps) * BM;
        M = (nb + 1) * hw_g;
    }
    if (m0 >= M) return;
    const int o0 = tn * BO;
    const int split = blockIdx.z;
    const int cpk = p.cin / BKT;
    // split-K over whole channel chunks (each chunk = the 4 shift steps, unrolled below)
    const int c_begin = (int)((int64_t)cpk * split / p.nsplit);
    const int c_end = (int)((int64_t)cpk * (split + 1) / p.nsplit);
    const int ks_begin = 4 * c_begin, ks_end = 4 * c_end;

    const int cw = wave % NCH, r0 = wave / NCH;
    const int m = m0 + cw * 64 + lane;
    const bool mvalid = m < M;
    int nn = 0, a = 0, b = 0;
    if (mvalid) {
        nn = m / hw_g;
        const int rem = m - nn * hw_g;
        a = rem / gw;
        b = rem - a * gw;
    }
    const int in_hw = p.in_h * p.in_w;
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * in_hw * 4), 0x00020000);
    const int xvbase = nn * p.cin * in_hw * 4;
    const int wn = m0 / hw_g;  // the workgroup's sample (per-sample weights)

    auto issue = [&](int ks, int slot) {
        const int c = ks >> 2, sh = ks & 3;
        const int ci0 = c * BKT;
        const int iy = a - (sh & 1), ix = b - (sh >> 1);
        const bool ok = mvalid && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w;
        const int voff = ok ? xvbase + (iy * p.in_w + ix) * 4 : 0x7ffffff0;
        float* xs = smem + slot * TILE;
#pragma unroll
        for (int j = 0; j < XI; ++j) {
            const int row = r0 + RSTEP * j;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                xrsrc, (__attribute__((address_space(3))) void*)(xs + row * BM + cw * 64), 4, voff,
                (ci0 + row) * in_hw * 4, 0, 0);
        }
        float* ws = xs + BKT * BM;
        const int nph = shift_nph(sh);
        for (int j = wave; j < nph * (WSL / 256); j += 4) {
            const int pj = j / (WSL / 256);                 // which phase slab of this shift
            const int phase = sh == 0 ? pj : (sh == 1 ? (pj ? 1 : 0) : (sh == 2 ? (pj ? 2 : 0) : 0));
            const int f = (j - pj * (WSL / 256)) * 256 + lane * 4;
            const int row = f / BO, col = f - row * BO;
            const PhaseDev& q = p.ph[phase];
            const float* src = q.wk + (q.wstride ? (int64_t)wn * q.wstride : 0) +
                               ((int64_t)tt.tap[sh][phase] * p.cin + ci0 + row) * p.cout + o0 + col;
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(ws + pj * WSL + f - lane * 4),
                                             16, 0, 0);
        }
    };

    f32x16 acc[4][TO][TM];
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int i = 0; i < TO; ++i)
#pragma unroll
            for (int j = 0; j < TM; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[ph][i][j][r] = 0.f;

    const int kh = lane >> 5, l32 = lane & 31;
    if (ks_begin < ks_end) issue(ks_begin, 0);
    // slot of step ks = (ks - ks_begin) & 1 = ks & 1 (ks_begin is a multiple of 4): shifts 0 / 2 in slot 0,
    // shifts 1 / 3 in slot 1; the shift loop is unrolled so every step's phase set is a compile-time constant
    auto step = [&](auto S_, int ks) {
        constexpr int S = decltype(S_)::value;
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // step ks landed for every wave; the other slot is free
        asm volatile("" ::: "memory");
        if (ks + 1 < ks_end) issue(ks + 1, (S + 1) & 1);
        const float* Xs = smem + (S & 1) * TILE;
        convt_lds_mma<S, TO, TM, BKT, BO, BM>(Xs + BKT * BM, Xs, wo, wm, kh, l32, acc);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    for (int ks = ks_begin; ks < ks_end; ks += 4) {
        step(std::integral_constant<int, 0>{}, ks);
        step(std::integral_constant<int, 1>{}, ks + 1);
        step(std::integral_constant<int, 2>{}, ks + 2);
        step(std::integral_constant<int, 3>{}, ks + 3);
    }

    // epilogue: raw T (mode STORE) or this split's partial plane
    float* dst = p.nsplit > 1 ? p.y + (int64_t)split * p.split_stride : p.y;
    const int64_t plane = (int64_t)p.y_h * p.y_w;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
        const int mc = m0 + wm * TM * 32 + j * 32 + l32;
        if (mc >= M) continue;
        const int en = mc / hw_g;
        const int erem = mc - en * hw_g;
        const int ea = erem / gw;
        const int eb = erem - ea * gw;
#pragma unroll
        for (int i = 0; i < TO; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = o0 + wo * TO * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                float* row0 = dst + ((int64_t)en * p.cout + o) * plane + (int64_t)(2 * ea) * p.y_w + 2 * eb;
                row0[0] = acc[0][i][j][r];
                if (eb < p.in_w) row0[1] = acc[1][i][j][r];
                if (ea < p.in_h) {
                    row0[p.y_w] = acc[2][i][j][r];
                    if (eb < p.in_w) row0[p.y_w + 1] = acc[3][i][j][r];
                }
            }
        }
    }
}

// Split-bf16 form of convt_lds_kernel (the products as in conv_gemm_x3_kernel): per K step (16 channels, one input
// shift) the fp32 input slab [16][BM] and, for every phase reading that shift, its weight planes [3][2][BO][8] bf16;
// a wave splits each B fragment once and feeds it to every phase's A fragments.
template <int WO, int WM, int TO, int TM>
__global__ __launch_bounds__(NT, 2) void convt_x3_kernel(GemmParams p, ConvTTaps tt) {
    static_assert(WO * WM == 4, "4 waves");
    constexpr int BKT = 16;
    constexpr int BO = WO * TO * 32;
    constexpr int BM = WM * TM * 32;
    constexpr int NCH = BM / 64;
    static_assert(NCH >= 1 && NCH <= 4 && 4 % NCH == 0, "BM in {64,128,256}");
    constexpr int RSTEP = 4 / NCH;
    constexpr int XI = BKT * NCH / 4;
    constexpr int PB = 6 * BO * 16;              // bytes of one phase's planes per step
    static_assert(PB % 1024 == 0, "phase planes split into whole 1-KB DMAs");
    constexpr int XB = BKT * BM * 4;
    constexpr int STAGE = XB + 4 * PB;           // input slab + up to 4 phases' planes
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wo = wave / WM, wm = wave % WM;
    const int gh = p.in_h + 1, gw = p.in_w + 1, hw_g = gh * gw;
    int tm = blockIdx.x, tn = blockIdx.y;
    if (p.ntn) {
        const int nwg = gridDim.x, orig = blockIdx.x;
        const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
        const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
        tm = wgid / p.ntn;
        tn = wgid - tm * p.ntn;
    }
    int M = p.n * hw_g;
    int m0 = tm * BM;
    if (p.per_sample) {
        const int tps = (hw_g + BM - 1) / BM;
        const int nb = tm / tps;
        if (nb >= p.n) return;
        m0 = nb * hw_g + (tm - nb * tps) * BM;
        M = (nb + 1) * hw_g;
    }
    if (m0 >= M) return;
    const int o0 = tn * BO;
    const int split = blockIdx.z;
    const int cpk = p.cin / BKT;
    const int c_begin = (int)((int64_t)cpk * split / p.nsplit);
    const int c_end = (int)((int64_t)cpk * (split + 1) / p.nsplit);
    const int ks_begin = 4 * c_begin, ks_end = 4 * c_end;

    const int cw = wave % NCH, r0 = wave / NCH;
    const int m = m0 + cw * 64 + lane;
    const bool mvalid = m < M;
    int nn = 0, a = 0, b = 0;
    if (mvalid) {
        nn = m / hw_g;
        const int rem = m - nn * hw_g;
        a = rem / gw;
        b = rem - a * gw;
    }
    const int in_hw = p.in_h * p.in_w;
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * in_hw * 4), 0x00020000);
    const int xvbase = nn * p.cin * in_hw * 4;
    const int wn = m0 / hw_g;
    const int c16n = p.cin / 16;

    auto issue = [&](int ks, int slot) {
        const int c = ks >> 2, sh = ks & 3;
        const int ci0 = c * BKT;
        const int iy = a - (sh & 1), ix = b - (sh >> 1);
        const bool ok = mvalid && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w;
        const int voff = ok ? xvbase + (iy * p.in_w + ix) * 4 : 0x7ffffff0;
        char* st = smem + slot * STAGE;
        float* xs = reinterpret_cast<float*>(st);
#pragma unroll
        for (int j = 0; j < XI; ++j) {
            const int row = r0 + RSTEP * j;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                xrsrc, (__attribute__((address_space(3))) void*)(xs + row * BM + cw * 64), 4, voff,
                (ci0 + row) * in_hw * 4, 0, 0);
        }
        const int nph = shift_nph(sh);
        for (int j = wave; j < nph * (PB / 1024); j += 4) {
            const int pj = j / (PB / 1024);          // which phase of this shift
            const int phase = sh == 0 ? pj : (sh == 1 ? (pj ? 1 : 0) : (sh == 2 ? (pj ? 2 : 0) : 0));
            const int L = (j - pj * (PB / 1024)) * 64 + lane;
            const int run = L / BO, o = L - run * BO;
            const PhaseDev& q = p.ph[phase];
            const short* src = q.wx3 + (q.wx3_stride ? (int64_t)wn * q.wx3_stride : 0) +
                               ((((int64_t)tt.tap[sh][phase] * c16n + ci0 / 16) * 6 + run) * p.cout + o0 + o) * 8;
            __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(st + XB + j * 1024),
                                             16, 0, 0);
        }
    };

    f32x16 acc[4][TO][TM];
#pragma unroll
    for (int ph = 0; ph < 4; ++ph)
#pragma unroll
        for (int i = 0; i < TO; ++i)
#pragma unroll
            for (int j = 0; j < TM; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[ph][i][j][r] = 0.f;

    const int kh = lane >> 5, l32 = lane & 31;
    if (ks_begin < ks_end) issue(ks_begin, 0);
    auto step = [&](auto S_, int ks) {
        constexpr int S = decltype(S_)::value;
        constexpr int NP = shift_nph(S);
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* st = smem + (S & 1) * STAGE;
        const float* xcol = reinterpret_cast<const float*>(st) + wm * TM * 32 + l32;
        bf16x8 bt[TM][3];
#pragma unroll
        for (int j = 0; j < TM; ++j) {
            float xv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[e] = xcol[(8 * kh + e) * BM + j * 32];
            x3_split8(xv, bt[j]);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (ks + 1 < ks_end) issue(ks + 1, (S + 1) & 1);
#pragma unroll
        for (int pj = 0; pj < NP; ++pj) {
            const short* Wp = reinterpret_cast<const short*>(st + XB + pj * PB);
            bf16x8 at[TO][3];
#pragma unroll
            for (int i = 0; i < TO; ++i)
#pragma unroll
                for (int s = 0; s < 3; ++s)
                    at[i][s] = *reinterpret_cast<const bf16x8*>(Wp + (((s * 2 + kh) * BO) + wo * TO * 32 + i * 32 + l32) * 8);
#pragma unroll
            for (int i = 0; i < TO; ++i)
#pragma unroll
                for (int j = 0; j < TM; ++j)
                    acc[shift_phase<S>(pj)][i][j] = x3_mma(at[i], bt[j], acc[shift_phase<S>(pj)][i][j]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    for (int ks = ks_begin; ks < ks_end; ks += 4) {
        step(std::integral_constant<int, 0>{}, ks);
        step(std::integral_constant<int, 1>{}, ks + 1);
        step(std::integral_constant<int, 2>{}, ks + 2);
        step(std::integral_constant<int, 3>{}, ks + 3);
    }

    float* dst = p.nsplit > 1 ? p.y + (int64_t)split * p.split_stride : p.y;
    const int64_t plane = (int64_t)p.y_h * p.y_w;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
        const int mc = m0 + wm * TM * 32 + j * 32 + l32;
        if (mc >= M) continue;
        const int en = mc / hw_g;
        const int erem = mc - en * hw_g;
        const int ea = erem / gw;
        const int eb = erem - ea * gw;
#pragma unroll
        for (int i = 0; i < TO; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = o0 + wo * TO * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                float* row0 = dst + ((int64_t)en * p.cout + o) * plane + (int64_t)(2 * ea) * p.y_w + 2 * eb;
                row0[0] = acc[0][i][j][r];
                if (eb < p.in_w) row0[1] = acc[1][i][j][r];
                if (ea < p.in_h) {
                    row0[p.y_w] = acc[2][i][j][r];
                    if (eb < p.in_w) row0[p.y_w + 1] = acc[3][i][j][r];
                }
            }
        }
    }
}

// Does this 4-phase description match the polyphase stride-2 transposed 3x3 conv built by
// stylemc_amd.modconv.PackedConv (phase index py*2+px, taps at shifts {0,-1}^2)?  Fills the table.
bool convt_structure(int cin, int cout, int in_h, int in_w, int y_h, int y_w, const smc_conv_phase* ph, int nph,
                     const smc_conv_epilogue* epi, ConvTParams* q) {
    if (nph != 4 || y_h != 2 * in_h + 1 || y_w != 2 * in_w + 1) return false;
    if (epi && (epi->mode != SMC_EPI_STORE || epi->residual)) return false;
    ConvTParams t{};
    int count = 0;
    for (int k = 0; k < 4; ++k) {
        const int py = k >> 1, px = k & 1;
        const smc_conv_phase& f = ph[k];
        if (f.in_stride != 1 || f.out_sy != 2 || f.out_sx != 2 || f.out_oy != py || f.out_ox != px) return false;
        for (int tp = 0; tp < f.ntaps; ++tp) {
            const int dy = f.tap_dy[tp], dx = f.tap_dx[tp];
            if ((dy != 0 && dy != -1) || (dx != 0 && dx != -1)) return false;
            const int s = (dy == -1 ? 1 : 0) + (dx == -1 ? 2 : 0);
            if (t.w[s][k]) return false;
            t.w[s][k] = f.wk + (int64_t)tp * cin * cout;
            ++count;
        }
    }
    if (count != 9) return false;
    for (int s = 0; s < 4; ++s)
        for (int k = 0; k < 4; ++k) {
            const bool want = s == 0 || (s == 1 && (k == 0 || k == 1)) || (s == 2 && (k == 0 || k == 2)) || (s == 3 && k == 0);
            if (want != (t.w[s][k] != nullptr)) return false;
        }
    if (q) *q = t;
    return true;
}

// The register-staged fused kernel: only where the LDS-DMA one cannot run (inputs of 2 GiB or more), and
// only for 32 output channels (1 wave/SIMD, 128 accumulators: slower than the per-phase kernel on every
// wider layer, tools/bench_gemm.py).
bool convt_fusable(int cin, int cout, int in_h, int in_w, int y_h, int y_w, const smc_conv_phase* ph, int nph,
                   const smc_conv_epilogue* epi, ConvTParams* q) {
    return cout <= 32 && convt_structure(cin, cout, in_h, in_w, y_h, y_w, ph, nph, epi, q);
}

struct ConvTCfg {
    int bo, bm, id;
};

ConvTCfg convt_cfg(int cout) {
    if (cout % 128 == 0) return {128, 64, 0};
    if (cout % 64 == 0) return {64, 128, 1};
    // 32 x 128 tile: 159 VGPR + 80 AGPR -> 2 workgroups per CU (the 32 x 256 tile's 256 + 160 allow one):
    // 763 -> 620 us on the r = 1024 conv0 (tools/bench_gemm.py)
    return {32, 128, 3};
}

int plan_split_convt(int n, int cin, int cout, int in_h, int in_w) {
    const ConvTCfg c = convt_cfg(cout);
    const int64_t M = (int64_t)smc::plan_batch(n) * (in_h + 1) * (in_w + 1);
    const int64_t blocks = smc::ceil_div(M, c.bm) * smc::ceil_div(cout, c.bo);
    const int ks = 4 * (cin / BK);
    const int64_t target = 2LL * smc::device_cu_count();
    if (blocks >= target) return 1;
    int s = (int)smc::ceil_div(target, blocks > 0 ? blocks : 1);
    int cap = ks / 4;
    if (cap > 16) cap = 16;
    if (s > cap) s = cap;
    return s < 1 ? 1 : s;
}

// convt_lds_kernel: the 4-phase stride-2 transposed conv of modconv.PackedConv (epilogue STORE: the blur +
// modconv epilogue follow in smc_modconv_blur_act_f32), 32-bit input offsets, whole column tiles.
struct ConvTL {
    int bo, bm, id;
};

bool convt_lds_plan(int n, int cin, int cout, int in_h, int in_w, int y_h, int y_w, const smc_conv_phase* ph, int nph,
                    const smc_conv_epilogue* epi, ConvTTaps* tt, ConvTL* cfg) {
    ConvTParams q{};
    if (!convt_structure(cin, cout, in_h, in_w, y_h, y_w, ph, nph, epi, &q)) return false;
    // measured (tools/bench_gemm.py, batch 4): r = 1024 (64 -> 32 ch) 615 -> 413 us, r = 512 (128 -> 64) 427 ->
    // 416 us against the per-phase kernel; from 128 output channels up the per-phase kernel stays ahead
    // (r = 256: 364 vs 434 us; the 4 phases' accumulators cost the wide tiles their occupancy)
    if (cin % 16 != 0 || cout % 32 != 0 || cout > 64 || (int64_t)n * cin * in_h * in_w * 4 >= (1LL << 31)) return false;
    if (tt) {
        for (int sh = 0; sh < 4; ++sh)
            for (int k = 0; k < 4; ++k)
                tt->tap[sh][k] = q.w[sh][k] ? (int)((q.w[sh][k] - ph[k].wk) / ((int64_t)cin * cout)) : -1;
    }
    if (cfg) *cfg = cout % 64 == 0 ? ConvTL{64, 128, 1} : ConvTL{32, 128, 0};
    return true;
}

int plan_split_convt_lds(int n, int cin, int cout, int in_h, int in_w, const ConvTL& c, bool per_sample) {
    n = smc::plan_batch(n);
    const int64_t hw_g = (int64_t)(in_h + 1) * (in_w + 1);
    const int64_t mt = per_sample ? n * smc::ceil_div(hw_g, c.bm) : smc::ceil_div(n * hw_g, c.bm);
    const int64_t blocks = mt * (cout / c.bo);
    const int64_t target = 2LL * smc::device_cu_count();
    if (blocks >= target) return 1;
    int s = (int)smc::ceil_div(target, blocks > 0 ? blocks : 1);
    int cap = (cin / 16) / 2;   // whole channel chunks per split, at least two
    if (cap > 16) cap = 16;
    if (s > cap) s = cap;
    return s < 1 ? 1 : s;
}

struct Cfg {
    int bo, bm;
};

int pick_cfg(int cout, Cfg* c) {
    // 32/64-channel layers: 128-position tiles (twice the workgroups of the 256-position ones, half the LDS
    // per workgroup): r = 512 conv0 451 -> 424 us, r = 1024 bwd conv0 426 -> 396 us, the rest within 1 %
    // (tools/bench_gemm.py)
    if (cout % 128 == 0) { *c = {128, 128}; return 0; }
    if (cout % 64 == 0) { *c = {64, 128}; return 5; }
    if (cout % 32 == 0 || cout == 16) { *c = {32, 128}; return 4; }  // cout 16: half-empty tile, masked
    return -1;
}

// Shared by the workspace query and the launch so both agree on the split.
int plan_split(int n, int cin, int cout, const smc_conv_phase* ph, int nph, const Cfg& c, int target_per_cu = 2) {
    int64_t blocks = 0;
    int min_ks = 1 << 30;
    for (int i = 0; i < nph; ++i) {
        const int64_t M = (int64_t)smc::plan_batch(n) * ph[i].out_h * ph[i].out_w;
        blocks += smc::ceil_div(M, c.bm) * smc::ceil_div(cout, c.bo);
        const int ks = ph[i].ntaps * (cin / BK);
        if (ks < min_ks) min_ks = ks;
    }
    const int64_t target = (int64_t)target_per_cu * smc::device_cu_count();
    if (blocks >= target) return 1;
    int s = (int)smc::ceil_div(target, blocks > 0 ? blocks : 1);
    int cap = min_ks / 4;
    if (cap > 16) cap = 16;
    if (s > cap) s = cap;
    return s < 1 ? 1 : s;
}

// The LDS-DMA kernel covers full column tiles, 32-bit input offsets and (for a style-scaled input)
// workgroups that never straddle two images.  `scaled_ok` reports the latter.
bool lds_shape_ok(int n, int cin, int cout, int in_h, int in_w, const smc_conv_phase* ph, int nph, const Cfg& c,
                  bool* scaled_ok) {
    bool so = true;
    for (int i = 0; i < nph; ++i) so = so && ((int64_t)ph[i].out_h * ph[i].out_w) % c.bm == 0;
    if (scaled_ok) *scaled_ok = so;
    return cout % c.bo == 0 && cin % BK == 0 && (int64_t)n * cin * in_h * in_w * 4 < (1LL << 31);
}

// conv_row_kernel shapes: one 9-tap phase covering {-1,0,1}^2 that maps the input grid onto an equal output
// grid (3x3 stride-1 'same'), rows of whole BM-position segments, cin % 16 == 0, cout a multiple of the tile.
bool row_ok(int n, int cin, int cout, int in_h, int in_w, int y_h, int y_w, const smc_conv_phase* ph, int nph,
            const Cfg& c, RowTaps* rt) {
    if (nph != 1 || cin % 16 != 0 || cout % c.bo != 0 || in_w % c.bm != 0 || in_w % 4 != 0) return false;
    const smc_conv_phase& q = ph[0];
    if (q.ntaps != 9 || q.in_stride != 1 || q.out_h != in_h || q.out_w != in_w || y_h != in_h || y_w != in_w ||
        q.out_oy != 0 || q.out_ox != 0 || q.out_sy != 1 || q.out_sx != 1)
        return false;
    int seen = 0;
    for (int t = 0; t < 9; ++t) {
        const int dy = q.tap_dy[t], dx = q.tap_dx[t];
        if (dy < -1 || dy > 1 || dx < -1 || dx > 1) return false;
        const int bit = 1 << ((dy + 1) * 3 + dx + 1);
        if (seen & bit) return false;
        seen |= bit;
        if (rt) rt->t[dy + 1][dx + 1] = t;
    }
    return seen == 511 && (int64_t)n * cin * in_h * in_w * 4 < (1LL << 31);
}

// floats of per-sample weights (n x sum_p taps_p * cin * cout), 64-float aligned; split-bf16 planes (three bf16
// terms per weight) take 1.5x that
bool phases_x3(const smc_conv_phase* ph, int nph) {
    for (int i = 0; i < nph; ++i)
        if (!ph[i].wk_x3) return false;
    return nph > 0;
}

int64_t wsample_floats(int n, int cin, int cout, const smc_conv_phase* ph, int nph) {
    int64_t t = 0;
    for (int i = 0; i < nph; ++i) t += (int64_t)ph[i].ntaps * cin * cout;
    if (phases_x3(ph, nph)) t = (t * 3 + 1) / 2;
    return ((t * n + 63) / 64) * 64;
}

// LDS ring depth: two stages (32-41 KB of LDS -> 3-4 workgroups per CU) beat three or four on every layer
// (measured on MI355X, tools/bench_gemm.py, FFHQ-1024 shapes, batch 4): the occupancy hides the DMA latency
// better than a deeper ring (total 12.6 vs 13.0 / 13.3 ms, register-staged kernel 13.2 ms).
// BK = 32 for the wide tile on the long-K 512-channel layers.
bool lds_bk32(int cfg, int cin) { return cfg == 0 && cin % 32 == 0 && cin >= 512; }

// 64x64 tile (4 waves of one 32x32 block each) for GEMMs whose cout-based tile leaves most CUs idle (the
// IR-SE50 7..28-px stages, the synthesis 4..32-px blocks): 4x the workgroups before any split-K, so fewer
// and shorter partial planes.  LDS-DMA kernel only; SMC_NO_SMALL_TILE=1 disables (A/B knob).
bool small_tile_ok(int n, int cin, int cout, int in_h, int in_w, const smc_conv_phase* ph, int nph, bool has_s,
                   const Cfg& base) {
    if (cout % 64 != 0) return false;
    int64_t blocks = 0;
    int taps_all = 0;
    for (int i = 0; i < nph; ++i) {
        blocks += smc::ceil_div((int64_t)smc::plan_batch(n) * ph[i].out_h * ph[i].out_w, base.bm) *
                  smc::ceil_div(cout, base.bo);
        taps_all += ph[i].ntaps;
    }
    // threshold measured on the FFHQ-1024 / IR-SE50 shapes (tools/bench_gemm.py, tools/prof_irse.py): the
    // 128x128 tile with split-K stays ahead from 128 tiles up (r = 32 conv1); below that the 64x64 tile wins on
    // the sum (synthesis GEMMs 12.14 ms at 128 vs 12.30 at 256; IR-SE50 pair 4.85 vs 5.06 ms at 32)
    if (blocks >= 128) return false;
    const Cfg sm{64, 64};
    bool scaled_ok = false;
    if (!lds_shape_ok(n, cin, cout, in_h, in_w, ph, nph, sm, &scaled_ok)) return false;
    return !has_s || scaled_ok || (int64_t)taps_all * cout <= (int64_t)in_h * in_w;
}

// Input prescale (x * s into the workspace, then the shared-weight GEMM) replaces the per-sample weights
// where the input is the smaller of the two: the 4..64-px layers (n*cin*hw < n*taps*cin*cout), which
// otherwise write n copies of a 512x512x9 weight tensor (37.7 MB at n = 4) or fall back to the
// register-staged kernel.  Returns the floats to reserve (0: not a prescale shape); stride-1 phases
// only, the phase output images bounding the input image (3x3 same conv, 4-phase transposed conv).
int64_t prescale_floats(int n, int cin, int cout, const smc_conv_phase* ph, int nph) {
    int64_t hw = 0;
    int taps_all = 0;
    for (int i = 0; i < nph; ++i) {
        if (ph[i].in_stride != 1) return 0;
        hw = std::max<int64_t>(hw, (int64_t)ph[i].out_h * ph[i].out_w);
        taps_all += ph[i].ntaps;
    }
    return hw <= (int64_t)taps_all * cout ? (((int64_t)n * cin * hw + 63) / 64) * 64 : 0;
}

int validate(const float* x, int n, int cin, int in_h, int in_w, float* y, int cout, int y_h, int y_w,
             const smc_conv_phase* phases, int nphases) {
    SMC_CHECK(x && y && phases, "smc_conv_gemm_f32: null pointer");
    SMC_CHECK(n >= 1 && in_h >= 1 && in_w >= 1 && y_h >= 1 && y_w >= 1, "smc_conv_gemm_f32: bad shape");
    SMC_CHECK(nphases >= 1 && nphases <= 4, "smc_conv_gemm_f32: 1..4 phases (got %d)", nphases);
    if (cin % BK != 0) {
        smc::set_error("smc_conv_gemm_f32: cin=%d must be a multiple of %d", cin, BK);
        return SMC_ERR_UNSUPPORTED;
    }
    Cfg c;
    if (pick_cfg(cout, &c) < 0) {
        smc::set_error("smc_conv_gemm_f32: cout=%d must be 16 or a multiple of 32", cout);
        return SMC_ERR_UNSUPPORTED;
    }
    for (int i = 0; i < nphases; ++i) {
        const smc_conv_phase& q = phases[i];
        SMC_CHECK(q.ntaps >= 1 && q.ntaps <= 9, "smc_conv_gemm_f32: phase %d ntaps=%d", i, q.ntaps);
        SMC_CHECK(q.in_stride >= 1 && q.out_h >= 1 && q.out_w >= 1 && q.out_sy >= 1 && q.out_sx >= 1,
                  "smc_conv_gemm_f32: phase %d bad geometry", i);
        SMC_CHECK(q.out_oy >= 0 && q.out_ox >= 0 && q.out_oy + q.out_sy * (q.out_h - 1) < y_h &&
                      q.out_ox + q.out_sx * (q.out_w - 1) < y_w,
                  "smc_conv_gemm_f32: phase %d writes outside y", i);
        SMC_CHECK(q.wk != nullptr && (reinterpret_cast<uintptr_t>(q.wk) & 15) == 0,
                  "smc_conv_gemm_f32: phase %d weights must be 16-B aligned", i);
    }
    return SMC_OK;
}

}  // namespace

namespace {

// Split-K target of the IR-SE50 executor's GEMMs (TAG 1), in workgroups per CU: its 7..28-px stages are
// latency-bound chains of small GEMMs where more, shorter splits pay alone (tools/prof_irse.py, IR-SE50 pair
// fwd(8) + bwd(4): 2 -> 4.34 ms, 4 -> 4.16; 1 -> 4.99) -- but in the pipelined step, beside the CLIP tower on the
// main stream, fewer splits leave the main stream more of the chip: 2 beat 4 in all 7 rounds of two interleaved
// A/Bs (+0.5 %).  1 beat 2 in all 7 rounds of two more (+0.8 % and +1.6 %) but moves the IR-SE50 input gradient of
// the one-face fp64 test to 2.9e-3 of its max (the bound is 1e-3 there: the reference's fp32 path is 1e-6 away), so
// it is not used (profiles/r06/irse_aux_split_ab/).
#ifndef SMC_AUX_SPLIT_PER_CU
#define SMC_AUX_SPLIT_PER_CU 2
#endif
constexpr int kSplitPerCuAux = SMC_AUX_SPLIT_PER_CU;

int64_t workspace_size_impl(int n, int cin, int cout, int y_h, int y_w, const smc_conv_phase* phases, int nphases,
                            int split_per_cu) {
    Cfg c;
    if (pick_cfg(cout, &c) < 0 || cin % BK != 0 || nphases < 1 || nphases > 4 || !phases) return 0;
    int s;
    ConvTL tl;
    if (nphases == 4 && y_h % 2 == 1 && y_w % 2 == 1 &&
        convt_lds_plan(n, cin, cout, (y_h - 1) / 2, (y_w - 1) / 2, y_h, y_w, phases, nphases, nullptr, nullptr, &tl))
        s = std::max(plan_split_convt_lds(n, cin, cout, (y_h - 1) / 2, (y_w - 1) / 2, tl, true),
                     plan_split_convt_lds(n, cin, cout, (y_h - 1) / 2, (y_w - 1) / 2, tl, false));
    else if (nphases == 4 && y_h % 2 == 1 && y_w % 2 == 1 &&
             convt_fusable(cin, cout, (y_h - 1) / 2, (y_w - 1) / 2, y_h, y_w, phases, nphases, nullptr, nullptr))
        s = plan_split_convt(n, cin, cout, (y_h - 1) / 2, (y_w - 1) / 2);
    else
        s = plan_split(n, cin, cout, phases, nphases, c, split_per_cu);
    if (cout % 64 == 0) s = std::max(s, plan_split(n, cin, cout, phases, nphases, Cfg{64, 64}, split_per_cu));  // small tile
    int64_t bytes = s > 1 ? (int64_t)s * n * cout * y_h * y_w * (int64_t)sizeof(float) : 0;
    // the LDS-DMA kernel's per-sample weights when the input is style-scaled (the query does not know
    // whether it will be: reserve whenever the shape qualifies)
    bool scaled_ok = false;
    // (input size 1x1: the query reserves for a superset of the launches that use the area)
    const int64_t pre = prescale_floats(n, cin, cout, phases, nphases);
    if (lds_shape_ok(n, cin, cout, 1, 1, phases, nphases, c, &scaled_ok) || pre > 0)
        bytes = ((bytes + 255) / 256) * 256 +
                std::max(wsample_floats(n, cin, cout, phases, nphases), pre) * (int64_t)sizeof(float);
    return bytes;
}

}  // namespace

SMC_API int64_t smc_conv_gemm_workspace_size(int n, int cin, int cout, int y_h, int y_w, const smc_conv_phase* phases,
                                             int nphases) {
    return workspace_size_impl(n, cin, cout, y_h, y_w, phases, nphases, 2);
}

namespace {

// whether the last conv_gemm_impl call of this thread launched split-bf16 products (smc_conv_gemm_last_x3)
thread_local int g_last_x3 = 0;

int conv_gemm_impl(const float* x, int n, int cin, int in_h, int in_w, float* y, int cout, int y_h, int y_w,
                   const smc_conv_phase* phases, int nphases, const float* s_in, const smc_conv_epilogue* epi,
                   float* workspace, int64_t workspace_bytes, void* stream, int tag) {
    g_last_x3 = 0;
    int rc = validate(x, n, cin, in_h, in_w, y, cout, y_h, y_w, phases, nphases);
    if (rc != SMC_OK) return rc;
    Cfg c;
    int cfg = pick_cfg(cout, &c);
    ConvTParams ctp{};
    ConvTTaps ctt{};
    ConvTL tl{};
    const bool x3 = phases_x3(phases, nphases);  // split-bf16 products (the caller passed wk_x3 planes)
    const bool convt_lds = convt_lds_plan(n, cin, cout, in_h, in_w, y_h, y_w, phases, nphases, epi, &ctt, &tl);
    const bool fused_t = !convt_lds && convt_fusable(cin, cout, in_h, in_w, y_h, y_w, phases, nphases, epi, &ctp);
    const int64_t pre_fl = prescale_floats(n, cin, cout, phases, nphases);
    const bool prescale = s_in && !fused_t && pre_fl > 0 && (int64_t)n * cin * in_h * in_w <= pre_fl &&
                          (in_h * in_w) % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    const float* s_prescale = s_in;
    if (prescale) s_in = nullptr;  // the GEMM reads x * s from the workspace with the shared weights
    if (!fused_t && !convt_lds && small_tile_ok(n, cin, cout, in_h, in_w, phases, nphases, s_in != nullptr, c)) {
        cfg = 3;
        c = Cfg{64, 64};
    }
    // split-bf16 wide tiles (conv_gemm_x3_kernel AS): 256 output channels where that grid fills the chip unsplit, for
    // shared weights only.  Measured (profiles/r05/x3_wide/, tools/bench_gemm.py): the r = 256 stride-2 data gradient
    // 226.3 -> 215.6 us; the style-scaled r = 128 transposed conv0 (per-sample weights) 259.9 -> 265.2, so not there.
    if (SMC_X3_WIDE && x3 && !tag && !s_in && cfg == 0 && !fused_t && !convt_lds && cout % 256 == 0 &&
        plan_split(n, cin, cout, phases, nphases, Cfg{256, 128}) == 1 &&
        lds_shape_ok(n, cin, cout, in_h, in_w, phases, nphases, Cfg{256, 128}, nullptr)) {
        cfg = 6;
        c = Cfg{256, 128};
    }
    const bool t_per_sample = convt_lds && s_in && ((int64_t)(in_h + 1) * (in_w + 1)) % tl.bm != 0;
    const int nsplit = convt_lds ? plan_split_convt_lds(n, cin, cout, in_h, in_w, tl, t_per_sample)
                                 : fused_t ? plan_split_convt(n, cin, cout, in_h, in_w)
                                           : plan_split(n, cin, cout, phases, nphases, c, tag ? kSplitPerCuAux : 2);
    const int64_t plane_elems = (int64_t)n * cout * y_h * y_w;
    if (nsplit > 1) {
        const int64_t need = nsplit * plane_elems * (int64_t)sizeof(float);
        SMC_CHECK(workspace && workspace_bytes >= need, "smc_conv_gemm_f32: workspace %lld < %lld bytes",
                  (long long)workspace_bytes, (long long)need);
    }
    if (prescale) {
        // x * s after the split-K partials (the query reserved max(per-sample weights, prescaled input))
        const int64_t part = nsplit > 1 ? ((nsplit * plane_elems * (int64_t)sizeof(float) + 255) / 256) * 256 : 0;
        const int64_t need = part + pre_fl * (int64_t)sizeof(float);
        SMC_CHECK(workspace && workspace_bytes >= need, "smc_conv_gemm_f32: workspace %lld < %lld bytes",
                  (long long)workspace_bytes, (long long)need);
        float* xs = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + part);
        const int64_t planes = (int64_t)n * cin, hw = (int64_t)in_h * in_w;
        hipLaunchKernelGGL(xscale_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(planes * hw / 4, 256), 4096)),
                           dim3(256), 0, smc::as_stream(stream), x, s_prescale, xs, hw, planes);
        rc = smc::check_launch("smc_conv_gemm_f32 (prescaled input)");
        if (rc != SMC_OK) return rc;
        x = xs;
    }
    GemmParams p{};
    p.x = x; p.n = n; p.cin = cin; p.in_h = in_h; p.in_w = in_w;
    p.y = nsplit > 1 ? workspace : y;
    p.cout = cout; p.y_h = y_h; p.y_w = y_w;
    p.nphases = nphases;
    int64_t max_m = 0;
    for (int i = 0; i < nphases; ++i) {
        const smc_conv_phase& q = phases[i];
        PhaseDev& d = p.ph[i];
        d.ntaps = q.ntaps;
        for (int t = 0; t < 9; ++t) { d.dy[t] = q.tap_dy[t]; d.dx[t] = q.tap_dx[t]; }
        d.in_stride = q.in_stride; d.out_h = q.out_h; d.out_w = q.out_w;
        d.out_oy = q.out_oy; d.out_ox = q.out_ox; d.out_sy = q.out_sy; d.out_sx = q.out_sx;
        d.wk = q.wk;
        d.wx3 = reinterpret_cast<const short*>(q.wk_x3);
        d.wx3_stride = 0;
        const int64_t M = (int64_t)n * q.out_h * q.out_w;
        if (M > max_m) max_m = M;
    }
    SMC_CHECK(max_m < (1LL << 31), "smc_conv_gemm_f32: too many positions");
    p.s = s_in;
    smc_conv_epilogue e{};
    e.mode = SMC_EPI_STORE; e.act = SMC_ACT_LINEAR; e.gain = 1.f; e.clamp = -1.f;
    if (epi) e = *epi;
    p.mode = e.mode; p.d = e.d; p.noise = e.noise; p.noise_nstride = e.noise_nstride;
    p.noise_strength = e.noise_strength; p.bias = e.bias; p.act = e.act; p.alpha = e.alpha; p.gain = e.gain;
    p.clamp = e.clamp; p.u_save = e.u_save;
    p.ext = smc::epi_ext(epi);
    if ((e.mode == SMC_EPI_PRELU || e.mode == SMC_EPI_PRELU_GRAD) && !e.alpha_c) {
        smc::set_error("smc_conv_gemm_f32: PReLU epilogue needs alpha_c");
        return SMC_ERR_INVALID;
    }
    SMC_CHECK(e.mode != SMC_EPI_PRELU_GRAD || e.act_ref, "smc_conv_gemm_f32: PRELU_GRAD needs act_ref");
    SMC_CHECK(e.mode >= SMC_EPI_STORE && e.mode <= SMC_EPI_AFFINE, "smc_conv_gemm_f32: bad epilogue mode %d", e.mode);
    p.nsplit = nsplit;
    p.split_stride = plane_elems;

    hipStream_t st = smc::as_stream(stream);
    // per-sample weights W[t][i][o] * s[n][i], [phase][n][taps*cin][cout], after the split-K partials
    auto make_wsample = [&]() -> int {
        const int64_t part = nsplit > 1 ? ((nsplit * plane_elems * (int64_t)sizeof(float) + 255) / 256) * 256 : 0;
        const int64_t need = part + wsample_floats(n, cin, cout, phases, nphases) * (int64_t)sizeof(float);
        SMC_CHECK(workspace && workspace_bytes >= need, "smc_conv_gemm_f32: workspace %lld < %lld bytes",
                  (long long)workspace_bytes, (long long)need);
        float* wsamp = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + part);
        if (x3) {  // the per-sample weights W * s as split-bf16 planes, [phase][n][planes of one sample]
            short* wp = reinterpret_cast<short*>(wsamp);
            int64_t off = 0;
            for (int i = 0; i < nphases; ++i) {
                const int64_t per = (int64_t)phases[i].ntaps * cin * cout;
                hipLaunchKernelGGL(x3_weights_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(per * n, 256), 4096)),
                                   dim3(256), 0, st, phases[i].wk, s_in, wp + off, phases[i].ntaps, cin, cout, n);
                p.ph[i].wx3 = wp + off;
                p.ph[i].wx3_stride = per * 3;
                off += per * 3 * n;
            }
            return smc::check_launch("smc_conv_gemm_f32 (per-sample split weights)");
        }
        int64_t off = 0;
        for (int i = 0; i < nphases; ++i) {
            const int rows = phases[i].ntaps * cin;
            const int64_t tot4 = (int64_t)rows * cout / 4 * n;
            hipLaunchKernelGGL(wscale_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(tot4, 256), 4096)),
                               dim3(256), 0, st, phases[i].wk, s_in, wsamp + off, rows, cin, cout, n);
            p.ph[i].wk = wsamp + off;
            p.ph[i].wstride = (int64_t)rows * cout;
            off += (int64_t)rows * cout * n;
        }
        return smc::check_launch("smc_conv_gemm_f32 (per-sample weights)");
    };
    if (convt_lds) {
        if (s_in) {
            rc = make_wsample();
            if (rc != SMC_OK) return rc;
        }
        p.s = nullptr;
        const int64_t hw_g = (int64_t)(in_h + 1) * (in_w + 1);
        const int64_t mt = t_per_sample ? n * smc::ceil_div(hw_g, tl.bm) : smc::ceil_div(n * hw_g, tl.bm);
        p.per_sample = t_per_sample ? 1 : 0;
        p.ntn = cout / tl.bo;
        dim3 g((unsigned)(mt * p.ntn), 1, (unsigned)nsplit);
        g_last_x3 = x3 ? 1 : 0;
        if (x3 && tl.id == 1 && SMC_X3_WO1) hipLaunchKernelGGL((convt_x3_kernel<1, 4, 2, 1>), g, dim3(NT), 0, st, p, ctt);
        else if (x3 && tl.id == 1) hipLaunchKernelGGL((convt_x3_kernel<2, 2, 1, 2>), g, dim3(NT), 0, st, p, ctt);
        else if (x3) hipLaunchKernelGGL((convt_x3_kernel<1, 4, 1, 1>), g, dim3(NT), 0, st, p, ctt);
        else if (tl.id == 1) hipLaunchKernelGGL((convt_lds_kernel<2, 2, 1, 2, 16>), g, dim3(NT), 0, st, p, ctt);
        else hipLaunchKernelGGL((convt_lds_kernel<1, 4, 1, 1, 16>), g, dim3(NT), 0, st, p, ctt);
        rc = smc::check_launch("smc_conv_gemm_f32 (fused transposed conv, LDS-DMA)");
        if (rc != SMC_OK || nsplit == 1) return rc;
        return smc_modconv_epilogue_f32(workspace, nsplit, plane_elems, y, n, cout, y_h, y_w, &e, stream);
    }
    if (fused_t) {
        const ConvTCfg tc = convt_cfg(cout);
        const int64_t M = (int64_t)n * (in_h + 1) * (in_w + 1);
        dim3 g((unsigned)smc::ceil_div(M, tc.bm), (unsigned)smc::ceil_div(cout, tc.bo), (unsigned)nsplit);
        if (tc.id == 0) hipLaunchKernelGGL((convt_gemm_kernel<2, 2, 2, 1, 16>), g, dim3(NT), 0, st, p, ctp);
        else if (tc.id == 1) hipLaunchKernelGGL((convt_gemm_kernel<1, 4, 2, 1, 16>), g, dim3(NT), 0, st, p, ctp);
        else if (tc.id == 3) hipLaunchKernelGGL((convt_gemm_kernel<1, 4, 1, 1, 16>), g, dim3(NT), 0, st, p, ctp);
        else hipLaunchKernelGGL((convt_gemm_kernel<1, 4, 1, 2, 16>), g, dim3(NT), 0, st, p, ctp);
        rc = smc::check_launch("smc_conv_gemm_f32 (fused transposed conv)");
        if (rc != SMC_OK || nsplit == 1) return rc;
        return smc_modconv_epilogue_f32(workspace, nsplit, plane_elems, y, n, cout, y_h, y_w, &e, stream);
    }
    dim3 grid((unsigned)smc::ceil_div(max_m, c.bm), (unsigned)smc::ceil_div(cout, c.bo), (unsigned)(nphases * nsplit));
    bool scaled_ok = false;
    // per-sample tiling pays where the per-sample weights are small next to the input planes (the
    // high-resolution conv0 layers); on the 512-channel low-resolution layers writing n weight copies
    // costs more than the register-staged kernel's in-loop scaling (tools/bench_gemm.py)
    int taps_all = 0;
    for (int i = 0; i < nphases; ++i) taps_all += phases[i].ntaps;
    const bool small_w = (int64_t)taps_all * cout <= (int64_t)in_h * in_w;
    if (lds_shape_ok(n, cin, cout, in_h, in_w, phases, nphases, c, &scaled_ok) && (!s_in || scaled_ok || small_w)) {
        if (s_in && !scaled_ok) {
            // per-sample tiling: grid.x = n x (tiles of the largest phase image)
            int64_t tps = 0;
            for (int i = 0; i < nphases; ++i)
                tps = std::max<int64_t>(tps, smc::ceil_div((int64_t)phases[i].out_h * phases[i].out_w, c.bm));
            grid.x = (unsigned)(tps * n);
            p.per_sample = 1;
        }
        if (s_in) {
            rc = make_wsample();
            if (rc != SMC_OK) return rc;
        }
        p.s = nullptr;
        // XCD-aware tile order: one grid dimension, column tiles fastest (see conv_gemm_lds_kernel)
        p.ntn = (int)grid.y;
        grid.x *= grid.y;
        grid.y = 1;
        RowTaps rt{};
        if (x3) {
            // 32-channel K steps wherever the channels allow (two 16-channel chunks per barrier, the second's reads and
            // split under the first's MFMAs)
            const bool k32 = cfg == 0 && cin % 32 == 0;
            // 32-channel K steps for the narrow tiles too (A/B knob SMC_X3_K32_SMALL: half the barriers per FLOP)
            const bool k32s = SMC_X3_K32_SMALL && cin % 32 == 0;
            g_last_x3 = cfg == 6 ? 2 : 1;
            if (cfg == 6) hipLaunchKernelGGL((conv_gemm_x3_kernel<1, 4, 8, 1, 16, 2, 0, true>), grid, dim3(NT), 0, st, p);
            else if (SMC_X3_WO1 && SMC_X3_WO1_K16 && cfg == 0 && !tag) hipLaunchKernelGGL((conv_gemm_x3_kernel<1, 4, 4, 1, 16>), grid, dim3(NT), 0, st, p);
            else if (SMC_X3_WO1 && SMC_X3_WO1_K16 && cfg == 5 && !tag) hipLaunchKernelGGL((conv_gemm_x3_kernel<1, 4, 2, 1, 16>), grid, dim3(NT), 0, st, p);
            else if (SMC_X3_WO1 && cfg == 0 && k32 && !tag) hipLaunchKernelGGL((conv_gemm_x3_kernel<1, 4, 4, 1, 32>), grid, dim3(NT), 0, st, p);
            else if (SMC_X3_WO1 && cfg == 5 && k32s && !tag) hipLaunchKernelGGL((conv_gemm_x3_kernel<1, 4, 2, 1, 32>), grid, dim3(NT), 0, st, p);
            else if (cfg == 0 && k32 && tag) hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 2, 2, 32, SMC_X3_NST, 1>), grid, dim3(NT), 0, st, p);
            else if (cfg == 0 && k32) hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 2, 2, 32>), grid, dim3(NT), 0, st, p);
            else if (cfg == 0 && tag) hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 2, 2, 16, SMC_X3_NST, 1>), grid, dim3(NT), 0, st, p);
            else if (cfg == 0) hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 2, 2, 16>), grid, dim3(NT), 0, st, p);
            else if (cfg == 3 && cin % 32 == 0 && tag)
                hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 1, 1, 32, SMC_X3_NST, 1>), grid, dim3(NT), 0, st, p);
            else if (cfg == 3 && tag) hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 1, 1, 16, SMC_X3_NST, 1>), grid, dim3(NT), 0, st, p);
            else if (cfg == 3 && k32s) hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 1, 1, 32>), grid, dim3(NT), 0, st, p);
            else if (cfg == 3) hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 1, 1, 16>), grid, dim3(NT), 0, st, p);
            else if (cfg == 4 && k32s) hipLaunchKernelGGL((conv_gemm_x3_kernel<1, 4, 1, 1, 32>), grid, dim3(NT), 0, st, p);
            else if (cfg == 4) hipLaunchKernelGGL((conv_gemm_x3_kernel<1, 4, 1, 1, 16>), grid, dim3(NT), 0, st, p);
            else if (k32s) hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 1, 2, 32>), grid, dim3(NT), 0, st, p);
            else hipLaunchKernelGGL((conv_gemm_x3_kernel<2, 2, 1, 2, 16>), grid, dim3(NT), 0, st, p);
            rc = smc::check_launch("smc_conv_gemm_f32 (split-bf16)");
            if (rc != SMC_OK || nsplit == 1) return rc;
            return smc_modconv_epilogue_f32(workspace, nsplit, plane_elems, y, n, cout, y_h, y_w, &e, stream);
        }
        if (nsplit == 1 && !p.per_sample && (cfg == 4 || cfg == 5) &&
            row_ok(n, cin, cout, in_h, in_w, y_h, y_w, phases, nphases, Cfg{c.bo, 256}, &rt)) {
            p.ntn = cout / c.bo;  // column tiles (a 96-channel data gradient: 3 x 32)
            // measured on MI355X (tools/bench_gemm.py, batch 4; tap-major kernel in brackets): 32 channels,
            // 32 x 256 tiles of 8-channel steps: r = 1024 conv1 710 / 701 us fwd / data grad (840 / 818); 64
            // channels, 64 x 256: r = 512 655 / 648 (688 / 679).  128+ channels stay tap-major (the 128 x 128
            // row tile: 690 vs 634 us at r = 256).
            const int tiles = (int)(((int64_t)n * in_h * in_w) / 256) * p.ntn;
            if (cfg == 4) hipLaunchKernelGGL((conv_row_kernel<1, 4, 1, 2, 8>), dim3(tiles), dim3(NT), 0, st, p, rt);
            else hipLaunchKernelGGL((conv_row_kernel<1, 4, 2, 2, 8>), dim3(tiles), dim3(NT), 0, st, p, rt);
            return smc::check_launch("smc_conv_gemm_f32 (row-halo)");
        }
#define SMC_LAUNCH_LDS(WO_, WM_, TO_, TM_)                                                                          \
    do {                                                                                                          \
        if (tag) hipLaunchKernelGGL((conv_gemm_lds_kernel<WO_, WM_, TO_, TM_, 16, 2, 1>), grid, dim3(NT), 0, st, p); \
        else hipLaunchKernelGGL((conv_gemm_lds_kernel<WO_, WM_, TO_, TM_, 16, 2>), grid, dim3(NT), 0, st, p);       \
    } while (0)
        if (cfg == 0 && lds_bk32(cfg, cin) && tag)
            hipLaunchKernelGGL((conv_gemm_lds_kernel<2, 2, 2, 2, 32, 2, 1>), grid, dim3(NT), 0, st, p);
        else if (cfg == 0 && lds_bk32(cfg, cin))
            hipLaunchKernelGGL((conv_gemm_lds_kernel<2, 2, 2, 2, 32, 2>), grid, dim3(NT), 0, st, p);
        else if (cfg == 0) SMC_LAUNCH_LDS(2, 2, 2, 2);
        // IR-SE50 (TAG 1) 64x64 tiles: 32-channel K steps (half the barriers of a 9-step split):
        // f(4) + b(4) 3.57 -> 3.52 ms (profiles/r03_irse_bk32_ab.txt)
        else if (cfg == 3 && cin % 32 == 0 && tag)
            hipLaunchKernelGGL((conv_gemm_lds_kernel<2, 2, 1, 1, 32, 2, 1>), grid, dim3(NT), 0, st, p);
        else if (cfg == 3) SMC_LAUNCH_LDS(2, 2, 1, 1);
        else if (cfg == 4) SMC_LAUNCH_LDS(1, 4, 1, 1);
        else SMC_LAUNCH_LDS(2, 2, 1, 2);
#undef SMC_LAUNCH_LDS
        rc = smc::check_launch("smc_conv_gemm_f32 (LDS-DMA)");
        if (rc != SMC_OK || nsplit == 1) return rc;
        return smc_modconv_epilogue_f32(workspace, nsplit, plane_elems, y, n, cout, y_h, y_w, &e, stream);
    }
    // Register-staged kernel: the shapes the LDS-DMA kernel does not take (inputs of 2 GiB or more, style-scaled
    // inputs whose tiles straddle images with large per-sample weights).  BK = 32 halves the barriers per FLOP; it
    // pays on the long-K 512-channel layers, BK = 16 (more workgroups per CU: 32-40 KB LDS vs 64-80 KB) on the
    // high-resolution ones (tools/bench_gemm.py).  Raw buffer loads need the input to fit a 32-bit byte offset.
    const bool k32 = cin % 32 == 0 && cin >= 512;
    const bool buf = (int64_t)n * cin * in_h * in_w * 4 < (1LL << 31);
#define SMC_LAUNCH(WO_, WM_, TO_, TM_)                                                                       \
    do {                                                                                                   \
        if (k32 && buf && tag) hipLaunchKernelGGL((conv_gemm_kernel<WO_, WM_, TO_, TM_, 32, true, 1>), grid, dim3(NT), 0, st, p); \
        else if (buf && tag) hipLaunchKernelGGL((conv_gemm_kernel<WO_, WM_, TO_, TM_, 16, true, 1>), grid, dim3(NT), 0, st, p); \
        else if (k32 && buf) hipLaunchKernelGGL((conv_gemm_kernel<WO_, WM_, TO_, TM_, 32, true>), grid, dim3(NT), 0, st, p);   \
        else if (k32) hipLaunchKernelGGL((conv_gemm_kernel<WO_, WM_, TO_, TM_, 32, false>), grid, dim3(NT), 0, st, p);    \
        else if (buf) hipLaunchKernelGGL((conv_gemm_kernel<WO_, WM_, TO_, TM_, 16, true>), grid, dim3(NT), 0, st, p);     \
        else hipLaunchKernelGGL((conv_gemm_kernel<WO_, WM_, TO_, TM_, 16, false>), grid, dim3(NT), 0, st, p);             \
    } while (0)
    if (cfg == 0) SMC_LAUNCH(2, 2, 2, 2);
    else if (cfg == 4) SMC_LAUNCH(1, 4, 1, 1);
    else if (cfg == 5) SMC_LAUNCH(2, 2, 1, 2);
    else SMC_LAUNCH(2, 2, 1, 1);
#undef SMC_LAUNCH
    rc = smc::check_launch("smc_conv_gemm_f32");
    if (rc != SMC_OK || nsplit == 1) return rc;
    return smc_modconv_epilogue_f32(workspace, nsplit, plane_elems, y, n, cout, y_h, y_w, &e, stream);
}

}  // namespace

SMC_API int smc_conv_gemm_last_x3(void) { return g_last_x3; }

SMC_API int64_t smc_conv_weights_x3_bytes(int ntaps, int cin, int cout) {
    if (ntaps < 1 || ntaps > 9 || cin < 16 || cin % 16 || cout < 1) return 0;
    return (int64_t)ntaps * cin * cout * 3 * (int64_t)sizeof(short);
}

SMC_API int smc_conv_weights_x3(const float* wk, int ntaps, int cin, int cout, void* wk_x3, void* stream) {
    SMC_CHECK(wk && wk_x3, "smc_conv_weights_x3: null pointer");
    SMC_CHECK(smc_conv_weights_x3_bytes(ntaps, cin, cout) > 0, "smc_conv_weights_x3: bad shape taps=%d cin=%d cout=%d",
              ntaps, cin, cout);
    SMC_CHECK((reinterpret_cast<uintptr_t>(wk_x3) & 15) == 0, "smc_conv_weights_x3: planes must be 16-B aligned");
    const int64_t total = (int64_t)ntaps * cin * cout;
    hipLaunchKernelGGL(x3_weights_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(total, 256), 4096)), dim3(256),
                       0, smc::as_stream(stream), wk, nullptr, reinterpret_cast<short*>(wk_x3), ntaps, cin, cout, 1);
    return smc::check_launch("smc_conv_weights_x3");
}

SMC_API int smc_conv_gemm_f32(const float* x, int n, int cin, int in_h, int in_w, float* y, int cout, int y_h,
                              int y_w, const smc_conv_phase* phases, int nphases, const float* s_in,
                              const smc_conv_epilogue* epi, float* workspace, int64_t workspace_bytes,
                              void* stream) {
    return conv_gemm_impl(x, n, cin, in_h, in_w, y, cout, y_h, y_w, phases, nphases, s_in, epi, workspace,
                          workspace_bytes, stream, 0);
}

namespace smc {
int64_t conv_gemm_aux_workspace_size(int n, int cin, int cout, int y_h, int y_w, const smc_conv_phase* phases,
                                     int nphases) {
    return workspace_size_impl(n, cin, cout, y_h, y_w, phases, nphases, kSplitPerCuAux);
}

int conv_gemm_aux(const float* x, int n, int cin, int in_h, int in_w, float* y, int cout, int y_h, int y_w,
                  const smc_conv_phase* phases, int nphases, const float* s_in, const smc_conv_epilogue* epi,
                  float* workspace, int64_t workspace_bytes, void* stream) {
    return conv_gemm_impl(x, n, cin, in_h, in_w, y, cout, y_h, y_w, phases, nphases, s_in, epi, workspace,
                          workspace_bytes, stream, 1);
}
}  // namespace smc
