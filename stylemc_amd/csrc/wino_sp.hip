// Winograd F(2x2, 3x3) for small planes (<= 16 x 16: the IR-SE50 14x14 and 7x7 stages), split-K, fp32 MFMA on gfx950.
//
// The IR-SE50 convolutions of id_loss/model_irse.py (helpers.py:86-119 bottleneck_IR_SE: 3x3 stride-1 'same' convs and
// their adjoints) at 14x14 x 256 and 7x7 x 512 are latency-bound GEMMs: M = n * 196 positions, N = 256, K = 2304.  As
// implicit GEMMs they ran as 832 workgroups of 9 K steps each plus a 16-way split-K reduction (20.9 + 5.2 us per conv,
// 52 convs per IDLoss forward + backward).  Here each work item holds whole images' tile sets, so the input patch of a
// K step is the images' full planes (one contiguous, 16-B aligned run of 8 channels x H x W floats per image, staged
// by LDS-DMA), the multiplies drop 2.25x (16 per 2x2 tile and channel pair) and the K range of a work item is a
// split of the input channels; partial sums of the OUTPUT transform (linear) go to the split-K workspace and the
// existing reduction (smc_modconv_epilogue_f32) applies the conv epilogue (PRELU / AFFINE / PRELU_GRAD / residual).
//
// Work item (256 threads = 4 waves): 32 output channels x 64 tile slots x one input-channel split.  Tile slots: the
// images' tiles rounded up to 16 per image (14x14: 49 -> 64, one image per item; 7x7: 16, four images per item).  Per
// K step (8 channels, <= 4 per split): the U slab [8][4][32][4] (smc_wino_taps_f32) and the
// planes by DMA into a 2-stage LDS ring; per
// k-quad every lane reads ITS tile's 4x4 patch of ITS channel from the staged plane (zero outside the image), transforms
// it in registers -- its B fragment for all 16 xi -- and the 8 A fragments are ds_read_b128 (as wino.hip).
#include <algorithm>

#include "common.hpp"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int SBK = 8;     // input channels per K step
constexpr int SBO = 32;    // output channels per work item
constexpr int SMAXP = 256; // max floats per plane (16 x 16)
#ifndef SP_MAXK
#define SP_MAXK 4
#endif
constexpr int SMAXK = SP_MAXK;   // max K steps per split
// split target: SP_WG_PER_CU workgroups per CU, divided by SP_WG_DIV (A/B knobs)
#ifndef SP_WG_PER_CU
#define SP_WG_PER_CU 1
#endif
#ifndef SP_WG_DIV
#define SP_WG_DIV 1
#endif

struct WspParams {
    const float* x;
    int n, cin, h, w;
    float* ws;             // split-K partial planes [nsplit][n][cout][h][w]
    int64_t split_stride;  // floats
    int cout;
    const float* uw;       // [cin][4][cout][4]
    int th, tw;            // tiles per image
    int tpi, ipi;          // tile slots per image (multiple of 16), images per item
    int ntn;               // output-channel blocks
    int nitems;            // image groups x ntn
    int nsplit;
};

template <int N>
__device__ __forceinline__ void sp_wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino_sp_kernel(WspParams p) {
    constexpr int UF = SBK * 16 * SBO;          // U slab floats (4096)
    constexpr int UJW = UF / 4 / 256;           // U DMA instructions per wave per step (4)
    constexpr int PF = SBK * SMAXP;             // plane floats: ipi images x (8 channels x HW, in whole DMAs) <= 2048
    constexpr int STAGE = UF + PF;
    // two-stage ring (one step ahead).  Staging every step of a split at once (96 KB, one workgroup per CU)
    // measured slower: 17.5 against 15.8 us per 14x14 conv (profiles/r03_wino_sp_ab.txt)
    __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = p.h, W = p.w, HW = H * W;
    const int item = blockIdx.x, split = blockIdx.y;
    const int ob = item % p.ntn, ig = item / p.ntn;
    const int o0 = ob * SBO;
    const int n0 = ig * p.ipi;
    const int nimg = min(p.ipi, p.n - n0);
    // K range of this split, whole 8-channel steps
    const int nst = p.cin / SBK;
    const int ks0 = (int)((int64_t)nst * split / p.nsplit), ks1 = (int)((int64_t)nst * (split + 1) / p.nsplit);

    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * HW * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ursrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.uw, (short)0, (int)((int64_t)p.cin * 16 * p.cout * 4), 0x00020000);
    // U lanes: run = channel * 4 + xi group (32 x 16 B each), 2 runs per wave-instruction
    int uv[UJW];
#pragma unroll
    for (int j = 0; j < UJW; ++j) {
        const int run = 2 * (wave + 4 * j) + (lane >> 5);
        uv[j] = (((run >> 2) * 4 + (run & 3)) * p.cout + o0 + (lane & 31)) * 16;
    }
    // plane lanes: image i's run of 8 channels x HW floats = 2 HW chunks of 16 B, staged at i * istr
    const int istr = PF / p.ipi;
    const int chunks = 2 * HW;                       // per image
    const int pinstr = (chunks + 63) / 64;           // wave-instructions per image
    const int pjw = (nimg * pinstr + 3) / 4;         // per wave
    auto issue = [&](int ks, int slot) {
        float* us = smem + slot * STAGE;
        const int uso = ks * (SBK * 16 * 4) * p.cout;
#pragma unroll
        for (int j = 0; j < UJW; ++j) {
            const int vo = uv[j];
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                ursrc, (__attribute__((address_space(3))) void*)(us + (wave + 4 * j) * 256), 16, vo, uso, 0, 0);
        }
        float* ps = us + UF;
        for (int jj = 0; jj < pjw; ++jj) {
            const int ins = wave + 4 * jj;           // instruction index over all images
            const int i = ins / pinstr, k = ins - i * pinstr;
            if (i < nimg) {
                const int ch = k * 64 + lane;        // 16-B chunk within the image's run
                const int vo = ch < chunks ? (int)((((int64_t)(n0 + i) * p.cin + ks * SBK) * HW + 4 * ch) * 4)
                                           : 0x7ffffff0;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    xrsrc, (__attribute__((address_space(3))) void*)(ps + i * istr + k * 256), 16, vo, 0, 0, 0);
            }
        }
    };

    // this lane's tile slot: t = 16 wave + (lane & 15) -> image t / tpi, tile t % tpi
    const int t = 16 * wave + (lane & 15);
    const int ti = t / p.tpi, tl = t - ti * p.tpi;
    const bool tvalid = ti < nimg && tl < p.th * p.tw;
    const int ty = tvalid ? tl / p.tw : 0, tx = tvalid ? tl - (tl / p.tw) * p.tw : 0;
    const int kq_lane = lane >> 4;
    const int uoff = (kq_lane * 4 * SBO + (lane & 15)) * 4;
    // patch element (r, c) = plane[2 ty - 1 + r][2 tx - 1 + c], zero outside the image
    const int pbase = ti * istr + (2 * ty - 1) * W + (2 * tx - 1);
    unsigned rok = 0, cok = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int yy = 2 * ty - 1 + r, xx = 2 * tx - 1 + r;
        rok |= (tvalid && yy >= 0 && yy < H ? 1u : 0u) << r;
        cok |= (xx >= 0 && xx < W ? 1u : 0u) << r;
    }

    f32x4 acc[16][2];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[xi][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (ks0 < ks1) issue(ks0, 0);
    for (int ks = ks0, gs = 0; ks < ks1; ++ks, ++gs) {
        sp_wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (ks + 1 < ks1) issue(ks + 1, (gs + 1) & 1);
        const float* us = smem + (gs & 1) * STAGE;
        const float* ps = us + UF;
#pragma unroll
        for (int kq = 0; kq < 2; ++kq) {
            // this lane's channel plane: k-quad kq, channel kq_lane (channel c of image i at i * istr + c * HW)
            const float* pl = ps + (4 * kq + kq_lane) * HW;
            float d[16];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const bool in = ((rok >> r) & (cok >> c) & 1u) != 0;
                    const float v = pl[in ? pbase + r * W + c : 0];
                    d[4 * r + c] = in ? v : 0.f;
                }
            float tt[4][4], vv[16];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                tt[0][j] = d[j] - d[8 + j];
                tt[1][j] = d[4 + j] + d[8 + j];
                tt[2][j] = d[8 + j] - d[4 + j];
                tt[3][j] = d[4 + j] - d[12 + j];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                vv[4 * i + 0] = tt[i][0] - tt[i][2];
                vv[4 * i + 1] = tt[i][1] + tt[i][2];
                vv[4 * i + 2] = tt[i][2] - tt[i][1];
                vv[4 * i + 3] = tt[i][1] - tt[i][3];
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float* up = us + kq * 4 * 4 * SBO * 4 + uoff + g * SBO * 4;
                f32x4 a[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) a[b] = *reinterpret_cast<const f32x4*>(up + 16 * 4 * b);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc[4 * g + j][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[b][j], vv[4 * g + j], acc[4 * g + j][b],
                                                                                0, 0, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    // output transform of this split's partial sums -> the split's partial plane (the reduction applies the epilogue)
    if (!tvalid) return;
    const int nn = n0 + ti;
    float* dst = p.ws + (int64_t)split * p.split_stride;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int o = o0 + 16 * b + 4 * kq_lane + r;
            float m[4][4];
#pragma unroll
            for (int xi = 0; xi < 16; ++xi) m[xi >> 2][xi & 3] = acc[xi][b][r];
            float rr[2][4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                rr[0][j] = m[0][j] + m[1][j] + m[2][j];
                rr[1][j] = m[1][j] - m[2][j] - m[3][j];
            }
            float* op = dst + ((int64_t)nn * p.cout + o) * HW;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int yy = 2 * ty + i;
                if (yy >= H) continue;
                const float v0 = rr[i][0] + rr[i][1] + rr[i][2];
                const float v1 = rr[i][1] - rr[i][2] - rr[i][3];
                op[yy * W + 2 * tx] = v0;
                if (2 * tx + 1 < W) op[yy * W + 2 * tx + 1] = v1;
            }
        }
}

// U = G g G^T (F(2x2)) per (k = input channel, n = output channel) from a packed 9-tap phase wk [tap][cin][cout] with
// taps (dy, dx) in {-1, 0, 1}^2 (the correlation out[y][x] = sum wk[t] in[y + dy_t][x + dx_t]): g[dy + 1][dx + 1].
// Out: [cin][4][cout][4] (the smc_wino_weights_f32 layout).
struct Taps9 {
    int idx[9];  // tap index of (ky, kx) = (dy + 1, dx + 1), row-major
};

__global__ __launch_bounds__(256) void wino_taps_kernel(const float* wk, Taps9 tp, int cin, int cout, float* uw) {
    const int64_t total = (int64_t)cin * cout;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(e / cout), nidx = (int)(e - (int64_t)k * cout);
        float g[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) g[i][j] = wk[((int64_t)tp.idx[3 * i + j] * cin + k) * cout + nidx];
        float gg[4][3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            gg[0][j] = g[0][j];
            gg[1][j] = 0.5f * (g[0][j] + g[1][j] + g[2][j]);
            gg[2][j] = 0.5f * (g[0][j] - g[1][j] + g[2][j]);
            gg[3][j] = g[2][j];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float u[4];
            u[0] = gg[i][0];
            u[1] = 0.5f * (gg[i][0] + gg[i][1] + gg[i][2]);
            u[2] = 0.5f * (gg[i][0] - gg[i][1] + gg[i][2]);
            u[3] = gg[i][2];
#pragma unroll
            for (int j = 0; j < 4; ++j) uw[(((int64_t)k * 4 + i) * cout + nidx) * 4 + j] = u[j];
        }
    }
}

bool taps_same3x3(const smc_conv_phase* ph, Taps9* tp) {
    if (!ph || ph->ntaps != 9 || ph->in_stride != 1 || ph->out_oy || ph->out_ox || ph->out_sy != 1 || ph->out_sx != 1)
        return false;
    int seen = 0;
    for (int t = 0; t < 9; ++t) {
        const int dy = ph->tap_dy[t], dx = ph->tap_dx[t];
        if (dy < -1 || dy > 1 || dx < -1 || dx > 1) return false;
        const int q = 3 * (dy + 1) + (dx + 1);
        if (seen & (1 << q)) return false;
        seen |= 1 << q;
        if (tp) tp->idx[q] = t;
    }
    return seen == 0x1ff;
}

struct SpPlan {
    int th, tw, tpi, ipi, ntn, nitems, nsplit;
};

SpPlan sp_plan(int n, int cin, int cout, int h, int w) {
    SpPlan s{};
    s.th = (h + 1) / 2;
    s.tw = (w + 1) / 2;
    s.tpi = ((s.th * s.tw + 15) / 16) * 16;
    s.ipi = 64 / s.tpi;
    s.ntn = cout / SBO;
    s.nitems = ((n + s.ipi - 1) / s.ipi) * s.ntn;
    // one workgroup per CU (two, i.e. twice the splits, measured 3.38 against 3.25 ms per IR-SE50 f4 + b4: the
    // split-K reduction grows with the splits), whole 8-channel steps per split, at most SMAXK of them
    const int target = SP_WG_PER_CU * smc::device_cu_count() / SP_WG_DIV;
    const int nst = cin / SBK;
    const int plan_items = ((smc::plan_batch(n) + s.ipi - 1) / s.ipi) * s.ntn;   // the split from the planning batch
    s.nsplit = std::min(nst, std::max((int)smc::ceil_div(nst, SMAXK), (int)smc::ceil_div(target, plan_items)));
    return s;
}

}  // namespace

SMC_API int smc_wino_sp_supported(int n, int cin, int cout, int h, int w) {
    if (n < 1 || cin < 2 * SBK || cin % SBK || cout < SBO || cout % SBO) return 0;
    if (h < 2 || w < 2 || h > 16 || w > 16) return 0;
    if ((int64_t)n * cin * h * w * 4 >= (1LL << 31)) return 0;
    if ((int64_t)cin * 16 * cout * 4 >= (1LL << 31)) return 0;   // the U slab's buffer range (num_records)
    return 1;
}

SMC_API int64_t smc_wino_sp_workspace_size(int n, int cin, int cout, int h, int w) {
    if (!smc_wino_sp_supported(n, cin, cout, h, w)) return 0;
    const SpPlan s = sp_plan(n, cin, cout, h, w);
    return (int64_t)s.nsplit * n * cout * h * w * (int64_t)sizeof(float);
}

SMC_API int smc_wino_taps_f32(const smc_conv_phase* ph, int cin, int cout, float* uw, void* stream) {
    Taps9 tp{};
    SMC_CHECK(ph && ph->wk && uw && cin >= 1 && cout >= 1, "smc_wino_taps_f32: bad arguments");
    SMC_CHECK(taps_same3x3(ph, &tp), "smc_wino_taps_f32: the phase is not a 9-tap 3x3 stride-1 'same' conv");
    SMC_CHECK((reinterpret_cast<uintptr_t>(uw) & 15) == 0, "smc_wino_taps_f32: uw must be 16-B aligned");
    const int64_t total = (int64_t)cin * cout;
    hipLaunchKernelGGL(wino_taps_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(total, 256), 4096)), dim3(256),
                       0, smc::as_stream(stream), ph->wk, tp, cin, cout, uw);
    return smc::check_launch("smc_wino_taps_f32");
}

SMC_API int smc_conv3x3_wino_sp_f32(const float* x, int n, int cin, int h, int w, float* y, int cout, const float* uw,
                                    const smc_conv_epilogue* epi, float* workspace, int64_t workspace_bytes,
                                    void* stream) {
    SMC_CHECK(x && y && uw && workspace, "smc_conv3x3_wino_sp_f32: null pointer");
    if (!smc_wino_sp_supported(n, cin, cout, h, w)) {
        smc::set_error("smc_conv3x3_wino_sp_f32: no small-plane Winograd kernel for n=%d cin=%d cout=%d %dx%d", n, cin,
                       cout, h, w);
        return SMC_ERR_UNSUPPORTED;
    }
    SMC_CHECK((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(uw) & 15) == 0,
              "smc_conv3x3_wino_sp_f32: x / uw must be 16-B aligned");
    SMC_CHECK(workspace_bytes >= smc_wino_sp_workspace_size(n, cin, cout, h, w),
              "smc_conv3x3_wino_sp_f32: workspace too small");
    const SpPlan s = sp_plan(n, cin, cout, h, w);
    WspParams p{};
    p.x = x; p.n = n; p.cin = cin; p.h = h; p.w = w; p.ws = workspace;
    p.split_stride = (int64_t)n * cout * h * w;
    p.cout = cout; p.uw = uw;
    p.th = s.th; p.tw = s.tw; p.tpi = s.tpi; p.ipi = s.ipi; p.ntn = s.ntn; p.nitems = s.nitems; p.nsplit = s.nsplit;
    hipStream_t st = smc::as_stream(stream);
    hipLaunchKernelGGL(wino_sp_kernel, dim3((unsigned)s.nitems, (unsigned)s.nsplit), dim3(256), 0, st, p);
    const int rc = smc::check_launch("smc_conv3x3_wino_sp_f32");
    if (rc != SMC_OK) return rc;
    smc_conv_epilogue e{};
    e.mode = SMC_EPI_STORE; e.act = SMC_ACT_LINEAR; e.gain = 1.f; e.clamp = -1.f;
    if (epi) e = *epi;
    return smc_modconv_epilogue_f32(workspace, s.nsplit, p.split_stride, y, n, cout, h, w, &e, stream);
}
