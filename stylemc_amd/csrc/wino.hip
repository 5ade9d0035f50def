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

// A/B knobs (SMC_AB_DEFINES builds a variant library): the forward's style scale folded into per-image U (kept:
// r = 512 / 1024 forward 426 -> 407 / 497 -> 489 us, profiles/r05/wino_ab/); the accumulators cleared by each one's
// first MFMA (zero C operand, the loop peeled) instead of 128 v_mov per item (not kept: the data gradient 396 -> 401 /
// 473 -> 479 us -- twice the loop code for ~10 % of the VALU stream)
#ifndef SMC_WINO_FOLD
#define SMC_WINO_FOLD 1
#endif
#ifndef SMC_WINO_ZEROC
#define SMC_WINO_ZEROC 0
#endif
// cache-policy bits of the input patch DMAs (A/B knob; 2 = nt)
#ifndef SMC_WINO_XAUX
#define SMC_WINO_XAUX 0
#endif

constexpr int WBK = 8;    // input channels per K step
constexpr int WBO = 32;   // output channels per workgroup
constexpr int WBT = 64;   // tiles per workgroup (4 waves x 16)

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
    int nsplit;            // K splits (grid.y): > 1 stores raw partial tiles (EK 3) for smc_modconv_epilogue_f32
    int64_t split_stride;  // floats between the partial planes of two splits
    float* ws;             // the partial planes [nsplit][n][cout][h][w]
    int64_t u_nstride;     // 0: one U for the batch; else floats between per-image U (s[n, c] folded in)
};

// Staged row pitch: CHP >= CH 16-B chunks (the pad chunks are sentinel DMA lanes, zero-filled) so that a channel slab
// is 32 floats mod 64.  A lane reads its 4 x 4 patch as three aligned 8-B reads per row (columns 2 tc + 2 .. + 7 of
// the staged row); in a read group the 16 tiles' pairs of one channel cover 32 consecutive dwords and the other
// channel's are one slab away, i.e. the other 32 of the 64 banks: conflict-free.  (Reads of the unaligned patch start
// compile to ds_read2_b32 pairs at lane stride 2: two lanes on every bank, a third of the kernel's LDS cycles.)
constexpr int wino_chp(int rows, int ch) {
    int c = ch;
    while ((rows * 4 * c) % 64 != 32) ++c;
    return c;
}

template <int TC>
struct WinoCfg {
    static constexpr int TR = WBT / TC;             // tile rows of the block
    static constexpr int ROWS = 2 * TR + 2;         // staged input rows
    static constexpr int CH = TC / 2 + 2;           // 16-B chunks per staged row (2 TC + 8 floats)
    static constexpr int CHP = wino_chp(ROWS, CH);  // ... with the pad chunks
    static constexpr int PITCH = 4 * CHP;
    static constexpr int SLAB = ROWS * PITCH;       // floats per channel (32 mod 64)
    static constexpr int PL = WBK * ROWS * CHP;     // DMA lanes of the patch (pad lanes included)
    static constexpr int PJ = (PL + 63) / 64;       // patch DMA wave-instructions per step
    static constexpr int PF = PJ * 256;             // floats reserved for the patch (whole instructions)
    static constexpr int UF = WBK * 16 * WBO;       // floats of the U slab
    static constexpr int UJ = UF / 256;             // U DMA wave-instructions per step (16 B per lane)
    static constexpr int STAGE = UF + PF;
    static constexpr int NW = 4;                    // waves per workgroup
    static constexpr int UJW = UJ / NW;             // U DMAs per wave per step
    static constexpr int PJW = (PJ + NW - 1) / NW;  // patch DMAs per wave per step (at most)
    static_assert(UJ % NW == 0, "U slab splits evenly over the 4 waves");
};

template <int N>
__device__ __forceinline__ void wino_wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One work item = 32 output channels x 64 tiles of one image: (image, tile group, output-channel block).
struct WinoItem {
    int nn, ty0, tx0, o0;
};

// PROBE (0 in the library) removes pieces for timing probes: 1 the U DMAs after the first step, 2 the patch DMAs
// after the first step, 4 the per-step wait + barrier, 8 the epilogue, 16 the transform, 32 the LDS fragment reads.
// SM: the style scale s[n, c] known at compile time (1: present, 2: absent).  PERSIST: the grid holds as many
// workgroups as fit on the chip and each loops over work items (stride gridDim.x); the next item's first DMA is
// issued during the current item's last K step, so the K loop's fill latency and the epilogue of one item overlap
// instead of starting every workgroup cold -- what the 4-step (cin 32) and 8-step (cin 64) layers lost most to.
// EK: the epilogue body, chosen at launch (1: MODACT lrelu + gain + clamp, 2: MODACT linear, 0: any mode, 3: the raw
// output tiles of a K split into the workspace -- the split-K form, p.nsplit > 1, grid.y = split).
template <int TC, int SM, int EK, int PERSIST, int PROBE = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void wino_kernel(WinoParams p) {
    using C = WinoCfg<TC>;
    constexpr int OBW = 2, NW = C::NW, UJW = C::UJW, PJW = C::PJW;
    constexpr int TR = C::TR, ROWS = C::ROWS, CH = C::CH, CHP = C::CHP, PITCH = C::PITCH, SLAB = C::SLAB;
    constexpr int STAGE = C::STAGE;
    __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = p.h, W = p.w;
    const int64_t plane = (int64_t)H * W;
    const int nsteps = p.cin / WBK / p.nsplit;  // this workgroup's K steps: channels [kb WBK, (kb + nsteps) WBK)
    const int kb = (int)blockIdx.y * nsteps;
    const int total = p.n * p.gx * p.gy * p.ntn;
    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * plane * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ursrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.uw, (short)0, (p.u_nstride ? p.n : 1) * p.cin * 16 * p.cout * 4, 0x00020000);

    // work item v -> (image, tile group, output-channel block) through the XCD-aware bijective order of conv_gemm.hip
    // (items v and v + 8 run on one XCD when the grid is a multiple of 8; output-channel blocks fastest, so the
    // workgroups that stage the same input patch share an L2)
    auto decode = [&](int v) {
        const int xcd = v % 8, q8 = total / 8, r8 = total % 8;
        const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + v / 8;
        const int ob = id % p.ntn, tg = id / p.ntn;
        const int per_img = p.gx * p.gy;
        WinoItem it;
        it.nn = tg / per_img;
        const int rem = tg - it.nn * per_img;
        it.ty0 = (rem / p.gx) * TR;
        it.tx0 = (rem % p.gx) * TC;
        it.o0 = ob * WBO;
        return it;
    };
    // per-lane byte offsets of an item's step 0; a step adds a scalar offset (U slab: 8 channels x 16 x cout floats;
    // patch: 8 planes).  The out-of-range sentinel 0x7ffffff0 + a step offset < 2^31 stays out of range.
    auto offsets = [&](const WinoItem& it, int (&uv)[UJW], int (&pv)[PJW]) {
#pragma unroll
        for (int j = 0; j < UJW; ++j) {
            const int run = 2 * (wave + NW * j) + (lane >> 5);  // run = channel * 4 + xi group: 32 x 16 B
            uv[j] = (((run >> 2) * 4 + (run & 3)) * p.cout + it.o0 + (lane & 31)) * 16;
        }
#pragma unroll
        for (int jj = 0; jj < PJW; ++jj) {
            const int L = (wave + NW * jj) * 64 + lane;
            const int c = L / (ROWS * CHP);
            const int r2 = L - c * (ROWS * CHP);
            const int r = r2 / CHP, ch = r2 - r * CHP;
            const int gyy = 2 * it.ty0 - 1 + r, gxx = 2 * it.tx0 - 4 + 4 * ch;
            const bool ok = c < WBK && ch < CH && gyy >= 0 && gyy < H && gxx >= 0 && gxx < W;
            pv[jj] = ok ? (int)((((int64_t)(it.nn * p.cin + c) * H + gyy) * W + gxx) * 4) : 0x7ffffff0;
        }
    };
    // step ks of an item into LDS slot `slot`: the U slab [8][4][32][4] and the raw input rows of the block's
    // (2 TR + 2) x (2 TC + 8) patch (16-B chunks from column 2 tx0 - 4, zero-filled by the buffer range check)
    auto issue = [&](const int (&uv)[UJW], const int (&pv)[PJW], int ks, int slot, int nn) {
        float* us = smem + slot * STAGE;
        const int uso = (kb + ks) * (WBK * 16 * 4) * p.cout + nn * (int)p.u_nstride * 4;
#pragma unroll
        for (int j = 0; j < ((PROBE & 1) != 0 && ks > 0 ? 0 : UJW); ++j) {
            const int vo = uv[j];  // (through a local: hipcc drops the kernel's host stub when the array is passed)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                ursrc, (__attribute__((address_space(3))) void*)(us + (wave + NW * j) * 256), 16, vo, uso, 0, 0);
        }
        if constexpr ((PROBE & 2) != 0)
            if (ks > 0) return;
        float* ps = us + C::UF;
        const int pso = (kb + ks) * WBK * (int)plane * 4;
#pragma unroll
        for (int jj = 0; jj < PJW; ++jj)
            if (wave + NW * jj < C::PJ) {
                const int vo = pv[jj];
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    xrsrc, (__attribute__((address_space(3))) void*)(ps + (wave + NW * jj) * 256), 16, vo, pso, 0,
                    SMC_WINO_XAUX);
            }
    };

    const int stride = PERSIST ? (int)gridDim.x : total;
    int v = blockIdx.x;
    if (v >= total) return;

    const int kq_lane = lane >> 4;   // MFMA k (channel within a k-quad)
    const int tl = 16 * wave + (lane & 15);
    const int tr = tl / TC, tc = tl - tr * TC;
    const int poff = kq_lane * SLAB + 2 * tr * PITCH + 2 * tc + 2;  // (even: 8-B aligned pairs; the patch starts at +1)
    const int uoff = (kq_lane * 4 * WBO + (lane & 15)) * 4;
    const bool has_s = SM == 1 ? true : SM == 2 ? false : p.s != nullptr;

    WinoItem it = decode(v);
    int uv[UJW], pv[PJW];
    offsets(it, uv, pv);
    issue(uv, pv, 0, 0, it.nn);
    const float* srow = has_s ? p.s + (int64_t)it.nn * p.cin + kb * WBK + kq_lane : p.x;
    float sv[2] = {1.f, 1.f}, sn[2] = {1.f, 1.f};
    if (has_s) { sn[0] = srow[0]; sn[1] = srow[4]; }
    int gs = 0;  // K steps run by this workgroup so far: LDS slot gs & 1

    // Fragment pipeline.  A step's 8 MFMA groups gi = 4 kq + g (k-quad kq, xi group g: 8 MFMAs each) read their A
    // fragments from a 2-deep register ring loaded one group ahead; the k-quad-1 patch is read under group 0 and
    // transformed under group 3.  The last group of a step is deferred past the next step's barrier, so its MFMAs
    // cover the LDS latency of the next step's first patch / A reads (it needs only registers).
    float pd[16], va[16], vb[16];
    f32x4 ar[2][OBW];
    f32x4 acc[16][OBW];
    auto load_patch = [&](const float* ps, int kq) {
        if constexpr ((PROBE & 32) != 0) return;
        const float* pp = ps + kq * 4 * SLAB + poff;
        typedef float f32x2 __attribute__((ext_vector_type(2), aligned(8)));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f32x2 a = *reinterpret_cast<const f32x2*>(pp + i * PITCH);
            const f32x2 b = *reinterpret_cast<const f32x2*>(pp + i * PITCH + 2);
            const f32x2 c = *reinterpret_cast<const f32x2*>(pp + i * PITCH + 4);
            pd[4 * i + 0] = a[1];
            pd[4 * i + 1] = b[0];
            pd[4 * i + 2] = b[1];
            pd[4 * i + 3] = c[0];
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
    auto transform = [&](float sc, float (&vv)[16]) {
        if constexpr ((PROBE & 16) != 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) vv[i] = pd[i];
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
            vv[4 * i + 0] = (t[i][0] - t[i][2]) * sc;
            vv[4 * i + 1] = (t[i][1] + t[i][2]) * sc;
            vv[4 * i + 2] = (t[i][2] - t[i][1]) * sc;
            vv[4 * i + 3] = (t[i][1] - t[i][3]) * sc;
        }
    };
    // ZERO: the first product into each accumulator of an item takes a zero C operand (an inline constant of the
    // MFMA) instead of accumulators cleared by 128 v_mov per item
    auto mma_group = [&](int g, const f32x4 (&a)[OBW], const float (&vv)[16], auto zero_c) {
        constexpr bool ZERO = decltype(zero_c)::value;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int b = 0; b < OBW; ++b)
                acc[4 * g + j][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                    a[b][j], vv[4 * g + j], ZERO ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[4 * g + j][b], 0, 0, 0);
    };
    using NZ = std::false_type;

    for (;;) {
        if constexpr (!SMC_WINO_ZEROC) {
#pragma unroll
            for (int xi = 0; xi < 16; ++xi)
#pragma unroll
                for (int b = 0; b < OBW; ++b) acc[xi][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        const int vn = v + stride;
        const bool has_next = PERSIST && vn < total;
        WinoItem nx = it;
        const float* srow_n = srow;
        bool pend = false;
        for (int ks = 0; ks < nsteps; ++ks, ++gs) {
            if constexpr ((PROBE & 4) == 0) {
                wino_wait_vmcnt<0>();
                __builtin_amdgcn_s_barrier();  // this step landed for every wave; the other slot is no longer read
            }
            asm volatile("" ::: "memory");
            sv[0] = sn[0]; sv[1] = sn[1];
            if (ks + 1 < nsteps) {
                issue(uv, pv, ks + 1, (gs + 1) & 1, it.nn);
                if (has_s) { sn[0] = srow[(ks + 1) * WBK]; sn[1] = srow[(ks + 1) * WBK + 4]; }
            } else if (has_next) {  // the next item's first step, under this item's last MFMAs and its epilogue
                nx = decode(vn);
                int uvn[UJW], pvn[PJW];
                offsets(nx, uvn, pvn);
                issue(uvn, pvn, 0, (gs + 1) & 1, nx.nn);
                if (has_s) {
                    srow_n = p.s + (int64_t)nx.nn * p.cin + kq_lane;
                    sn[0] = srow_n[0]; sn[1] = srow_n[4];
                }
            }
            const float* us = smem + (gs & 1) * STAGE;
            const float* ps = us + C::UF;
            // (sched_barrier fences keep each phase where it is written: the compiler would otherwise sink the
            // prefetches next to their use to save registers and wait on them with lgkmcnt(0))
            load_patch(ps, 0);
            load_a(us, 0, ar[0]);
            __builtin_amdgcn_sched_barrier(0);
            if (pend) mma_group(3, ar[1], vb, NZ{});  // the previous step's last group
            __builtin_amdgcn_sched_barrier(0);
            transform(sv[0], va);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int gi = 0; gi < 8; ++gi) {
                if (gi + 1 < 8) load_a(us, gi + 1, ar[(gi + 1) & 1]);
                if (gi == 0) load_patch(ps, 1);
                __builtin_amdgcn_sched_barrier(0);
                if (SMC_WINO_ZEROC && gi < 4 && ks == 0) {
                    mma_group(gi, ar[gi & 1], va, std::true_type{});   // each accumulator's first product
                } else if (gi < 7) {
                    mma_group(gi & 3, ar[gi & 1], gi < 4 ? va : vb, NZ{});
                } else {
                    pend = ks + 1 < nsteps;
                    if (!pend) mma_group(3, ar[1], vb, NZ{});
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
        } else {
            const int nn = it.nn;
            const int yy0 = 2 * (it.ty0 + tr), xx0 = 2 * (it.tx0 + tc);
            // The MODACT epilogue's per-channel / per-pixel operands, all loaded before the first store (issued after
            // a store that may alias them, each would wait out that store's round trip)
            float e_d[OBW][4], e_b[OBW][4], nz[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
            if (EK != 3 && p.mode == SMC_EPI_MODACT) {
#pragma unroll
                for (int b = 0; b < OBW; ++b)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int o = it.o0 + 16 * b + 4 * kq_lane + r;
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
            // The synthesis' two MODACT forms get a body with the activation fixed at compile time (KIND 1: lrelu
            // with 0 <= alpha <= 1, gain, clamp -- the conv1 forward; KIND 2: linear, no clamp -- the data gradient's
            // x s[n, i]): lrelu(z) = max(z, alpha z) and clamp = min / max, bit-identical to smc::epi_y for every
            // finite value, without the per-element tests of the runtime activation.  KIND 0: any epilogue through
            // smc::epi_y / epi_ext_apply.
            auto body = [&](auto kind_c) {
                constexpr int KIND = decltype(kind_c)::value;
#pragma unroll
                for (int b = 0; b < OBW; ++b) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int o = it.o0 + 16 * b + 4 * kq_lane + r;
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
                        if constexpr (KIND == 3) {
                            float* wp = p.ws + blockIdx.y * p.split_stride;
#pragma unroll
                            for (int i = 0; i < 2; ++i)
                                *reinterpret_cast<float2*>(wp + obase + (int64_t)(yy0 + i) * W + xx0) =
                                    make_float2(out[i][0], out[i][1]);
                        } else if (KIND != 0 || p.mode == SMC_EPI_MODACT) {
                            const float dsc = e_d[b][r], bo = e_b[b][r];
#pragma unroll
                            for (int i = 0; i < 2; ++i) {
                                const int64_t idx = obase + (int64_t)(yy0 + i) * W + xx0;
                                if (p.u_save)
                                    *reinterpret_cast<float2*>(p.u_save + idx) = make_float2(out[i][0], out[i][1]);
                                float q[2];
#pragma unroll
                                for (int j = 0; j < 2; ++j) {
                                    if constexpr (KIND == 1) {
                                        const float z = __fmaf_rn(out[i][j], dsc, nz[i][j]) + bo;
                                        q[j] = smc::lrelu_gain_clamp(z, p.alpha, p.gain, p.clamp);
                                    } else if constexpr (KIND == 2) {
                                        q[j] = (__fmaf_rn(out[i][j], dsc, nz[i][j]) + bo) * p.gain;
                                    } else {
                                        q[j] = smc::epi_y(out[i][j], dsc, nz[i][j], bo, p.act, p.alpha, p.gain, p.clamp);
                                        if (p.ext.residual)
                                            q[j] = smc::epi_ext_apply(SMC_EPI_STORE, q[j], nn, o, idx + j, yy0 + i,
                                                                      xx0 + j, p.cout, H, W, nullptr, nullptr, p.ext);
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
                                    q[j] = smc::epi_ext_apply(p.mode, out[i][j], nn, o, idx + j, yy0 + i, xx0 + j,
                                                              p.cout, H, W, p.bias, p.u_save, p.ext);
                                *reinterpret_cast<float2*>(p.y + idx) = make_float2(q[0], q[1]);
                            }
                        }
                    }
                }
            };
            body(std::integral_constant<int, EK>{});
        }
        if (!has_next) break;
        v = vn;
        it = nx;
        offsets(it, uv, pv);  // (recomputed: cheaper than keeping the next item's offsets alive through the epilogue)
        srow = srow_n;
    }
}

// Per-image U with the style folded in: out[nn][c][...] = uw[c][...] * s[nn][c] (float4 runs of the [cin][4][cout][4]
// layout).  The forward's x s[n, c] then costs nothing in the kernel's input transform (16 multiplies per patch and
// channel, ~10 % of its VALU stream, which shares the SIMD issue port with the fp32 MFMA).
__global__ __launch_bounds__(256) void wino_ufold_kernel(const float4* uw, const float* s, float4* out, int cin,
                                                         int per4, int64_t total4) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total4; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t nn = e / per4;
        const int r = (int)(e - nn * per4);
        const int c = r / (per4 / cin);
        const float sc = s[nn * cin + c];
        float4 v = uw[r];
        v.x *= sc; v.y *= sc; v.z *= sc; v.w *= sc;
        out[e] = v;
    }
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
// Tile columns per block, at most (A/B knob).  A cap of 32 (2 tile rows at W >= 64) measured 477 / 468 against
// 480 / 473 us at r = 1024 fwd / data grad and 18.64-18.70 against 18.72-18.74 ms per step over three interleaved
// rounds (profiles/r03_wino_tc_ab.txt); the default since round 4.
#ifndef SMC_WINO_TC_MAX
#define SMC_WINO_TC_MAX 32
#endif
int wino_tc(int h, int w) {
    if (h % 2 || w % 4 || w < 32) return 0;
    for (int tc = SMC_WINO_TC_MAX; tc >= 16; tc /= 2)
        if ((w / 2) % tc == 0 && (h / 2) % (WBT / tc) == 0) return tc;
    return 0;
}

// One workgroup per work item.  (The persistent form -- PERSIST = 1, a resident grid looping over items with the
// next item's first DMA under the current item's last step -- measured 3-18 % slower on every synthesis shape:
// tools/probes/wino_ab.hip, profiles/r03_wino_ab.txt.)
// (timing / counter probes only: tools/ builds a variant library with -DSMC_WINO_PROBE=n, see wino_kernel's PROBE)
#ifndef SMC_WINO_PROBE
#define SMC_WINO_PROBE 0
#endif
template <int TC, int SM, int EK>
void launch_wino(const WinoParams& p, int64_t items, hipStream_t st) {
    hipLaunchKernelGGL((wino_kernel<TC, SM, EK, 0, SMC_WINO_PROBE>), dim3((unsigned)items, (unsigned)p.nsplit), dim3(256),
                       0, st, p);
}

template <int SM, int EK>
void launch_wino_tc(int tc, const WinoParams& p, int64_t items, hipStream_t st) {
    if (tc == 64) launch_wino<64, SM, EK>(p, items, st);
    else if (tc == 32) launch_wino<32, SM, EK>(p, items, st);
    else launch_wino<16, SM, EK>(p, items, st);
}

template <int EK>
void launch_wino_s(bool has_s, int tc, const WinoParams& p, int64_t items, hipStream_t st) {
    if (has_s) launch_wino_tc<1, EK>(tc, p, items, st);
    else launch_wino_tc<2, EK>(tc, p, items, st);
}

// K splits of a launch: a grid of fewer than two workgroups per CU (the kernel's occupancy) leaves each SIMD one
// wave to hide the DMA and LDS latency with -- the 32 x 32 synthesis conv of cin 512 (256 items, 64 K steps) ran at
// a quarter of the MFMA rate.  Split K (a power of two dividing the step count, >= 8 steps per split) until the grid
// holds kWinoSplitTarget workgroups; the partial tiles are summed by the modconv epilogue kernel.
#ifndef SMC_WINO_SPLIT_TARGET
#define SMC_WINO_SPLIT_TARGET 512
#endif
constexpr int64_t kWinoSplitTarget = SMC_WINO_SPLIT_TARGET;

int wino_nsplit(int n, int cin, int cout, int h, int w) {
    const int tc = wino_tc(h, w);
    if (!tc) return 1;
    const int64_t items = (int64_t)smc::plan_batch(n) * ((w / 2) / tc) * ((h / 2) / (WBT / tc)) * (cout / WBO);
    const int nsteps = cin / WBK;
    int ns = 1;
    while (items * ns < kWinoSplitTarget && nsteps % (2 * ns) == 0 && nsteps / (2 * ns) >= 8) ns *= 2;
    return ns;
}

// The fold applies where the per-image U is small (the 32 / 64-channel layers: 64 / 256 KB per image).
constexpr int64_t kWinoFoldMaxCinCout = 128 * 128;
int64_t wino_fold_bytes(int n, int cin, int cout) {
    return (int64_t)cin * cout <= kWinoFoldMaxCinCout ? (int64_t)n * cin * 16 * cout * 4 : 0;
}
int64_t wino_split_bytes(int n, int cin, int cout, int h, int w) {
    const int ns = wino_nsplit(n, cin, cout, h, w);
    return ns > 1 ? (((int64_t)ns * n * cout * h * w * 4 + 255) / 256) * 256 : 0;
}

// ---------------------------------------------------------------------------------------------------
// Split-bf16 F(2x2) for the 32-channel layer (cin = cout = 32: the r = 1024 conv1 forward and its data gradient).
// The fp32 kernel above spends most of that launch in the fp32 MFMA K loop (219 us of 505 at r = 1024, batch 4:
// profiles/r06/fir_fwd_ab/README).  Here the 16 per-xi GEMMs run on the bf16 matrix core as three-term splits (the
// scheme of conv_gemm.hip's x3 kernels: a = a0 + a1 + a2 by truncation, the six products a_i b_j with i + j <= 2,
// smallest first, error <= 2^-23 |a b| per product): 6 v_mfma_f32_16x16x32_bf16 (16 cycles) per 16x16x32 block in
// place of 8 v_mfma_f32_16x16x4f32 (32 cycles) -- 2.7x fewer matrix-core cycles.
//   * the whole K = 32 is one MFMA K block, so a workgroup keeps its image's split U planes in LDS for all its items:
//     [xi 16][term 3][out block 2][k-octet 4][out 16][8] bf16 = 96 KB (wino_x3_pack_kernel; x s[n, c] folded in for the
//     style-scaled forward), DMA'd once; an A fragment is one conflict-free ds_read_b128 per term.
//   * one workgroup per CU (LDS), persistent over the items of one image (grid.y = image; items v, v + gridDim.x, ...),
//     4 waves x 16 tiles of the item's 2 x 32 tile block.  Lane (tile, k-octet g) transforms the 4 x 4 patches of its
//     tile for the 8 channels 4 j + g (the read pattern of the fp32 kernel's k-quads: conflict-free), so its B fragment
//     of every xi -- 8 consecutive MFMA k = channels 4 j + g, j = 0..7 -- is already in its registers; the A planes
//     store k in the same order.
//   * one patch buffer: the item's patch is transformed into registers (V[8][16]), then the next item's patch DMA is
//     issued under this item's MFMAs and epilogue.  The C layout of the 16x16x32 MFMA is the 16x16x4 one, so the
//     epilogue is the fp32 kernel's.
// Mode (smc_set_wino_x3, process-wide; SMC_WINO_X3 the build's initial value): 0 the fp32 kernel for these shapes, 1
// the split-bf16 kernel for the conv1 forward form (EK 1), 2 also for the data gradient's (EK 2).
#ifndef SMC_WINO_X3
#define SMC_WINO_X3 0
#endif
int g_wino_x3 = SMC_WINO_X3;
typedef short wbf16x8 __attribute__((ext_vector_type(8)));
constexpr int X3C = 32;                                   // cin = cout
constexpr int X3_UPLANE = 16 * 3 * 2 * 4 * 16 * 8;        // bf16 per image
constexpr int X3_UBYTES = X3_UPLANE * 2;                  // 96 KB

// x = t0 + t1 + t2 for 8 values, as three bf16x8 fragments (the high halves of x, x - t0, x - t0 - t1)
__device__ __forceinline__ void wx3_split8(const float (&x)[8], wbf16x8 (&t)[3]) {
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
    for (int j = 0; j < 4; ++j) {
        w0[j] = __builtin_amdgcn_perm(u0[2 * j + 1], u0[2 * j], 0x07060302u);
        w1[j] = __builtin_amdgcn_perm(u1[2 * j + 1], u1[2 * j], 0x07060302u);
        w2[j] = __builtin_amdgcn_perm(u2[2 * j + 1], u2[2 * j], 0x07060302u);
    }
    t[0] = __builtin_bit_cast(wbf16x8, w0);
    t[1] = __builtin_bit_cast(wbf16x8, w1);
    t[2] = __builtin_bit_cast(wbf16x8, w2);
}

// out[nn][xi][term][b][g][o16][j] = term of uw[c = 4 j + g][xi / 4][o = 16 b + o16][xi % 4] * (s ? s[nn][c] : 1)
__global__ __launch_bounds__(256) void wino_x3_pack_kernel(const float* uw, const float* s, short* out, int64_t total) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(e & 7), o16 = (int)((e >> 3) & 15), g = (int)((e >> 7) & 3), b = (int)((e >> 9) & 1);
        const int xi = (int)((e >> 10) & 15);
        const int64_t nn = e >> 14;
        const int c = 4 * j + g, o = 16 * b + o16;
        float v = uw[((c * 4 + (xi >> 2)) * X3C + o) * 4 + (xi & 3)];
        if (s) v *= s[nn * X3C + c];
        const unsigned u = __float_as_uint(v);
        const float r1 = v - __uint_as_float(u & 0xffff0000u);
        const unsigned w = __float_as_uint(r1);
        const float r2 = r1 - __uint_as_float(w & 0xffff0000u);
        const unsigned term[3] = {u >> 16, w >> 16, __float_as_uint(r2) >> 16};
#pragma unroll
        for (int t = 0; t < 3; ++t)
            out[((((nn * 16 + xi) * 3 + t) * 2 + b) * 4 + g) * 128 + o16 * 8 + j] = (short)term[t];
    }
}

// (timing probes only, variant libraries: 1 no MFMAs, 2 no epilogue stores, 4 no transform LDS reads, 8 no waits)
#ifndef SMC_WINO_X3_PROBE
#define SMC_WINO_X3_PROBE 0
#endif
template <int EK>
__global__ __launch_bounds__(256, 1) void wino_x3_kernel(WinoParams p, const short* planes, int64_t plane_nstride) {
    static_assert(EK == 1 || EK == 2, "the synthesis' MODACT epilogue forms");
    using C = WinoCfg<32>;
    constexpr int TC = 32, TR = C::TR, ROWS = C::ROWS, CH = C::CH, CHP = C::CHP, PITCH = C::PITCH, SLAB = C::SLAB;
    static_assert(8 * ROWS * CHP == 15 * 64, "a quarter (8 channels) is 15 DMA wave-instructions");
    constexpr int QF = 16 * 256;                // floats per quarter slot: 15 KB of patch + 1 KB (slot 0: the noise)
    constexpr int UJW = X3_UBYTES / 1024 / 4;   // U DMA wave-instructions per wave (24)
    constexpr int OBW = 2;
    static_assert(X3_UBYTES % 4096 == 0, "U planes split evenly over the 4 waves");
    __shared__ __attribute__((aligned(16))) char smem[X3_UBYTES + 4 * QF * 4];
    float* ps = reinterpret_cast<float*>(smem + X3_UBYTES);
    const float* nsm = ps + 15 * 256;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = p.h, W = p.w;
    const int nn = blockIdx.y;
    const int items = p.gx * p.gy;
    const int S = gridDim.x;
    int k = blockIdx.x;
    if (k >= items) return;
    const bool has_noise = p.noise != nullptr, has_u = p.u_save != nullptr;
    const int kg = lane >> 4;   // MFMA k-octet: channels 4 j + kg
    const int tl = 16 * wave + (lane & 15);
    const int tr = tl / TC, tc = tl - tr * TC;

    // the epilogue's per-channel operands, once per workgroup (one image), parked in accumulation registers (the arch
    // VGPRs hold V, fragments and splits) -- loaded before any DMA, so their wait drains nothing
    float e_dA[OBW][4], e_bA[OBW][4];
#pragma unroll
    for (int b = 0; b < OBW; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int o = 16 * b + 4 * kg + r;
            const float dv = (p.d ? p.d[(int64_t)nn * p.cout + o] : 1.f) * (p.ext.scale_c ? p.ext.scale_c[o] : 1.f);
            const float bv = p.bias ? p.bias[o] : 0.f;
            asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(e_dA[b][r]) : "v"(dv));
            asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(e_bA[b][r]) : "v"(bv));
        }
    const float nstr = has_noise ? (p.noise_strength ? *p.noise_strength : 1.f) : 0.f;

    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * H * W * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ursrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(planes + nn * plane_nstride), (short)0, X3_UBYTES, 0x00020000);
    const __amdgpu_buffer_rsrc_t nrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.noise, (short)0, has_noise ? (int)(((int64_t)(p.n - 1) * p.noise_nstride + (int64_t)H * W) * 4) : 0,
        0x00020000);
#pragma unroll
    for (int j = 0; j < UJW; ++j) {
        const int J = wave * UJW + j;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ursrc, (__attribute__((address_space(3))) void*)(smem + J * 1024), 16,
                                                 (J * 64 + lane) * 16, 0, 0, 0);
    }
    // Patch DMA by quarters (8 channels: 15 wave-instructions, + 1: slot 0's 16th is the item's noise [4][64], the others
    // a zero-fill), every wave exactly 4 per quarter.  The transform reads quarter q of item k while quarters q..3 of
    // item k + 1 are still to be issued; vmcnt counts loads, stores and LDS-DMA together in issue order, so "quarter q
    // of k landed" is vmcnt(N): its later quarters (12 - 4 q), the S epilogue stores of item k - 1, and item k + 1's
    // quarters issued so far in this item (4 (q - 1) at q >= 1: quarter q - 1 goes out after quarter q's barrier), so
    // N = 12 + S at q = 0 and 8 + S after.
    auto dma = [&](int kk, int q) {  // item kk's quarter q (kk >= items: all lanes zero-fill)
        const bool valid = kk < items;
        const int ty0 = (kk / p.gx) * TR, tx0 = (kk % p.gx) * TC;
        float* slot = ps + q * QF;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int jq = wave + 4 * jj;
            int ln = lane;   // (opaque: the loop-invariant parts of these offsets would be hoisted into 16 registers)
            asm volatile("" : "+v"(ln));
            if (jq == 15) {
                const bool ok = valid && q == 0 && has_noise;
                const int vo = ok ? ((int)(nn * p.noise_nstride) + (2 * ty0 + (ln >> 4)) * W + 2 * tx0 + 4 * (ln & 15)) * 4
                                  : 0x7ffffff0;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(nrsrc, (__attribute__((address_space(3))) void*)(slot + 15 * 256),
                                                         16, vo, 0, 0, 0);
            } else {
                const int L = jq * 64 + ln;
                const int cc = L / (ROWS * CHP);
                const int r2 = L - cc * (ROWS * CHP);
                const int r = r2 / CHP, ch = r2 - r * CHP;
                const int gyy = 2 * ty0 - 1 + r, gxx = 2 * tx0 - 4 + 4 * ch;
                const bool ok = valid && ch < CH && gyy >= 0 && gyy < H && gxx >= 0 && gxx < W;
                const int vo = ok ? (((nn * p.cin + 8 * q + cc) * H + gyy) * W + gxx) * 4 : 0x7ffffff0;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, (__attribute__((address_space(3))) void*)(slot + jq * 256),
                                                         16, vo, 0, 0, 0);
            }
        }
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) dma(k, q);

    // LDS read bases kept opaque so that every fragment / patch read is base + a 16-bit immediate (offsets past 64 KB
    // would each take a register, hoisted out of the item loop)
    typedef __attribute__((address_space(3))) const short lds_cshort;
    typedef __attribute__((address_space(3))) const float lds_cfloat;
    typedef float f32x2 __attribute__((ext_vector_type(2), aligned(8)));
    typedef __attribute__((address_space(3))) const f32x2 lds_cf32x2;
    lds_cshort* ua = (lds_cshort*)smem + (kg * 16 + (lane & 15)) * 8;
    lds_cshort* ua8 = ua + 8 * 3 * 2 * 512;
    lds_cfloat* pb = (lds_cfloat*)ps + kg * SLAB + 2 * tr * PITCH + 2 * tc + 2;
    asm volatile("" : "+v"(ua), "+v"(ua8), "+v"(pb));

    // channel j (= 4 j + kg) of the lane's tile: its 4 x 4 patch from quarter slot j / 2, and V = B^T d B
    auto transform = [&](int j, float (&vv)[16]) {
        lds_cfloat* pp = pb + (j >> 1) * QF + (j & 1) * 4 * SLAB;
        float pd[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr ((SMC_WINO_X3_PROBE & 4) != 0) {
                pd[4 * i] = (float)(j + i + tid);
                pd[4 * i + 1] = pd[4 * i] + 1.f;
                pd[4 * i + 2] = pd[4 * i] * 3.f;
                pd[4 * i + 3] = pd[4 * i] - 2.f;
                continue;
            }
            const f32x2 a = *reinterpret_cast<lds_cf32x2*>(pp + i * PITCH);
            const f32x2 b = *reinterpret_cast<lds_cf32x2*>(pp + i * PITCH + 2);
            const f32x2 c = *reinterpret_cast<lds_cf32x2*>(pp + i * PITCH + 4);
            pd[4 * i + 0] = a[1];
            pd[4 * i + 1] = b[0];
            pd[4 * i + 2] = b[1];
            pd[4 * i + 3] = c[0];
        }
        float t[4][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            t[0][q] = pd[q] - pd[8 + q];
            t[1][q] = pd[4 + q] + pd[8 + q];
            t[2][q] = pd[8 + q] - pd[4 + q];
            t[3][q] = pd[4 + q] - pd[12 + q];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            vv[4 * i + 0] = t[i][0] - t[i][2];
            vv[4 * i + 1] = t[i][1] + t[i][2];
            vv[4 * i + 2] = t[i][2] - t[i][1];
            vv[4 * i + 3] = t[i][1] - t[i][3];
        }
    };
    auto load_a = [&](int xi, wbf16x8 (&a)[OBW][3]) {
#pragma unroll
        for (int b = 0; b < OBW; ++b)
#pragma unroll
            for (int t = 0; t < 3; ++t)
                a[b][t] = *reinterpret_cast<__attribute__((address_space(3))) const wbf16x8*>(
                    (xi < 8 ? ua : ua8) + (((xi & 7) * 3 + t) * 2 + b) * 512);
    };

    f32x4 acc[16][OBW];
    for (;;) {
        const int kn = k + S;
        // ---- V = B^T d B of item k, quarter by quarter; each freed slot takes item k + 1's quarter at once
        float V[8][16], nr[2][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if ((SMC_WINO_X3_PROBE & 8) != 0) {}
            else if (k < (int)blockIdx.x + S) {   // (no stores yet)
                if (q == 0) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            } else if (has_u) {
                if (q == 0) asm volatile("s_waitcnt vmcnt(44)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
            } else {
                if (q == 0) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // quarter q landed for every wave; every wave is done with slot q - 1
            asm volatile("" ::: "memory");
            if (q > 0) dma(kn, q - 1);
            if (q == 0) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x2 z = *reinterpret_cast<const f32x2*>(nsm + (2 * tr + i) * 64 + 2 * tc);
                    nr[i][0] = z[0];
                    nr[i][1] = z[1];
                }
            }
            transform(2 * q, V[2 * q]);
            transform(2 * q + 1, V[2 * q + 1]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        dma(kn, 3);

        // ---- M[xi] = U[xi] V[xi]: per xi 2 output blocks x 6 split products; the split (VALU) and A fragment reads of
        // xi + 1 go between the MFMAs of xi (one wave per SIMD: only its own stream fills the slots an MFMA leaves)
        auto split = [&](int xi, wbf16x8 (&bt)[3]) {
            const float xv[8] = {V[0][xi], V[1][xi], V[2][xi], V[3][xi], V[4][xi], V[5][xi], V[6][xi], V[7][xi]};
            wx3_split8(xv, bt);
        };
        wbf16x8 at[2][OBW][3], bt[2][3];
        load_a(0, at[0]);
        split(0, bt[0]);
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) {
            __builtin_amdgcn_sched_barrier(0);
            if (xi + 1 < 16) {
                load_a(xi + 1, at[(xi + 1) & 1]);
                split(xi + 1, bt[(xi + 1) & 1]);
            }
            const wbf16x8 (&a)[OBW][3] = at[xi & 1];
            const wbf16x8 (&b3)[3] = bt[xi & 1];
            if constexpr ((SMC_WINO_X3_PROBE & 1) != 0) {
                acc[xi][0] = f32x4{(float)b3[0][0] + (float)a[0][0][0], (float)b3[1][0], (float)b3[2][0], (float)b3[0][1]};
                acc[xi][1] = f32x4{(float)b3[0][3] + (float)a[1][2][0], (float)b3[1][4], (float)b3[2][5], (float)b3[2][1]};
                __builtin_amdgcn_sched_barrier(0);
                continue;
            }
            // four independent chains (each output block: the three small products, the three large ones), each
            // MFMA four issues after its predecessor in the chain -- two chains left the matrix core waiting on results
            f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, l0 = s0, l1 = s0;
            s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][2], b3[0], s0, 0, 0, 0);
            s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][2], b3[0], s1, 0, 0, 0);
            l0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][1], b3[0], l0, 0, 0, 0);
            l1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][1], b3[0], l1, 0, 0, 0);
            s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][1], b3[1], s0, 0, 0, 0);
            s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][1], b3[1], s1, 0, 0, 0);
            l0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][0], b3[1], l0, 0, 0, 0);
            l1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][0], b3[1], l1, 0, 0, 0);
            s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][0], b3[2], s0, 0, 0, 0);
            s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][0], b3[2], s1, 0, 0, 0);
            l0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][0], b3[0], l0, 0, 0, 0);
            l1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][0], b3[0], l1, 0, 0, 0);
            acc[xi][0] = l0 + s0;
            acc[xi][1] = l1 + s1;
            if (xi + 1 < 16) {
#pragma unroll
                for (int m = 0; m < 12; ++m) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);               // one MFMA
                    if (m < 6) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // one LDS read
                    __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);               // four VALU
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }

        // ---- Y = A^T M A per (channel, tile) and the MODACT epilogue (wino_kernel's KIND 1 / 2); 32-bit offsets from
        // the image's base (64-bit per-row addresses would be hoisted out of the loop into registers it does not have).
        // Exactly 16 y stores (+ 16 u stores): the vmcnt counts above depend on it.
        {
            const int plane = H * W;
            float* yb = p.y + (int64_t)nn * p.cout * plane;
            float* ub = has_u ? p.u_save + (int64_t)nn * p.cout * plane : nullptr;
            const int pix = (2 * ((k / p.gx) * TR + tr)) * W + 2 * ((k % p.gx) * TC + tc) + 4 * kg * plane;
            float nz[2][2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) nz[i][j] = nr[i][j] * nstr;
#pragma unroll
            for (int b = 0; b < OBW; ++b) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
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
                    float dsc, bo;
                    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(dsc) : "a"(e_dA[b][r]));
                    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(bo) : "a"(e_bA[b][r]));
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const int idx = pix + (16 * b + r) * plane + i * W;
                        if constexpr ((SMC_WINO_X3_PROBE & 2) != 0) {
                            if (out[i][0] == 12345.f) yb[idx] = out[i][1];
                            continue;
                        }
                        if (has_u) *reinterpret_cast<float2*>(ub + idx) = make_float2(out[i][0], out[i][1]);
                        float q[2];
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            if constexpr (EK == 1) {
                                const float z = __fmaf_rn(out[i][j], dsc, nz[i][j]) + bo;
                                q[j] = smc::lrelu_gain_clamp(z, p.alpha, p.gain, p.clamp);
                            } else {
                                q[j] = (__fmaf_rn(out[i][j], dsc, nz[i][j]) + bo) * p.gain;
                            }
                        }
                        *reinterpret_cast<float2*>(yb + idx) = make_float2(q[0], q[1]);
                    }
                }
            }
        }
        if (kn >= items) break;
        k = kn;
    }
}

// Register-U form (SMC_WINO_X3R, the default for the split-bf16 path): the 96 KB of U planes left one 256-thread
// workgroup -- one wave per SIMD -- per CU above, and one wave alone issues a vector instruction every 4 cycles and
// hides no LDS latency (profiles/r06/wino_x3/README).  Here the waves split the work by Winograd row: an item is one
// tile row of 32 tiles (a 2 x 64 output block), wave w owns row a = w % 4 (xi = 4 a .. 4 a + 3) of tile block
// tb = w / 4 (16 tiles), so its A fragments -- 4 xi x 2 output blocks x 3 terms -- fit in registers (the two larger
// terms, 64 VGPRs; the smallest from a 32 KB LDS copy): 8 waves per workgroup, two per SIMD.  A wave transforms only its
// row of V (two patch rows per channel); the output transform Y = A^T M A is split the same way -- each wave writes
// R[a] = M[a][:] A to a 32 KB LDS exchange and, after a barrier, sums the four rows of an eighth of the item's outputs
// and runs the epilogue.  Patch staging: the quarter ring and counted waits of the kernel above, 16 DMA
// wave-instructions per quarter (9 of patch, slot 0's 10th the noise rows, the rest zero-fill) = 2 per wave.
#ifndef SMC_WINO_X3R
#define SMC_WINO_X3R 1
#endif
template <int EK>
__global__ __launch_bounds__(512, 1) void wino_x3r_kernel(WinoParams p, const short* planes, int64_t plane_nstride) {
    static_assert(EK == 1 || EK == 2, "the synthesis' MODACT epilogue forms");
    constexpr int TC = 32, ROWS = 4, CH = TC / 2 + 2, CHP = wino_chp(ROWS, CH), PITCH = 4 * CHP, SLAB = ROWS * PITCH;
    constexpr int PJ = 8 * ROWS * CHP / 64;   // patch DMA wave-instructions per quarter (9)
    static_assert(8 * ROWS * CHP == PJ * 64 && PJ < 16, "a quarter's patch is whole wave-instructions, plus the noise");
    constexpr int QF = 16 * 256;    // floats per quarter slot (16 KB: PJ KB of patch, the noise, zero-fill)
    constexpr int RINGF = 4 * QF;   // 64 KB
    constexpr int EXF = 8192;       // exchange: [a 4][tb 2][b 2][r 4][lane 64][2] floats = 32 KB
    __shared__ __attribute__((aligned(16))) char smem[RINGF * 4 + EXF * 4 + 32768];
    float* ps = reinterpret_cast<float*>(smem);
    const float* nsm = ps + PJ * 256;   // slot 0: the item's noise rows [2][64]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ra = wave & 3, tb = wave >> 2;   // this wave's Winograd row a and tile block
    const int H = p.h, W = p.w;
    const int nn = blockIdx.y;
    const int items = p.gx * p.gy;
    const int SG = gridDim.x;
    int k = blockIdx.x;
    if (k >= items) return;
    const bool has_noise = p.noise != nullptr, has_u = p.u_save != nullptr;
    const int kg = lane >> 4, o16 = lane & 15;
    // combine role: tile block ctb, output block cb, rows r = 2 crp, 2 crp + 1 of the lane's k-octet
    const int ctb = wave >> 2, cb = (wave >> 1) & 1, crp = wave & 1;

    // epilogue operands and the two larger U terms of this wave's row, loaded and consumed before any DMA (a later first
    // use would make the compiler wait for the DMAs)
    float e_d[2], e_b[2];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const int o = 16 * cb + 4 * kg + 2 * crp + rr;
        e_d[rr] = (p.d ? p.d[(int64_t)nn * p.cout + o] : 1.f) * (p.ext.scale_c ? p.ext.scale_c[o] : 1.f);
        e_b[rr] = p.bias ? p.bias[o] : 0.f;
    }
    const float nstr = has_noise ? (p.noise_strength ? *p.noise_strength : 1.f) : 0.f;
    const short* up = planes + nn * plane_nstride;
    wbf16x8 ua0[4][2], ua1[4][2];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int xi = 4 * ra + x;
            ua0[x][b] = *reinterpret_cast<const wbf16x8*>(up + (((xi * 3 + 0) * 2 + b) * 4 + kg) * 128 + o16 * 8);
            ua1[x][b] = *reinterpret_cast<const wbf16x8*>(up + (((xi * 3 + 1) * 2 + b) * 4 + kg) * 128 + o16 * 8);
        }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) asm volatile("" ::"v"(e_d[rr]), "v"(e_b[rr]));
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int b = 0; b < 2; ++b) asm volatile("" ::"v"(ua0[x][b]), "v"(ua1[x][b]));

    const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, (short)0, (int)((int64_t)p.n * p.cin * H * W * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ursrc = __builtin_amdgcn_make_buffer_rsrc((void*)up, (short)0, X3_UBYTES, 0x00020000);
    const __amdgpu_buffer_rsrc_t nrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.noise, (short)0, has_noise ? (int)(((int64_t)(p.n - 1) * p.noise_nstride + (int64_t)H * W) * 4) : 0,
        0x00020000);
    // the smallest term: block J = 2 xi + b is the planes' [kg 4][o16 16][8] run of term 2 -- 1 KB, one DMA each
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        const int J = wave + 8 * jj;
        const int xi = J >> 1, b = J & 1;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            ursrc, (__attribute__((address_space(3))) void*)(smem + RINGF * 4 + EXF * 4 + J * 1024), 16,
            ((((xi * 3 + 2) * 2 + b) * 512) + lane * 8) * 2, 0, 0, 0);
    }
    auto dma = [&](int kk, int q) {  // item kk's quarter q: 16 wave-instructions, 2 per wave (kk >= items: zero-fill)
        const bool valid = kk < items;
        const int ty0 = kk / p.gx, tx0 = (kk % p.gx) * TC;
        float* slot = ps + q * QF;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const int jq = wave + 8 * jj;
            int ln = lane;   // (opaque: keeps the loop-invariant parts of the offsets out of registers)
            asm volatile("" : "+v"(ln));
            if (jq >= PJ) {  // the noise (slot 0) / zero-fill
                const bool ok = valid && q == 0 && jq == PJ && has_noise && ln < 32;
                const int vo = ok ? ((int)(nn * p.noise_nstride) + (2 * ty0 + (ln >> 4)) * W + 2 * tx0 + 4 * (ln & 15)) * 4
                                  : 0x7ffffff0;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(nrsrc, (__attribute__((address_space(3))) void*)(slot + jq * 256),
                                                         16, vo, 0, 0, 0);
            } else {
                const int L = jq * 64 + ln;
                const int cc = L / (ROWS * CHP);
                const int r2 = L - cc * (ROWS * CHP);
                const int r = r2 / CHP, ch = r2 - r * CHP;
                const int gyy = 2 * ty0 - 1 + r, gxx = 2 * tx0 - 4 + 4 * ch;
                const bool ok = valid && ch < CH && gyy >= 0 && gyy < H && gxx >= 0 && gxx < W;
                const int vo = ok ? (((nn * p.cin + 8 * q + cc) * H + gyy) * W + gxx) * 4 : 0x7ffffff0;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xrsrc, (__attribute__((address_space(3))) void*)(slot + jq * 256),
                                                         16, vo, 0, 0, 0);
            }
        }
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) dma(k, q);

    typedef __attribute__((address_space(3))) const float lds_cfloat;
    typedef float f32x2 __attribute__((ext_vector_type(2), aligned(8)));
    typedef __attribute__((address_space(3))) const f32x2 lds_cf32x2;
    typedef __attribute__((address_space(3))) f32x2 lds_f32x2;
    typedef __attribute__((address_space(3))) const wbf16x8 lds_cbf16x8;
    // the row pair of this wave's Winograd row: t[a] = d[r0] + sg d[r1] (B^T rows 1 0 -1 0 / 0 1 1 0 / 0 -1 1 0 /
    // 0 1 0 -1); the 16 tiles' columns are 2 tc + 2 .. 2 tc + 7 of the staged rows
    const int r0 = ra == 0 ? 0 : ra == 2 ? 2 : 1;
    const int r1 = ra == 0 ? 2 : ra == 2 ? 1 : ra == 1 ? 2 : 3;
    const float sg = ra == 1 ? 1.f : -1.f;
    lds_cfloat* pb = (lds_cfloat*)ps + kg * SLAB + 2 * (16 * tb + o16) + 2;
    lds_cfloat* pr0 = pb + r0 * PITCH;
    lds_cfloat* pr1 = pb + r1 * PITCH;
    lds_cbf16x8* a2p = (lds_cbf16x8*)(smem + RINGF * 4 + EXF * 4) + (8 * ra) * 64 + lane;   // + (2 x + b) * 64
    lds_f32x2* exw = (lds_f32x2*)(ps + RINGF) + (ra * 2 + tb) * 2 * 4 * 64 + lane;          // + (b 4 + r) 64
    lds_cf32x2* exr = (lds_cf32x2*)(ps + RINGF) + (ctb * 2 + cb) * 4 * 64 + 2 * crp * 64 + lane;  // + a 1024 + rr 64
    asm volatile("" : "+v"(pr0), "+v"(pr1), "+v"(a2p), "+v"(exw), "+v"(exr));

    auto row = [&](lds_cfloat* pp, float (&d)[4]) {
        const f32x2 a = *reinterpret_cast<lds_cf32x2*>(pp);
        const f32x2 b = *reinterpret_cast<lds_cf32x2*>(pp + 2);
        const f32x2 c = *reinterpret_cast<lds_cf32x2*>(pp + 4);
        d[0] = a[1];
        d[1] = b[0];
        d[2] = b[1];
        d[3] = c[0];
    };

    for (;;) {
        const int kn = k + SG;
        // ---- this wave's row of V = B^T d B, quarter by quarter
        float V[8][4], nr[2][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            // quarter q of item k landed: all but its later quarters (6 - 2 q), the S stores of item k - 1 and the
            // 2 (q - 1) DMAs of item k + 1 issued at quarters 1 .. q - 1 -- N = 6 + S at q = 0, 4 + S after
            if (k < (int)blockIdx.x + SG) {   // (no stores yet)
                if (q == 0) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            } else if (has_u) {
                if (q == 0) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            } else {
                if (q == 0) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();   // quarter q landed for every wave; slot q - 1 and the exchange are free
            asm volatile("" ::: "memory");
            if (q > 0) dma(kn, q - 1);
            if (q == 0) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const f32x2 z = *reinterpret_cast<const f32x2*>(nsm + i * 64 + 2 * (16 * ctb + o16));
                    nr[i][0] = z[0];
                    nr[i][1] = z[1];
                }
            }
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const int off = q * QF + jj * 4 * SLAB;
                float d0[4], d1[4], t[4];
                row(pr0 + off, d0);
                row(pr1 + off, d1);
#pragma unroll
                for (int c = 0; c < 4; ++c) t[c] = d0[c] + sg * d1[c];
                float* v = V[2 * q + jj];
                v[0] = t[0] - t[2];
                v[1] = t[1] + t[2];
                v[2] = t[2] - t[1];
                v[3] = t[1] - t[3];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        dma(kn, 3);

        // ---- M[a][x] = U[4a + x] V[4a + x] (4 independent chains per x), then R[a] = M[a][:] A into the exchange
        {
            f32x4 acc[4][2];
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const float xv[8] = {V[0][x], V[1][x], V[2][x], V[3][x], V[4][x], V[5][x], V[6][x], V[7][x]};
                wbf16x8 bt[3];
                wx3_split8(xv, bt);
                const wbf16x8 a2_0 = a2p[(2 * x + 0) * 64], a2_1 = a2p[(2 * x + 1) * 64];
                f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, l0 = s0, l1 = s0;
                s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2_0, bt[0], s0, 0, 0, 0);
                s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2_1, bt[0], s1, 0, 0, 0);
                l0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua1[x][0], bt[0], l0, 0, 0, 0);
                l1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua1[x][1], bt[0], l1, 0, 0, 0);
                s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua1[x][0], bt[1], s0, 0, 0, 0);
                s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua1[x][1], bt[1], s1, 0, 0, 0);
                l0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua0[x][0], bt[1], l0, 0, 0, 0);
                l1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua0[x][1], bt[1], l1, 0, 0, 0);
                s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua0[x][0], bt[2], s0, 0, 0, 0);
                s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua0[x][1], bt[2], s1, 0, 0, 0);
                l0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua0[x][0], bt[0], l0, 0, 0, 0);
                l1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua0[x][1], bt[0], l1, 0, 0, 0);
                acc[x][0] = l0 + s0;
                acc[x][1] = l1 + s1;
            }
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float m0 = acc[0][b][r], m1 = acc[1][b][r], m2 = acc[2][b][r], m3 = acc[3][b][r];
                    exw[(b * 4 + r) * 64] = f32x2{m0 + m1 + m2, m1 - m2 - m3};
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // every row's R is in the exchange
        asm volatile("" ::: "memory");

        // ---- Y = A^T R (rows 1 1 1 0 / 0 1 -1 -1) for tile block ctb, output block cb, rows 2 crp .. + 1; the
        // epilogue.  Exactly 4 y stores (+ 4 u stores) per wave: the vmcnt counts above depend on it.
        {
            const int plane = H * W;
            float* yb = p.y + (int64_t)nn * p.cout * plane;
            float* ub = has_u ? p.u_save + (int64_t)nn * p.cout * plane : nullptr;
            const int pix = (2 * (k / p.gx)) * W + 2 * ((k % p.gx) * TC + 16 * ctb + o16) +
                            (16 * cb + 4 * kg + 2 * crp) * plane;
            float nz[2][2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) nz[i][j] = nr[i][j] * nstr;
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                f32x2 R[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) R[a] = exr[a * 1024 + rr * 64];
                float out[2][2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    out[0][j] = R[0][j] + R[1][j] + R[2][j];
                    out[1][j] = R[1][j] - R[2][j] - R[3][j];
                }
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int idx = pix + rr * plane + i * W;
                    if (has_u) *reinterpret_cast<float2*>(ub + idx) = make_float2(out[i][0], out[i][1]);
                    float qv[2];
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        if constexpr (EK == 1) {
                            const float z = __fmaf_rn(out[i][j], e_d[rr], nz[i][j]) + e_b[rr];
                            qv[j] = smc::lrelu_gain_clamp(z, p.alpha, p.gain, p.clamp);
                        } else {
                            qv[j] = (__fmaf_rn(out[i][j], e_d[rr], nz[i][j]) + e_b[rr]) * p.gain;
                        }
                    }
                    *reinterpret_cast<float2*>(yb + idx) = make_float2(qv[0], qv[1]);
                }
            }
        }
        if (kn >= items) break;
        k = kn;
    }
}

// bytes of split U planes the x3 path takes from the workspace (0: the shape runs the fp32 kernel)
int64_t wino_x3_bytes(int n, int cin, int cout, int h, int w) {
    return g_wino_x3 && cin == X3C && cout == X3C && wino_tc(h, w) == 32 ? (int64_t)n * X3_UBYTES : 0;
}

template <int EK>
void launch_wino_x3(const WinoParams& p, const short* planes, int64_t nstride, hipStream_t st) {
    const int items = p.gx * p.gy;
    const int per_img = (int)std::max<int64_t>(1, std::min<int64_t>(items, smc::device_cu_count() / p.n));
    if (SMC_WINO_X3R) {   // items of one tile row (32 tiles)
        WinoParams q = p;
        q.gy = p.h / 2;
        const int per = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)q.gx * q.gy, smc::device_cu_count() / p.n));
        hipLaunchKernelGGL(wino_x3r_kernel<EK>, dim3((unsigned)per, (unsigned)p.n), dim3(512), 0, st, q, planes, nstride);
    } else
        hipLaunchKernelGGL(wino_x3_kernel<EK>, dim3((unsigned)per_img, (unsigned)p.n), dim3(256), 0, st, p, planes,
                           nstride);
}


}  // namespace

SMC_API int smc_set_wino_x3(int mode) {
    const int prev = g_wino_x3;
    g_wino_x3 = mode < 0 ? 0 : mode > 2 ? 2 : mode;
    return prev;
}

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

// [split-K partial planes (when the grid is too small)][per-image folded U (forward with a style scale)]
SMC_API int64_t smc_conv3x3_wino_workspace_size(int n, int cin, int cout, int h, int w) {
    if (!smc_conv3x3_wino_supported(n, cin, cout, h, w)) return 0;
    return std::max(wino_split_bytes(n, cin, cout, h, w) + wino_fold_bytes(n, cin, cout), wino_x3_bytes(n, cin, cout, h, w));
}

SMC_API int smc_conv3x3_wino_f32(const float* x, int n, int cin, int h, int w, float* y, int cout, const float* uw,
                                 const float* s_in, const smc_conv_epilogue* epi, void* stream) {
    return smc_conv3x3_wino_ws_f32(x, n, cin, h, w, y, cout, uw, s_in, epi, nullptr, 0, stream);
}

SMC_API int smc_conv3x3_wino_ws_f32(const float* x, int n, int cin, int h, int w, float* y, int cout, const float* uw,
                                    const float* s_in, const smc_conv_epilogue* epi, float* workspace,
                                    int64_t workspace_bytes, void* stream) {
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
    const int64_t items = (int64_t)n * p.gx * p.gy * p.ntn;
    SMC_CHECK(items < (1LL << 31), "smc_conv3x3_wino_f32: grid too large");
    hipStream_t st = smc::as_stream(stream);
    // split K when the caller passed the workspace smc_conv3x3_wino_workspace_size() asks for (without one: one
    // workgroup per item over the whole K range, as before)
    const int64_t need = smc_conv3x3_wino_workspace_size(n, cin, cout, h, w);
    const int64_t split_bytes = wino_split_bytes(n, cin, cout, h, w), fold_bytes = wino_fold_bytes(n, cin, cout);
    const bool ws_ok = need > 0 && workspace && workspace_bytes >= need;
    const bool modact_plain = p.mode == SMC_EPI_MODACT && !p.ext.residual;
    const bool ek1 = modact_plain && p.act == SMC_ACT_LRELU && p.alpha >= 0.f && p.alpha <= 1.f && p.clamp >= 0.f;
    const bool ek2 = modact_plain && p.act == SMC_ACT_LINEAR && p.clamp < 0.f;
    const bool noise_ok = !e.noise || ((reinterpret_cast<uintptr_t>(e.noise) & 15) == 0 && e.noise_nstride % 4 == 0);
    if (wino_x3_bytes(n, cin, cout, h, w) > 0 && ws_ok && noise_ok && (ek1 || (ek2 && g_wino_x3 >= 2))) {
        // the 32-channel layer on the bf16 matrix core: split U planes (x s[n, c] when scaled) into the workspace
        SMC_CHECK((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "smc_conv3x3_wino_ws_f32: workspace alignment");
        short* planes = reinterpret_cast<short*>(workspace);
        const int64_t total = (int64_t)(s_in ? n : 1) * (X3_UPLANE / 3);
        hipLaunchKernelGGL(wino_x3_pack_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(total, 256), 4096)),
                           dim3(256), 0, st, uw, s_in, planes, total);
        const int rc = smc::check_launch("smc_conv3x3_wino_ws_f32 (x3 planes)");
        if (rc != SMC_OK) return rc;
        const int64_t ns = s_in ? X3_UPLANE : 0;
        if (ek1) launch_wino_x3<1>(p, planes, ns, st);
        else launch_wino_x3<2>(p, planes, ns, st);
        return smc::check_launch("smc_conv3x3_wino_ws_f32 (x3)");
    }
    if (SMC_WINO_FOLD && s_in && fold_bytes > 0 && ws_ok) {
        float* uf = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + split_bytes);
        SMC_CHECK((reinterpret_cast<uintptr_t>(uf) & 15) == 0, "smc_conv3x3_wino_ws_f32: workspace alignment");
        const int per4 = cin * 4 * cout;   // float4 per image
        const int64_t total4 = (int64_t)n * per4;
        hipLaunchKernelGGL(wino_ufold_kernel, dim3((unsigned)std::min<int64_t>(smc::ceil_div(total4, 256), 4096)),
                           dim3(256), 0, st, reinterpret_cast<const float4*>(uw), s_in, reinterpret_cast<float4*>(uf),
                           cin, per4, total4);
        const int rc = smc::check_launch("smc_conv3x3_wino_ws_f32 (style fold)");
        if (rc != SMC_OK) return rc;
        p.uw = uf;
        p.u_nstride = (int64_t)cin * 16 * cout;
        p.s = nullptr;
        s_in = nullptr;
    }
    p.nsplit = 1;
    if (split_bytes > 0 && ws_ok) {
        SMC_CHECK((reinterpret_cast<uintptr_t>(workspace) & 7) == 0, "smc_conv3x3_wino_ws_f32: workspace alignment");
        p.nsplit = wino_nsplit(n, cin, cout, h, w);
        p.split_stride = (int64_t)n * cout * h * w;
        p.ws = workspace;
        launch_wino_s<3>(s_in != nullptr, tc, p, items, st);
        const int rc = smc::check_launch("smc_conv3x3_wino_ws_f32");
        if (rc != SMC_OK) return rc;
        return smc_modconv_epilogue_f32(workspace, p.nsplit, p.split_stride, y, n, cout, h, w, &e, stream);
    }
    // the synthesis' two MODACT forms get an epilogue body with the activation fixed at compile time
    if (ek1)
        launch_wino_s<1>(s_in != nullptr, tc, p, items, st);
    else if (ek2)
        launch_wino_s<2>(s_in != nullptr, tc, p, items, st);
    else
        launch_wino_s<0>(s_in != nullptr, tc, p, items, st);
    return smc::check_launch("smc_conv3x3_wino_f32");
}
