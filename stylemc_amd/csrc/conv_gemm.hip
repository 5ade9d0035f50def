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
#include <cstdlib>

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
    int nsplit;
    int64_t split_stride;
};

template <int WO, int WM, int TO, int TM, int BKT>
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

    // Prefetch registers.  Loads are unconditional (out-of-image taps read a valid dummy address) and
    // the style scale / zero mask is applied only when the tile is written to LDS, after the MFMAs:
    // nothing consumes a loaded value before the next barrier, so the loads overlap the whole step.
    float xr[XR];
    float4 sr[XR / 4];
    float4 wr[WPT];
    bool xok = false;
    const bool has_s = p.s != nullptr;
    const float* swhere = has_s ? sbase : p.x;  // any valid address when there is no scale

    auto load_step = [&](int ks) {
        const int t = ks / cpk;
        const int ci0 = (ks - t * cpk) * BKT;
        const int iy = ay + ph.dy[t], ix = bx + ph.dx[t];
        xok = mvalid && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w;
        const float* src = xbase + (int64_t)ci0 * in_hw + (xok ? (int64_t)iy * p.in_w + ix : 0);
#pragma unroll
        for (int r = 0; r < XR; ++r) xr[r] = src[r * in_hw];
#pragma unroll
        for (int r = 0; r < XR; r += 4) sr[r / 4] = *reinterpret_cast<const float4*>(swhere + (has_s ? ci0 + r : 0));
#pragma unroll
        for (int q = 0; q < WPT; ++q) {
            int v = tid + q * NT;
            v = v < WV ? v : v - WV;  // surplus threads re-read a valid vector; the store skips them
            const int wkk = v / (BO / 4), wc4 = v - wkk * (BO / 4);
            const int o = o0 + wc4 * 4;
            wr[q] = *reinterpret_cast<const float4*>(ph.wk + ((int64_t)t * p.cin + ci0 + wkk) * p.cout +
                                                     (o < p.cout ? o : 0));
        }
    };
    auto store_step = [&](int stage) {
        float* Ws = smem + stage * TILE;
        float* Xs = Ws + BKT * BO;
#pragma unroll
        for (int r = 0; r < XR; ++r) {
            const float4 sv = sr[r / 4];
            const float sc = has_s ? ((r & 3) == 0 ? sv.x : (r & 3) == 1 ? sv.y : (r & 3) == 2 ? sv.z : sv.w) : 1.f;
            Xs[(kr0 + r) * BM + ml] = xok ? xr[r] * sc : 0.f;
        }
#pragma unroll
        for (int q = 0; q < WPT; ++q) {
            const int v = tid + q * NT;
            const int wkk = v / (BO / 4), wc4 = v - wkk * (BO / 4);
            float4 w = wr[q];
            if (o0 + wc4 * 4 >= p.cout) w = make_float4(0.f, 0.f, 0.f, 0.f);  // cout = 16 in a 32-wide tile
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

    // ---- epilogue: lane owns column m, registers walk output channels
    const float nstr = p.noise_strength ? *p.noise_strength : 1.f;
    float* dst = p.nsplit > 1 ? p.y + (int64_t)split * p.split_stride : p.y;
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
        const int64_t plane = (int64_t)p.y_h * p.y_w;
        float nz = 0.f;
        if (p.nsplit == 1 && p.mode == SMC_EPI_MODACT && p.noise) nz = p.noise[en * p.noise_nstride + pix] * nstr;
#pragma unroll
        for (int i = 0; i < TO; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = o0 + wo * TO * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                if (o >= p.cout) continue;
                const int64_t idx = ((int64_t)en * p.cout + o) * plane + pix;
                const float v = acc[i][j][r];
                if (p.nsplit > 1 || p.mode == SMC_EPI_STORE) {
                    dst[idx] = v;
                } else {
                    if (p.u_save) p.u_save[idx] = v;
                    dst[idx] = smc::epi_y(v, p.d ? p.d[(int64_t)en * p.cout + o] : 1.f, nz,
                                          p.bias ? p.bias[o] : 0.f, p.act, p.alpha, p.gain, p.clamp);
                }
            }
        }
    }
}

struct Cfg {
    int bo, bm;
};

int pick_cfg(int cout, Cfg* c) {
    if (cout % 128 == 0) { *c = {128, 128}; return 0; }
    if (cout % 64 == 0) { *c = {64, 256}; return 1; }
    if (cout % 32 == 0) { *c = {32, 256}; return 2; }
    if (cout == 16) { *c = {32, 256}; return 2; }  // half-empty tile, masked
    return -1;
}

// Shared by the workspace query and the launch so both agree on the split.
int plan_split(int n, int cin, int cout, const smc_conv_phase* ph, int nph, const Cfg& c) {
    int64_t blocks = 0;
    int min_ks = 1 << 30;
    for (int i = 0; i < nph; ++i) {
        const int64_t M = (int64_t)n * ph[i].out_h * ph[i].out_w;
        blocks += smc::ceil_div(M, c.bm) * smc::ceil_div(cout, c.bo);
        const int ks = ph[i].ntaps * (cin / BK);
        if (ks < min_ks) min_ks = ks;
    }
    if (const char* f = getenv("SMC_FORCE_SPLIT")) {
        int v = atoi(f);
        if (v >= 1) return v < min_ks ? v : min_ks;
    }
    const int64_t target = 2LL * smc::device_cu_count();
    if (blocks >= target) return 1;
    int s = (int)smc::ceil_div(target, blocks > 0 ? blocks : 1);
    int cap = min_ks / 4;
    if (cap > 16) cap = 16;
    if (s > cap) s = cap;
    return s < 1 ? 1 : s;
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

SMC_API int64_t smc_conv_gemm_workspace_size(int n, int cin, int cout, int y_h, int y_w, const smc_conv_phase* phases,
                                             int nphases) {
    Cfg c;
    if (pick_cfg(cout, &c) < 0 || cin % BK != 0 || nphases < 1 || nphases > 4 || !phases) return 0;
    const int s = plan_split(n, cin, cout, phases, nphases, c);
    return s > 1 ? (int64_t)s * n * cout * y_h * y_w * (int64_t)sizeof(float) : 0;
}

SMC_API int smc_conv_gemm_f32(const float* x, int n, int cin, int in_h, int in_w, float* y, int cout, int y_h,
                              int y_w, const smc_conv_phase* phases, int nphases, const float* s_in,
                              const smc_conv_epilogue* epi, float* workspace, int64_t workspace_bytes,
                              void* stream) {
    int rc = validate(x, n, cin, in_h, in_w, y, cout, y_h, y_w, phases, nphases);
    if (rc != SMC_OK) return rc;
    Cfg c;
    const int cfg = pick_cfg(cout, &c);
    const int nsplit = plan_split(n, cin, cout, phases, nphases, c);
    const int64_t plane_elems = (int64_t)n * cout * y_h * y_w;
    if (nsplit > 1) {
        const int64_t need = nsplit * plane_elems * (int64_t)sizeof(float);
        SMC_CHECK(workspace && workspace_bytes >= need, "smc_conv_gemm_f32: workspace %lld < %lld bytes",
                  (long long)workspace_bytes, (long long)need);
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
    p.nsplit = nsplit;
    p.split_stride = plane_elems;

    hipStream_t st = smc::as_stream(stream);
    dim3 grid((unsigned)smc::ceil_div(max_m, c.bm), (unsigned)smc::ceil_div(cout, c.bo), (unsigned)(nphases * nsplit));
    // BK=32 halves the barriers per FLOP; it pays on the long-K 512-channel layers, BK=16 (more
    // workgroups per CU: 32-40 KB LDS vs 64-80 KB) on the high-resolution ones (tools/bench_gemm.py).
    bool k32 = cin % 32 == 0 && cin >= 512;
    if (const char* f = getenv("SMC_FORCE_BK")) k32 = k32 && atoi(f) != 16;  // A/B knob (tools/bench_gemm.py)
    if (cfg == 0) {
        if (k32) hipLaunchKernelGGL((conv_gemm_kernel<2, 2, 2, 2, 32>), grid, dim3(NT), 0, st, p);
        else hipLaunchKernelGGL((conv_gemm_kernel<2, 2, 2, 2, 16>), grid, dim3(NT), 0, st, p);
    } else if (cfg == 1) {
        if (k32) hipLaunchKernelGGL((conv_gemm_kernel<1, 4, 2, 2, 32>), grid, dim3(NT), 0, st, p);
        else hipLaunchKernelGGL((conv_gemm_kernel<1, 4, 2, 2, 16>), grid, dim3(NT), 0, st, p);
    } else {
        if (k32) hipLaunchKernelGGL((conv_gemm_kernel<1, 4, 1, 2, 32>), grid, dim3(NT), 0, st, p);
        else hipLaunchKernelGGL((conv_gemm_kernel<1, 4, 1, 2, 16>), grid, dim3(NT), 0, st, p);
    }
    rc = smc::check_launch("smc_conv_gemm_f32");
    if (rc != SMC_OK || nsplit == 1) return rc;
    return smc_modconv_epilogue_f32(workspace, nsplit, plane_elems, y, n, cout, y_h, y_w, &e, stream);
}
