// ArcFace IR-SE50 (the identity-loss backbone) on gfx950: forward + data gradient, native executor.
//
// Replaces the PyTorch modules the reference runs in IDLoss.extract_feats (id_loss/id_loss.py:20-24,
// id_loss/model_irse.py:10-49, id_loss/helpers.py:56-119).  Weights are frozen and eval-mode, so the
// backward is the gradient w.r.t. the input face only.
//
// Every 3x3 / 1x1 convolution runs on the MFMA implicit-GEMM kernel (smc_conv_gemm_f32) with the
// unit's elementwise work fused into its epilogue:
//   stem   : y0 = PReLU(BN(conv3x3(x)))                 -> mode PRELU (BN as scale_c / bias), saves z
//   unit   : y1 = PReLU(conv3x3(BN1(x)))                -> mode PRELU, saves the pre-activation u1
//            r  = BN2(conv3x3_s(y1))                     -> mode AFFINE
//            out = r * SE(r) + shortcut(x)               -> SE kernels + one combine pass, which also
//                                                           writes BN1 of the next unit (xbn)
//   output : BN2d -> flatten -> Linear -> BN1d           -> one GEMM (smc_linear_f32), all BNs folded
// Backward: the conv adjoints are again gather GEMMs (stride-2 forward -> 4-phase polyphase adjoint),
// with the BN scales folded into the packed adjoint weights, PReLU' fused as epilogue PRELU_GRAD, and
// the shortcut gradient added by the conv1 adjoint's strided-residual epilogue.
//
// Layout: fp32 NCHW (the reference layout), batch-major; SE vectors [n][C].
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "common.hpp"

namespace {

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

inline unsigned ew_grid(int64_t n) { return (unsigned)std::min<int64_t>(smc::ceil_div(n, 256), 16384); }

// out[plane] = scale * sum_p a[plane][p] * (b ? b[plane][p] : 1): one wave per plane, 8 loads per lane in flight
// (added in the plain lane order: i = lane, lane + 64, ...; + 0 past the plane is exact).
template <bool B>
__global__ __launch_bounds__(256) void plane_dot_kernel(const float* a, const float* b, float* out, int64_t planes,
                                                        int hw, float scale) {
    const int64_t pl = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (pl >= planes) return;
    const float* ap = a + pl * hw;
    const float* bp = B ? b + pl * hw : nullptr;
    float s = 0.f;
    for (int i0 = lane; i0 < hw; i0 += 64 * 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + 64 * k;
            const int ic = min(i, hw - 1);
            const float t = B ? ap[ic] * bp[ic] : ap[ic];
            v[k] = i < hw ? t : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
    }
    s = wsum(s);
    if (lane == 0) out[pl] = s * scale;
}

// Squeeze-and-excite.  The chain is latency-bound (a few KB of weights per sample, n <= 8 samples): the plane sums
// come from plane_dot_kernel (summed inside the excitation kernel instead, 8..16 planes per wave, the 14x14 / 7x7
// stages measured 10.5 / 17 us forward against 4.8 + 4.8 / 4.8 + 10 as two launches, tools/prof_irse.py); the
// excitation MLP is recomputed per channel block inside the combine / dr kernels below (it replaced a separate
// excitation launch per unit and direction).
// y = x * a[c] + b[c]
__global__ __launch_bounds__(256) void channel_affine_kernel(const float* x, const float* a, const float* b, float* y,
                                                             int C, int64_t hw, int64_t total) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)((i / hw) % C);
        y[i] = x[i] * a[c] + b[c];
    }
}

// SE excitation + combine (forward), one workgroup per (sample n, block of kSeCpb channels).  Each workgroup
// recomputes the sample's hidden layer h = relu(W1 m) (hid C-dots: a few KFLOP, cheaper than the launch of a separate
// excitation kernel on this latency-bound chain), then g = sigmoid(W2 h) for its channels, and applies
// out = r * g + shortcut (shortcut = sc (conv path) or x[n, c, s*y, s*x] (MaxPool2d(1, s))) and, optionally,
// xbn = out * a[c] + b[c] (BN1 of the next unit).  h (channel block 0) and g are stored for the backward.
constexpr int kSeCpb = 16;
constexpr int SE_RG = 4;    // excitation rows per wave in flight
constexpr int SE_MAXQ = 8;  // channels per lane (C <= 512, checked at pack time)
// pixel-range split of a plane for the SE kernels: at most 256 pixels (one per thread) of each of the kSeCpb channels
// per workgroup
inline unsigned se_zsplit(int64_t hw) { return (unsigned)std::max<int64_t>(1, smc::ceil_div(hw, 256)); }
__global__ __launch_bounds__(256) void se_fwd_combine_kernel(const float* m, const float* w1, const float* w2,
                                                             float* hout, float* gout, int C, int hid, const float* r,
                                                             const float* sc, const float* x, int s, int in_h,
                                                             int in_w, float* out, float* xbn, const float* a,
                                                             const float* b, int oh, int ow) {
    extern __shared__ float sm[];
    float* ms = sm;         // [C]
    float* hs = sm + C;     // [hid]
    float* gs = hs + hid;   // [kSeCpb]
    float* as = gs + kSeCpb;  // [kSeCpb] BN1 scale / shift of the next unit (xbn)
    float* bs = as + kSeCpb;
    const int n = blockIdx.x, c0 = blockIdx.y * kSeCpb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // this thread's pixel (se_zsplit: at most 256 pixels of a plane per workgroup), its kSeCpb channels of r and of
    // the shortcut loaded first: their round trips overlap the excitation MLP's
    const int ohw = oh * ow;
    const int chunk = (ohw + gridDim.z - 1) / gridDim.z;
    const int p = blockIdx.z * chunk + tid;
    const bool live = tid < chunk && p < ohw;
    const int pc = live ? p : 0;
    const int64_t nb = (int64_t)n * C + c0;
    float rv[kSeCpb], sv[kSeCpb];
    {
        int64_t xo = 0;
        if (!sc) {
            const int yy = pc / ow, xx = pc - yy * ow;
            xo = (int64_t)(s * yy) * in_w + s * xx;
        }
#pragma unroll
        for (int cl = 0; cl < kSeCpb; ++cl) {
            const int64_t i = (nb + cl) * ohw + pc;
            rv[cl] = r[i];
            sv[cl] = sc ? sc[i] : x[(nb + cl) * ((int64_t)in_h * in_w) + xo];
        }
    }
    for (int c = tid; c < C; c += 256) ms[c] = m[(int64_t)n * C + c];
    __syncthreads();
    // excitation layer 1, SE_RG rows per wave at a time with all their weight loads in flight (one row at a time, each
    // row's loads waited out a round trip: hid / 4 of them per workgroup)
    for (int j0 = wave; j0 < hid; j0 += 4 * SE_RG) {
        float wv[SE_RG][SE_MAXQ];
#pragma unroll
        for (int r = 0; r < SE_RG; ++r)
#pragma unroll
            for (int q = 0; q < SE_MAXQ; ++q) {
                const int j = min(j0 + 4 * r, hid - 1), c = min(lane + 64 * q, C - 1);
                wv[r][q] = w1[(int64_t)j * C + c];
            }
#pragma unroll
        for (int r = 0; r < SE_RG; ++r) {
            float t = 0.f;
#pragma unroll
            for (int q = 0; q < SE_MAXQ; ++q)
                if (lane + 64 * q < C) t += wv[r][q] * ms[lane + 64 * q];
            t = wsum(t);
            const int j = j0 + 4 * r;
            if (lane == 0 && j < hid) hs[j] = t > 0.f ? t : 0.f;
        }
    }
    __syncthreads();
    if (tid < kSeCpb) {
        const int c = c0 + tid;
        float t = 0.f;
#pragma unroll 8
        for (int j = 0; j < hid; ++j) t += w2[(int64_t)c * hid + j] * hs[j];
        as[tid] = xbn ? a[c] : 0.f;
        bs[tid] = xbn ? b[c] : 0.f;
        gs[tid] = 1.f / (1.f + expf(-t));
    }
    __syncthreads();
    // (the stores after every load: a load issued behind a store waits for its round trip)
    if (tid < kSeCpb) gout[(int64_t)n * C + c0 + tid] = gs[tid];
    if (blockIdx.y == 0 && blockIdx.z == 0 && tid < hid) hout[(int64_t)n * hid + tid] = hs[tid];
    if (live) {
#pragma unroll
        for (int cl = 0; cl < kSeCpb; ++cl) {
            const int64_t i = (nb + cl) * ohw + p;
            const float o = rv[cl] * gs[cl] + sv[cl];
            out[i] = o;
            if (xbn) xbn[i] = o * as[cl] + bs[cl];
        }
    }
}

// SE backward + dr (one workgroup per (sample, channel block), like se_fwd_combine_kernel): from dg = sum_hw dout * r
// (plane_dot_kernel) every workgroup recomputes dz = dg g (1 - g) and dh = (h > 0) W2^T dz for its sample, then
// dm = W1^T dh * inv_hw for its channels and dr = dout * g + dm.
__global__ __launch_bounds__(256) void se_bwd_dr_kernel(const float* dg, const float* g, const float* h,
                                                        const float* w1, const float* w2, int C, int hid, float inv_hw,
                                                        const float* dout, float* dr, int64_t hw) {
    extern __shared__ float sm[];
    float* dz = sm;          // [C]
    float* dh = sm + C;      // [hid]
    float* dms = dh + hid;   // [kSeCpb]
    float* gsb = dms + kSeCpb;  // [kSeCpb]
    const int n = blockIdx.x, c0 = blockIdx.y * kSeCpb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int chunk = (int)((hw + gridDim.z - 1) / gridDim.z);
    const int p = blockIdx.z * chunk + tid;
    const bool live = tid < chunk && p < hw;
    const int64_t nb = (int64_t)n * C + c0;
    float dv[kSeCpb];  // this thread's pixel of dout, loaded before the SE chain
#pragma unroll
    for (int cl = 0; cl < kSeCpb; ++cl) dv[cl] = dout[(nb + cl) * hw + (live ? p : 0)];
    for (int c = tid; c < C; c += 256) {
        const float gv = g[(int64_t)n * C + c];
        dz[c] = dg[(int64_t)n * C + c] * gv * (1.f - gv);
    }
    __syncthreads();
    for (int j0 = wave; j0 < hid; j0 += 4 * SE_RG) {  // SE_RG rows at a time, loads first (se_fwd_combine_kernel)
        float wv[SE_RG][SE_MAXQ], hv[SE_RG];
#pragma unroll
        for (int r = 0; r < SE_RG; ++r) {
            const int j = min(j0 + 4 * r, hid - 1);
            hv[r] = h[(int64_t)n * hid + j];
#pragma unroll
            for (int q = 0; q < SE_MAXQ; ++q) wv[r][q] = w2[(int64_t)min(lane + 64 * q, C - 1) * hid + j];
        }
#pragma unroll
        for (int r = 0; r < SE_RG; ++r) {
            float t = 0.f;
#pragma unroll
            for (int q = 0; q < SE_MAXQ; ++q)
                if (lane + 64 * q < C) t += wv[r][q] * dz[lane + 64 * q];
            t = wsum(t);
            const int j = j0 + 4 * r;
            if (lane == 0 && j < hid) dh[j] = hv[r] > 0.f ? t : 0.f;
        }
    }
    __syncthreads();
    if (tid < kSeCpb) {
        const int c = c0 + tid;
        float t = 0.f;
#pragma unroll 8
        for (int j = 0; j < hid; ++j) t += w1[(int64_t)j * C + c] * dh[j];
        dms[tid] = t * inv_hw;
        gsb[tid] = g[(int64_t)n * C + c];
    }
    __syncthreads();
    if (live) {
#pragma unroll
        for (int cl = 0; cl < kSeCpb; ++cl) dr[(nb + cl) * hw + p] = dv[cl] * gsb[cl] + dms[cl];
    }
}

// dz = dy * (z >= 0 ? 1 : alpha[c])
__global__ __launch_bounds__(256) void prelu_grad_kernel(const float* dy, const float* z, const float* alpha, float* dz,
                                                         int C, int64_t hw, int64_t total) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)((i / hw) % C);
        dz[i] = z[i] >= 0.f ? dy[i] : dy[i] * alpha[c];
    }
}

// Channel padding of the face [n][c_src][hw] <-> [n][c_dst][hw] (extra channels zero), either way.
__global__ __launch_bounds__(256) void channel_copy_kernel(const float* src, int c_src, float* dst, int c_dst,
                                                           int64_t hw, int64_t total /* n*c_dst*hw */) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t nc = i / hw;
        const int64_t p = i - nc * hw;
        const int c = (int)(nc % c_dst);
        const int64_t n = nc / c_dst;
        dst[i] = c < c_src ? src[(n * c_src + c) * hw + p] : 0.f;
    }
}

// ------------------------------------------------------------------------------------------- executor

inline int64_t rnd(int64_t n) { return (n + 63) & ~int64_t(63); }

struct UnitS {
    float *u1, *r, *h, *g;
};

int64_t unit_out_hw(const smc_irse_unit& u) { return (int64_t)(u.in_h / u.stride) * (u.in_w / u.stride); }

int64_t saved_floats(const smc_irse_net& net, int n, float* base, UnitS* per_unit, float** stem_z) {
    int64_t off = 0;
    auto seg = [&](int64_t k) {
        float* p = base ? base + off : nullptr;
        off += rnd(k);
        return p;
    };
    float* z = seg((int64_t)n * net.stem_cout * net.in_h * net.in_w);
    if (stem_z) *stem_z = z;
    for (int k = 0; k < net.n_units; ++k) {
        const smc_irse_unit& u = net.units[k];
        UnitS s;
        s.u1 = seg((int64_t)n * u.depth * u.in_h * u.in_w);
        s.r = seg((int64_t)n * u.depth * unit_out_hw(u));
        s.h = seg((int64_t)n * u.se_hidden);
        s.g = seg((int64_t)n * u.depth);
        if (per_unit) per_unit[k] = s;
    }
    return off;
}

struct Ws {
    float *pad, *xa, *xb, *xbn, *y1, *r, *sc, *m, *h, *g, *dm, *conv;
    int64_t conv_bytes;
};

int64_t max_act(const smc_irse_net& net) {
    int64_t m = (int64_t)net.stem_cout * net.in_h * net.in_w;
    m = std::max(m, (int64_t)net.stem_cin * net.in_h * net.in_w);
    for (int k = 0; k < net.n_units; ++k) {
        const smc_irse_unit& u = net.units[k];
        m = std::max(m, (int64_t)u.cin * u.in_h * u.in_w);
        m = std::max(m, (int64_t)u.depth * u.in_h * u.in_w);
    }
    return m;
}

int max_channels(const smc_irse_net& net) {
    int c = net.stem_cout;
    for (int k = 0; k < net.n_units; ++k) c = std::max(c, net.units[k].depth);
    return c;
}

int64_t conv_ws_need(const smc_irse_net& net, int n) {
    int64_t m = 0;
    auto q = [&](int cin, int cout, int yh, int yw, const smc_conv_phase* ph, int nph) {
        m = std::max(m, smc::conv_gemm_aux_workspace_size(n, cin, cout, yh, yw, ph, nph));
        if (nph == 1 && ph->wino_u) m = std::max(m, smc_wino_sp_workspace_size(n, cin, cout, yh, yw));
    };
    q(net.stem_cin, net.stem_cout, net.in_h, net.in_w, &net.stem_fwd, 1);
    q(net.stem_cout, net.stem_cin, net.in_h, net.in_w, &net.stem_bwd, 1);
    for (int k = 0; k < net.n_units; ++k) {
        const smc_irse_unit& u = net.units[k];
        const int oh = u.in_h / u.stride, ow = u.in_w / u.stride;
        q(u.cin, u.depth, u.in_h, u.in_w, &u.c1_fwd, 1);
        q(u.depth, u.cin, u.in_h, u.in_w, &u.c1_bwd, 1);
        q(u.depth, u.depth, oh, ow, &u.c2_fwd, 1);
        q(u.depth, u.depth, u.in_h, u.in_w, u.c2_bwd, u.c2_bwd_nphases);
        if (u.sc_conv) {
            q(u.cin, u.depth, oh, ow, &u.sc_fwd, 1);
            q(u.depth, u.cin, oh, ow, &u.sc_bwd, 1);
        }
    }
    const int64_t lin = std::max(smc_linear_workspace_size(n, net.feat, net.flat),
                                 smc_linear_workspace_size(n, net.flat, net.feat));
    return std::max(m, lin);
}

int64_t ws_floats(const smc_irse_net& net, int n, float* base, Ws* w) {
    int64_t off = 0;
    auto seg = [&](int64_t k) {
        float* p = base ? base + off : nullptr;
        off += rnd(k);
        return p;
    };
    const int64_t act = (int64_t)n * max_act(net);
    const int64_t vec = (int64_t)n * max_channels(net);
    Ws t{};
    t.pad = seg(act);
    t.xa = seg(act);
    t.xb = seg(act);
    t.xbn = seg(act);
    t.y1 = seg(act);
    t.r = seg(act);
    t.sc = seg(act);
    t.m = seg(vec);
    t.h = seg(vec);
    t.g = seg(vec);
    t.dm = seg(vec);
    const int64_t cb = conv_ws_need(net, n);
    t.conv = seg(smc::ceil_div(cb, 4) + 1);
    t.conv_bytes = cb;
    if (w) *w = t;
    return off;
}

int net_validate(const smc_irse_net* net, int n) {
    SMC_CHECK(net && net->units && net->n_units >= 1 && n >= 1, "smc_irse: bad net / batch");
    SMC_CHECK(net->stem_cin >= net->img_ch && net->stem_cin % 16 == 0, "smc_irse: stem_cin must pad img_ch to 16k");
    SMC_CHECK(net->fc_wt && net->fc_w && net->flat % 32 == 0 && net->feat % 32 == 0, "smc_irse: bad output layer");
    for (int k = 0; k < net->n_units; ++k) {
        const smc_irse_unit& u = net->units[k];
        SMC_CHECK(u.stride == 1 || u.stride == 2, "smc_irse: unit %d stride %d", k, u.stride);
        SMC_CHECK(u.in_h % u.stride == 0 && u.in_w % u.stride == 0, "smc_irse: unit %d odd size", k);
        SMC_CHECK(u.se_hidden >= 1 && u.se_w1 && u.se_w2 && u.bn1_a && u.bn2_a && u.prelu, "smc_irse: unit %d", k);
        SMC_CHECK(u.depth % kSeCpb == 0, "smc_irse: unit %d depth %d not a multiple of %d", k, u.depth, kSeCpb);
        SMC_CHECK(u.depth <= 64 * SE_MAXQ, "smc_irse: unit %d depth %d > %d", k, u.depth, 64 * SE_MAXQ);
        SMC_CHECK(u.se_hidden <= 256, "smc_irse: unit %d SE hidden width %d > 256", k, u.se_hidden);
        SMC_CHECK(u.sc_conv || u.cin == u.depth, "smc_irse: unit %d identity shortcut needs cin == depth", k);
        SMC_CHECK(u.c2_bwd_nphases == (u.stride == 2 ? 4 : 1), "smc_irse: unit %d adjoint phases", k);
    }
    const smc_irse_unit& last = net->units[net->n_units - 1];
    SMC_CHECK((int64_t)last.depth * unit_out_hw(last) == net->flat, "smc_irse: flat %d mismatch", net->flat);
    return SMC_OK;
}

smc_conv_epilogue epi_mode(int mode) {
    smc_conv_epilogue e{};
    e.mode = mode;
    e.act = SMC_ACT_LINEAR;
    e.gain = 1.f;
    e.clamp = -1.f;
    return e;
}

#define SMC_TRY(expr)                  \
    do {                               \
        const int rc_ = (expr);        \
        if (rc_ != SMC_OK) return rc_; \
    } while (0)

}  // namespace

SMC_API int64_t smc_irse_saved_floats(const smc_irse_net* net, int n) {
    if (net_validate(net, n) != SMC_OK) return -1;
    return saved_floats(*net, n, nullptr, nullptr, nullptr);
}

SMC_API int64_t smc_irse_workspace_bytes(const smc_irse_net* net, int n) {
    if (net_validate(net, n) != SMC_OK) return -1;
    return ws_floats(*net, n, nullptr, nullptr) * (int64_t)sizeof(float);
}

SMC_API int smc_irse_forward_f32(const smc_irse_net* net, const float* img, int n, float* feat, float* saved,
                                 float* workspace, int64_t workspace_bytes, void* stream) {
    SMC_TRY(net_validate(net, n));
    SMC_CHECK(img && feat && workspace, "smc_irse_forward_f32: null pointer");
    SMC_CHECK(workspace_bytes >= ws_floats(*net, n, nullptr, nullptr) * (int64_t)sizeof(float),
              "smc_irse_forward_f32: workspace too small");
    hipStream_t st = smc::as_stream(stream);
    Ws w;
    ws_floats(*net, n, workspace, &w);
    std::vector<UnitS> us(net->n_units);
    float* stem_z = nullptr;
    if (saved) saved_floats(*net, n, saved, us.data(), &stem_z);
    auto conv = [&](const float* x, int cin, int ih, int iw, float* y, int cout, int yh, int yw,
                    const smc_conv_phase* ph, int nph, const smc_conv_epilogue& e) {
        if (nph == 1 && ph->wino_u && ih == yh && iw == yw && smc_wino_sp_supported(n, cin, cout, ih, iw))
            return smc_conv3x3_wino_sp_f32(x, n, cin, ih, iw, y, cout, ph->wino_u, &e, w.conv, w.conv_bytes, stream);
        return smc::conv_gemm_aux(x, n, cin, ih, iw, y, cout, yh, yw, ph, nph, nullptr, &e, w.conv, w.conv_bytes,
                                 stream);
    };
    const int H = net->in_h, W = net->in_w;
    const int64_t hw0 = (int64_t)H * W;
    // stem: pad the face to stem_cin channels, conv3x3 -> BN -> PReLU, then BN1 of unit 0
    int64_t tot = (int64_t)n * net->stem_cin * hw0;
    hipLaunchKernelGGL(channel_copy_kernel, dim3(ew_grid(tot)), dim3(256), 0, st, img, net->img_ch, w.pad,
                       net->stem_cin, hw0, tot);
    SMC_TRY(smc::check_launch("irse pad"));
    smc_conv_epilogue e = epi_mode(SMC_EPI_PRELU);
    e.scale_c = net->stem_bn_a;
    e.bias = net->stem_bn_b;
    e.alpha_c = net->stem_prelu;
    e.u_save = stem_z;
    float* x = w.xa;
    SMC_TRY(conv(w.pad, net->stem_cin, H, W, x, net->stem_cout, H, W, &net->stem_fwd, 1, e));
    tot = (int64_t)n * net->stem_cout * hw0;
    hipLaunchKernelGGL(channel_affine_kernel, dim3(ew_grid(tot)), dim3(256), 0, st, x, net->units[0].bn1_a,
                       net->units[0].bn1_b, w.xbn, net->stem_cout, hw0, tot);
    SMC_TRY(smc::check_launch("irse bn1"));

    for (int k = 0; k < net->n_units; ++k) {
        const smc_irse_unit& u = net->units[k];
        const int oh = u.in_h / u.stride, ow = u.in_w / u.stride;
        const int64_t ohw = (int64_t)oh * ow;
        float* r = saved ? us[k].r : w.r;
        float* hbuf = saved ? us[k].h : w.h;
        float* gbuf = saved ? us[k].g : w.g;
        // y1 = PReLU(conv3x3(xbn))
        e = epi_mode(SMC_EPI_PRELU);
        e.alpha_c = u.prelu;
        e.u_save = saved ? us[k].u1 : nullptr;
        SMC_TRY(conv(w.xbn, u.cin, u.in_h, u.in_w, w.y1, u.depth, u.in_h, u.in_w, &u.c1_fwd, 1, e));
        // r = BN2(conv3x3_s(y1))
        e = epi_mode(SMC_EPI_AFFINE);
        e.scale_c = u.bn2_a;
        e.bias = u.bn2_b;
        SMC_TRY(conv(w.y1, u.depth, u.in_h, u.in_w, r, u.depth, oh, ow, &u.c2_fwd, 1, e));
        // SE: m = mean_hw(r); h = relu(W1 m); g = sigmoid(W2 h)
        const int64_t planes = (int64_t)n * u.depth;
        hipLaunchKernelGGL(plane_dot_kernel<false>, dim3((unsigned)smc::ceil_div(planes, 4)), dim3(256), 0, st, r,
                           (const float*)nullptr, w.m, planes, (int)ohw, 1.f / (float)ohw);
        // shortcut
        const float* sc = nullptr;
        if (u.sc_conv) {
            e = epi_mode(SMC_EPI_AFFINE);
            e.scale_c = u.sc_a;
            e.bias = u.sc_b;
            SMC_TRY(conv(x, u.cin, u.in_h, u.in_w, w.sc, u.depth, oh, ow, &u.sc_fwd, 1, e));
            sc = w.sc;
        }
        // g = sigmoid(W2 relu(W1 m)); out = r * g + shortcut (+ BN1 of the next unit): one fused launch
        float* out = x == w.xa ? w.xb : w.xa;
        const bool next = k + 1 < net->n_units;
        hipLaunchKernelGGL(se_fwd_combine_kernel, dim3(n, u.depth / kSeCpb, se_zsplit(ohw)), dim3(256),
                           sizeof(float) * (u.depth + u.se_hidden + 3 * kSeCpb), st, w.m, u.se_w1, u.se_w2, hbuf, gbuf,
                           u.depth, u.se_hidden, r, sc, x, u.stride, u.in_h, u.in_w, out, next ? w.xbn : nullptr,
                           next ? net->units[k + 1].bn1_a : nullptr, next ? net->units[k + 1].bn1_b : nullptr, oh, ow);
        SMC_TRY(smc::check_launch("irse se + combine"));
        x = out;
    }
    // output layer: folded BN2d + Linear + BN1d
    smc_linear_epilogue le{};
    le.bias = net->fc_b;
    return smc_linear_f32(x, net->flat, net->fc_wt, net->feat, feat, net->feat, n, net->feat, net->flat, &le, w.conv,
                          w.conv_bytes, stream);
}

SMC_API int smc_irse_backward_f32(const smc_irse_net* net, const float* dfeat, int n_saved, int n, const float* saved,
                                  float* dimg, float* workspace, int64_t workspace_bytes, void* stream) {
    SMC_TRY(net_validate(net, n_saved));
    SMC_CHECK(dfeat && saved && dimg && workspace, "smc_irse_backward_f32: null pointer");
    SMC_CHECK(n >= 1 && n <= n_saved, "smc_irse_backward_f32: n %d not in [1, %d]", n, n_saved);
    SMC_CHECK(workspace_bytes >= ws_floats(*net, n, nullptr, nullptr) * (int64_t)sizeof(float),
              "smc_irse_backward_f32: workspace too small");
    hipStream_t st = smc::as_stream(stream);
    Ws w;
    ws_floats(*net, n, workspace, &w);
    // saved activations laid out for n_saved faces; the leading n are differentiated ([n_saved][C][H][W] prefixes)
    std::vector<UnitS> us(net->n_units);
    float* stem_z = nullptr;
    saved_floats(*net, n_saved, const_cast<float*>(saved), us.data(), &stem_z);
    auto conv = [&](const float* x, int cin, int ih, int iw, float* y, int cout, int yh, int yw,
                    const smc_conv_phase* ph, int nph, const smc_conv_epilogue& e) {
        if (nph == 1 && ph->wino_u && ih == yh && iw == yw && smc_wino_sp_supported(n, cin, cout, ih, iw))
            return smc_conv3x3_wino_sp_f32(x, n, cin, ih, iw, y, cout, ph->wino_u, &e, w.conv, w.conv_bytes, stream);
        return smc::conv_gemm_aux(x, n, cin, ih, iw, y, cout, yh, yw, ph, nph, nullptr, &e, w.conv, w.conv_bytes,
                                 stream);
    };
    // d(flattened last output) = dfeat @ fc_w
    float* dx = w.xa;
    SMC_TRY(smc_linear_f32(dfeat, net->feat, net->fc_w, net->flat, dx, net->flat, n, net->flat, net->feat, nullptr,
                           w.conv, w.conv_bytes, stream));
    for (int k = net->n_units - 1; k >= 0; --k) {
        const smc_irse_unit& u = net->units[k];
        const int oh = u.in_h / u.stride, ow = u.in_w / u.stride;
        const int64_t ohw = (int64_t)oh * ow;
        const int64_t planes = (int64_t)n * u.depth;
        const float* dout = dx;
        // SE + combine backward: dg = sum_hw dout * r; dm = SE chain; dr = dout * g + dm
        hipLaunchKernelGGL(plane_dot_kernel<true>, dim3((unsigned)smc::ceil_div(planes, 4)), dim3(256), 0, st, dout,
                           us[k].r, w.m, planes, (int)ohw, 1.f);
        hipLaunchKernelGGL(se_bwd_dr_kernel, dim3(n, u.depth / kSeCpb, se_zsplit(ohw)), dim3(256),
                           sizeof(float) * (u.depth + u.se_hidden + 2 * kSeCpb), st, w.m, us[k].g, us[k].h, u.se_w1,
                           u.se_w2, u.depth, u.se_hidden, 1.f / (float)ohw, dout, w.r, ohw);
        SMC_TRY(smc::check_launch("irse se bwd"));
        // du1 = PReLU'(u1) * conv2^T(dr)   (BN2 scale folded into the adjoint weights)
        smc_conv_epilogue e = epi_mode(SMC_EPI_PRELU_GRAD);
        e.alpha_c = u.prelu;
        e.act_ref = us[k].u1;
        SMC_TRY(conv(w.r, u.depth, oh, ow, w.y1, u.depth, u.in_h, u.in_w, u.c2_bwd, u.c2_bwd_nphases, e));
        // shortcut gradient: dout itself (MaxPool2d(1, s)) or the 1x1 conv adjoint (compact grid)
        const float* res = dout;
        if (u.sc_conv) {
            SMC_TRY(conv(dout, u.depth, oh, ow, w.sc, u.cin, oh, ow, &u.sc_bwd, 1, epi_mode(SMC_EPI_STORE)));
            res = w.sc;
        }
        // dx = conv1^T(du1) (BN1 scale folded) + shortcut gradient scattered at stride s
        float* dnew = dx == w.xa ? w.xb : w.xa;
        e = epi_mode(SMC_EPI_STORE);
        e.residual = res;
        e.residual_stride = u.stride;
        SMC_TRY(conv(w.y1, u.depth, u.in_h, u.in_w, dnew, u.cin, u.in_h, u.in_w, &u.c1_bwd, 1, e));
        dx = dnew;
    }
    // stem: dz = dy0 * PReLU'(z); d(padded face) = conv^T(dz) (BN scale folded); drop the pad channels
    const int H = net->in_h, W = net->in_w;
    const int64_t hw0 = (int64_t)H * W;
    int64_t tot = (int64_t)n * net->stem_cout * hw0;
    hipLaunchKernelGGL(prelu_grad_kernel, dim3(ew_grid(tot)), dim3(256), 0, st, dx, stem_z, net->stem_prelu, w.y1,
                       net->stem_cout, hw0, tot);
    SMC_TRY(smc::check_launch("irse stem prelu'"));
    SMC_TRY(conv(w.y1, net->stem_cout, H, W, w.pad, net->stem_cin, H, W, &net->stem_bwd, 1, epi_mode(SMC_EPI_STORE)));
    tot = (int64_t)n * net->img_ch * hw0;
    hipLaunchKernelGGL(channel_copy_kernel, dim3(ew_grid(tot)), dim3(256), 0, st, w.pad, net->stem_cin, dimg,
                       net->img_ch, hw0, tot);
    return smc::check_launch("irse unpad");
}
