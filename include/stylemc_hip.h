/*
 * stylemc_hip.h -- C ABI of the MI355X (gfx950) kernels for StyleMC's find_direction hot path.
 *
 * Conventions (all entry points):
 *   - extern "C", plain device pointers + explicit sizes, fp32 NCHW-contiguous tensors.
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream).  Kernels are
 *     enqueued asynchronously; nothing synchronises the host.
 *   - Return SMC_OK (0) or an SMC_ERR_* code; smc_last_error() returns a thread-local message.
 *   - The caller owns every buffer.  Nothing allocates device memory internally: ops that need
 *     scratch space take a `workspace` whose size the matching *_workspace_size() query returns.
 *   - Pointers documented "may be NULL" mean "absent" (the reference passes empty tensors for that,
 *     torch_utils/ops/bias_act.py:39,150-157).
 *
 * Each entry point cites the reference interface it replaces.
 */
#ifndef STYLEMC_HIP_H
#define STYLEMC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMC_ABI_VERSION 4

#define SMC_OK 0
#define SMC_ERR_INVALID 1     /* bad argument / shape (reference: TORCH_CHECK -> RuntimeError)   */
#define SMC_ERR_UNSUPPORTED 2 /* valid request this build has no kernel for                       */
#define SMC_ERR_LAUNCH 3      /* hipGetLastError() after a launch was not hipSuccess             */

/* activation codes: identical to the reference's cuda_idx (torch_utils/ops/bias_act.py:23-33) */
#define SMC_ACT_LINEAR 1
#define SMC_ACT_RELU 2
#define SMC_ACT_LRELU 3
#define SMC_ACT_TANH 4
#define SMC_ACT_SIGMOID 5
#define SMC_ACT_ELU 6
#define SMC_ACT_SELU 7
#define SMC_ACT_SOFTPLUS 8
#define SMC_ACT_SWISH 9

int smc_abi_version(void);

/* Batch-invariant planning.  Split-K factors, tile configurations and channel splits are normally chosen per call
 * to fill the chip, so the same image computed in a batch of 2 and in a batch of 4 may be summed in a different fp32
 * order.  After smc_set_plan_batch(plan, local) every such decision for a call on n images (m rows of a token-major
 * GEMM) is made as for n * plan / local images (m * plan / local rows): a data-parallel shard of `local` images of
 * a `plan`-image batch then computes each image bit for bit as the whole batch does.  (0, 0) restores the default.
 * Process-wide; set it from the thread that enqueues the work, before enqueueing it. */
int smc_set_plan_batch(int plan, int local);
const char* smc_last_error(void);

/* ---------------------------------------------------------------------------------------------
 * bias_act -- replaces the pybind `_plugin.bias_act(x, b, xref, yref, dy, grad, dim, act, alpha,
 * gain, clamp)` of torch_utils/ops/bias_act.cpp:32-90 (called at bias_act.py:153,182,201).
 *   bias index of element i = (i / step_b) % size_b   (step_b = x.stride(dim), size_b = b.numel())
 *   grad 0: y = clamp(act(x + b) * gain)
 *   grad 1: y = d/dx   (x holds the incoming gradient, xref/yref the saved forward tensors)
 *   grad 2: second-order term (only for activations with a 2nd derivative)
 * b, xref, yref, dy may be NULL.  clamp < 0 disables clamping.
 */
int smc_bias_act_f32(const float* x, const float* b, const float* xref, const float* yref, const float* dy,
                     float* y, int64_t numel, int64_t size_b, int64_t step_b, int grad, int act, float alpha,
                     float gain, float clamp, void* stream);

/* ---------------------------------------------------------------------------------------------
 * upfirdn2d -- replaces `_plugin.upfirdn2d(x, f, upx, upy, downx, downy, padx0, padx1, pady0, pady1,
 * flip, gain)` of torch_utils/ops/upfirdn2d.cpp:16-94 (called at upfirdn2d.py:237-240).
 *   x [major, in_h, in_w], f [fh, fw] (device fp32), y [major, out_h, out_w] with
 *   out_h = (in_h*upy + pady0 + pady1 - fh + downy) / downy  (checked).
 *   flip = 0: convolution (taps flipped), 1: correlation.  Negative padding crops.
 */
int smc_upfirdn2d_f32(const float* x, const float* f, float* y, int64_t major, int in_h, int in_w, int out_h,
                      int out_w, int fh, int fw, int upx, int upy, int downx, int downy, int padx0, int padx1,
                      int pady0, int pady1, int flip, float gain, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Modulated convolution (replaces the cuDNN grouped F.conv2d / F.conv_transpose2d of
 * torch_utils/ops/conv2d_resample.py:29-54,125-147 driven by the upstream modulated_conv2d).
 * The build uses the non-fused form: x*s -> shared-weight conv -> *d[n,o] -> +noise -> bias_act,
 * mathematically identical to the reference's fused grouped conv, without per-sample weights.
 *
 * smc_conv_gemm_f32 is an implicit-GEMM "gather convolution" on MFMA (v_mfma_f32_32x32x2_f32):
 *   for every phase p, output position (a, b) in [0,out_h) x [0,out_w) of sample n:
 *     acc[n,o,a,b] = sum_{t < ntaps, i < cin} W_p[t][i][o] * s[n,i] * x[n, i, a*in_stride + tap_dy[t],
 *                                                                      b*in_stride + tap_dx[t]]
 *   (out-of-range input reads are 0), written to y[n, o, out_oy + out_sy*a, out_ox + out_sx*b]
 *   through the epilogue.  One phase = a plain (strided) conv; four phases = the polyphase
 *   stride-2 transposed conv of the up=2 layers.
 */
typedef struct {
    int ntaps;            /* 1..9                                             */
    int tap_dy[9];
    int tap_dx[9];
    int in_stride;        /* 1 or 2                                           */
    int out_h, out_w;     /* output grid of this phase                        */
    int out_oy, out_ox;   /* offset of the grid in y                          */
    int out_sy, out_sx;   /* stride of the grid in y                          */
    const float* wk;      /* [ntaps][cin][cout] packed weights                */
    const float* wino_u;  /* optional (IR-SE50 executor): Winograd F(2x2) taps of a 9-tap 3x3 stride-1 'same'
                             phase from smc_wino_taps_f32, used for its <= 16x16 planes; NULL = none        */
    const void* wk_x3;    /* optional: wk split into three bf16 terms (smc_conv_weights_x3).  When every phase of a
                             call has them, the LDS-DMA GEMM runs the fp32 products as split-bf16 MFMAs (each
                             operand a = a0 + a1 + a2 exactly, the six products a_i b_j with i + j <= 2: error per
                             product <= 2^-23 |a b|, fp32-class) at 6/16 of the fp32 MFMA's cost; the per-sample
                             weights of a style-scaled call are split on the fly.  NULL = exact-fp32 MFMA        */
} smc_conv_phase;

/* Bytes of the split-bf16 planes of a phase's [ntaps][cin][cout] weights (cin % 16 == 0; 0 = unsupported), and
 * the planes themselves: layout [ntaps][cin/16][3 terms][2 octets][cout][8] bf16, term s of wk[t][16c + 8q + e][o]
 * at ((((t*(cin/16) + c)*3 + s)*2 + q)*cout + o)*8 + e; wk_x3 16-B aligned. */
int64_t smc_conv_weights_x3_bytes(int ntaps, int cin, int cout);
int smc_conv_weights_x3(const float* wk, int ntaps, int cin, int cout, void* wk_x3, void* stream);

#define SMC_EPI_STORE 0   /* y = acc                                                           */
#define SMC_EPI_MODACT 1  /* u = acc; y = clamp(act(u*d[n,o] + noise*strength + bias[o])*gain)  */
/* modes of the IR-SE50 (ArcFace) convolutions, id_loss/model_irse.py:                           */
#define SMC_EPI_PRELU 2      /* z = acc*scale_c[o] + bias[o]; u_save = z; y = z >= 0 ? z : alpha_c[o]*z */
#define SMC_EPI_PRELU_GRAD 3 /* y = acc * (act_ref >= 0 ? 1 : alpha_c[o])  (PReLU backward)          */
#define SMC_EPI_AFFINE 4     /* y = acc*scale_c[o] + bias[o]  (eval-mode BatchNorm)                  */

typedef struct {
    int mode;                      /* SMC_EPI_*                                                  */
    const float* d;                /* [n][cout] demodulation coefficients, may be NULL (=1)       */
    const float* noise;            /* may be NULL; element = noise[n*noise_nstride + y*W + x]     */
    int64_t noise_nstride;         /* 0 for the const [H, W] noise buffer                          */
    const float* noise_strength;   /* device scalar, may be NULL (=1)                             */
    const float* bias;             /* [cout], may be NULL                                          */
    int act;                       /* SMC_ACT_* (linear / relu / lrelu on this path)               */
    float alpha, gain, clamp;      /* clamp < 0: none                                              */
    float* u_save;                 /* may be NULL: stores u (pre-demod acc), layout of y            */
    const float* scale_c;          /* [cout] per-channel scale (multiplies d in MODACT), may be NULL */
    const float* alpha_c;          /* [cout] PReLU slopes (PRELU / PRELU_GRAD)                      */
    const float* act_ref;          /* PRELU_GRAD: the saved pre-activation, layout of y             */
    const float* residual;         /* may be NULL: added last, [n][cout][y_h/rs][y_w/rs] at the      */
    int residual_stride;           /*   positions with y % rs == 0 and x % rs == 0 (rs 0 -> 1)      */
    int grad_from_y;               /* MODACT backward entry points (act_bwd, blur_act_bwd): their `u`
                                    * argument holds the forward OUTPUT y instead of u -- the
                                    * activation mask needs only y, so a layer whose styles need no
                                    * gradient saves no u -- and dd must be NULL (it needs u)         */
} smc_conv_epilogue;

/* bytes of workspace smc_conv_gemm_f32 needs for these sizes (0 = none). */
/* nonzero if the last smc_conv_gemm_f32 call of this thread launched the split-bf16 kernels (the phases carried wk_x3
 * and the LDS-DMA tiles took the shape; 2: the 256-channel wide tile), 0 if it ran exact-fp32 products (timing /
 * roofline attribution, tests). */
int smc_conv_gemm_last_x3(void);
int64_t smc_conv_gemm_workspace_size(int n, int cin, int cout, int y_h, int y_w, const smc_conv_phase* phases,
                                     int nphases);

int smc_conv_gemm_f32(const float* x, int n, int cin, int in_h, int in_w, float* y, int cout, int y_h, int y_w,
                      const smc_conv_phase* phases, int nphases, const float* s_in, const smc_conv_epilogue* epi,
                      float* workspace, int64_t workspace_bytes, void* stream);

/* Winograd F(2x2, 3x3) form of the 3x3 stride-1 pad-1 convolution (the SynthesisLayer conv1 forward and its
 * data gradient -- the one-phase smc_conv_gemm_f32 call with taps (dy, dx) in {-1,0,1}^2), same operands and
 * epilogue semantics (modes STORE / MODACT / PRELU / PRELU_GRAD / AFFINE, no split-K workspace):
 *   acc[n,o,y,x] = sum_{c,dy,dx} W[o][c][dy+1][dx+1] * s[n,c] * x[n, c, y+dy, x+dx]
 * uw holds the transformed taps written by smc_wino_weights_f32 (flip 0 for this forward form).
 * smc_conv3x3_wino_supported() says whether a shape has a kernel (cin % 8, cout % 32, w % 4 == 0, w >= 32,
 * h even, input < 2 GiB); unsupported shapes return SMC_ERR_UNSUPPORTED. */
int smc_conv3x3_wino_supported(int n, int cin, int cout, int h, int w);
int smc_conv3x3_wino_f32(const float* x, int n, int cin, int h, int w, float* y, int cout, const float* uw,
                         const float* s_in, const smc_conv_epilogue* epi, void* stream);
/* The same conv with split K for grids too small to fill the chip (smc_conv3x3_wino_workspace_size() > 0: fewer than
 * 512 work items): K splits write raw partial tiles into `workspace` and smc_modconv_epilogue_f32 sums them and
 * applies `epi`.  A NULL / too small workspace runs the single-pass kernel. */
int64_t smc_conv3x3_wino_workspace_size(int n, int cin, int cout, int h, int w);
int smc_conv3x3_wino_ws_f32(const float* x, int n, int cin, int h, int w, float* y, int cout, const float* uw,
                            const float* s_in, const smc_conv_epilogue* epi, float* workspace, int64_t workspace_bytes,
                            void* stream);
/* Experimental split-bf16 F(2x2) for cin = cout = 32, w % 64 == 0, h % 4 == 0 (the r = 1024 conv1), taken by
 * smc_conv3x3_wino_ws_f32 with its workspace when enabled: mode 0 off (the default: slower in the full step,
 * profiles/r06/wino_x3/README), 1 for the MODACT lrelu form, 2 also for the linear form.  Process-wide; returns the
 * previous mode.  The workspace size follows the mode in force. */
int smc_set_wino_x3(int mode);
/* w [cout][cin][3][3] -> uw [K][4][N][4] floats (16 * cin * cout, 16-B aligned), U = G g G^T per (k, n):
 * flip = 0: K = cin, N = cout, g = w[n][k] (the forward correlation);
 * flip = 1: K = cout, N = cin, g = w[k][n] rotated 180 degrees (the data gradient, conv^T). */
int smc_wino_weights_f32(const float* w, int cout, int cin, int flip, float* uw, void* stream);

/* Winograd F(4x4, 3x3) form of the same convolution (4x4 output tiles, 36 multiplies per channel pair instead of
 * 144; interpolation points 0, +-1, +-2), same operands and epilogue semantics as smc_conv3x3_wino_f32 and the same
 * C-ABI contract (replaces the same grouped conv2d of conv2d_resample.py:147-154).  uw holds the taps written by
 * smc_wino4_weights_f32.  smc_conv3x3_wino4_supported(): cin % 4 == 0, w % 64 == 0, h % 8 == 0, cout % 64 == 0;
 * input and taps < 2 GiB.  x, y, uw, u_save and noise 16-B aligned (noise_nstride % 4 == 0). */
int smc_conv3x3_wino4_supported(int n, int cin, int cout, int h, int w);
int smc_conv3x3_wino4_f32(const float* x, int n, int cin, int h, int w, float* y, int cout, const float* uw,
                          const float* s_in, const smc_conv_epilogue* epi, void* stream);
/* w [cout][cin][3][3] -> uw [K][9][N][4] floats (36 * cin * cout, 16-B aligned), U = G g G^T (6x6) per (k, n) computed
 * in fp64 and rounded once, element (a, b) at xi = 6 b + a; flip as for smc_wino_weights_f32. */
int smc_wino4_weights_f32(const float* w, int cout, int cin, int flip, float* uw, void* stream);

/* Small-plane Winograd F(2x2, 3x3) with split-K for the IR-SE50 14x14 / 7x7 stages (id_loss/model_irse.py,
 * helpers.py:86-119): the 3x3 stride-1 'same' conv of a 9-tap phase, x [n][cin][h][w] -> y [n][cout][h][w], any
 * smc_conv_epilogue mode applied by the split-K reduction (smc_modconv_epilogue_f32).  uw from smc_wino_taps_f32
 * ([cin][4][cout][4]).  Supported: h, w in [2, 16], cin % 8 == 0 (>= 16), cout % 32 == 0. */
int smc_wino_sp_supported(int n, int cin, int cout, int h, int w);
int64_t smc_wino_sp_workspace_size(int n, int cin, int cout, int h, int w);
int smc_wino_taps_f32(const smc_conv_phase* phase, int cin, int cout, float* uw, void* stream);
int smc_conv3x3_wino_sp_f32(const float* x, int n, int cin, int h, int w, float* y, int cout, const float* uw,
                            const smc_conv_epilogue* epi, float* workspace, int64_t workspace_bytes, void* stream);

/* Apply the modconv epilogue to a raw accumulator tensor, summing `nsplit` partial planes
 * (src + k*split_stride).  src/y/u_save: [n, c, h, w]. */
int smc_modconv_epilogue_f32(const float* src, int nsplit, int64_t split_stride, float* y, int n, int c, int h,
                             int w, const smc_conv_epilogue* epi, void* stream);

/* Fused conv0 epilogue: U = upfirdn2d(T, f, pad=(padx0,pady0 on both sides), gain=fgain) (1:1 FIR),
 * then the modconv epilogue (u_save receives U).  T: [n, c, t_h, t_pitch] of which the first t_w columns
 * are the image (t_pitch = 0: t_w; a pitch that is a multiple of 4 -- the transposed conv's odd 2h + 1
 * width padded -- takes the 16-B load path), may be `nsplit` partial planes; y: [n, c, y_h, y_w].  Only
 * the 4x4 FIR of the [1,3,3,1] resample filter has a fused kernel; other sizes return SMC_ERR_UNSUPPORTED.
 * f = NULL (fh = fw = 4): the built-in setup_filter([1,3,3,1]) taps as compile-time constants (bit-identical to
 * passing that filter; the kernel then holds no taps in registers). */
int smc_modconv_blur_act_f32(const float* t, int nsplit, int64_t split_stride, float* y, int n, int c, int t_h,
                             int t_w, int t_pitch, int y_h, int y_w, const float* f, int fh, int fw, int padx0,
                             int pady0, float fgain, int flip, const smc_conv_epilogue* epi, void* stream);

/* Backward of smc_modconv_blur_act_f32 in one pass: du = bias_act'(g; y re-derived from u) * d[n,o],
 * dt = adjoint FIR of du (pad (pady0, padx0) = (fh-1-p, fw-1-p) of the forward pad p, flip, gain fgain;
 * upfirdn2d.py:245-264 rule), and if dd != NULL: dd[n,o] += sum_hw dz*u.  g/u: [n,c,u_h,u_w],
 * dt: [n,c,t_h,t_pitch] (t_pitch = 0: t_w; columns >= t_w are not written).  4x4 filters only
 * (SMC_ERR_UNSUPPORTED otherwise); f = NULL: the built-in [1,3,3,1] taps (as smc_modconv_blur_act_f32). */
int smc_modconv_blur_act_bwd_f32(const float* g, const float* u, float* dt, float* dd, int n, int c, int u_h, int u_w,
                                 int t_h, int t_w, int t_pitch, const float* f, int fh, int fw, int padx0, int pady0,
                                 float fgain, int flip, const smc_conv_epilogue* epi, void* workspace,
                                 int64_t workspace_bytes, void* stream);
/* Workspace smc_modconv_blur_act_bwd_f32 needs when dd != NULL (0: none; the per-tile dd partials of planes wider
 * than two FIR tiles, summed per plane in a fixed order -- bit-reproducible dd). */
int64_t smc_modconv_blur_act_bwd_workspace_size(int n, int c, int u_h, int u_w, int t_h, int t_w);

/* Loss-head row reductions, one wave per row in a fixed order: the same row gives the same bits in any batch
 * (PyTorch's row reductions pick their block shape from the row count).  out[r] = sum_k a[r,k] * b[r,k]; ldb = 0
 * broadcasts b's first row.  Replaces the sums / norms of clip_loss.py:28-34, id_loss.py:26-39, model_irse.py:48. */
int smc_row_dot_f32(const float* a, int64_t lda, const float* b, int64_t ldb, float* out, int rows, int len,
                    void* stream);

/* The directional CLIP head (clip_loss.py:28-34) per row: f = e - src, u = f / |f|,
 * loss[r] = 1 - cosine_similarity(u, t) (eps as torch's), grad[r] = d loss[r] / d e[r] = (cos uh - th) / |f|
 * ([rows, len], dense).  t: one row (the normalised text direction).  len <= 1024. */
int smc_direction_head_f32(const float* e, int64_t lde, const float* src, int64_t lds, const float* t, float* loss,
                           float* grad, int rows, int len, float eps, void* stream);

/* d[n,o] = rsqrt(sum_i s[n,i]^2 * wsq[o,i] + eps), wsq[o,i] = sum_k W[o,i,k]^2 (demodulation). */
int smc_modconv_demod_f32(const float* s, const float* wsq, float* d, int n, int cin, int cout, float eps,
                          void* stream);

/* Backward of the modconv epilogue: recompute y from u, dz = bias_act grad (CUDA-kernel semantics,
 * bias_act.cu:51-142), du = dz * d[n,o]; if dd != NULL: dd[n,o] += sum_hw dz*u. */
int smc_modconv_act_bwd_f32(const float* g, const float* u, float* du, float* dd, int n, int c, int h, int w,
                            const smc_conv_epilogue* epi, void* workspace, int64_t workspace_bytes, void* stream);
/* Workspace smc_modconv_act_bwd_f32 needs when dd != NULL (0: none; per-workgroup dd partials of planes that span
 * more than two workgroups). */
int64_t smc_modconv_act_bwd_workspace_size(int n, int c, int h, int w);

/* out[r] (+)= sum_p a[r,p]*b[r,p] over rows r < rows of length len; if a_scaled != NULL also
 * a_scaled[r,p] = a[r,p]*scale[r] (scale may be NULL only when a_scaled is NULL). */
int smc_channel_dot_f32(const float* a, const float* b, const float* scale, float* out, float* a_scaled,
                        int64_t rows, int64_t len, int accumulate, void* stream);

/* ds[n,i] += -s[n,i] * sum_o dd[n,o] * d[n,o]^3 * wsq[o,i]   (gradient through the demodulation). */
int smc_modconv_demod_bwd_f32(const float* s, const float* d, const float* dd, const float* wsq, float* ds, int n,
                              int cin, int cout, void* stream);

/* ToRGB (1x1 modulated conv without demodulation + linear bias_act with clamp), replacing the
 * [upstream] ToRGBLayer.forward path (utils.py:47):  y[n,c,p] = clamp(sum_i w[c,i]*s[n,i]*x[n,i,p] + b[c]).
 * w: [cout][cin], s: [n][cin] (already multiplied by the layer's weight_gain), b: [cout] or NULL. */
int smc_torgb_fwd_f32(const float* x, const float* w, const float* s, const float* b, float* y, int n, int cin,
                      int cout, int h, int w_, float clamp, void* stream);

/* dx[n,i,p] (+)= (scale ? s[n,i] : 1) * sum_c w[c,i] * g[n,c,p] * [|y[n,c,p]| < clamp] */
int smc_torgb_bwd_f32(const float* g, const float* y, const float* w, const float* s, float* dx, int n, int cin,
                      int cout, int h, int w_, float clamp, int scale, int accumulate, void* stream);

/* Block-tail backward (the synthesis block output y = conv1's output feeds this block's ToRGB and the next block's
 * conv0): du[n,k,p] = act'(g_next[n,k,p] + (ToRGB^T g_rgb)[n,k,p]; y[n,k,p]) * d[n,k] with conv1's MODACT epilogue
 * `epi` (grad_from_y must be set: y is conv1's output; its d/act/alpha/gain/clamp), ToRGB^T as smc_torgb_bwd_f32
 * with scale = 1 (g_rgb masked by |y_rgb| < clamp_rgb), g_next may be NULL (the last block).  Bit-identical to
 * smc_torgb_bwd_f32 + the sum + smc_modconv_act_bwd_f32 (grad_from_y).  Replaces the autograd sum of the two
 * gradients of [upstream] SynthesisBlock's `x` (utils.py:47 torgb + the next block's conv0). */
int smc_torgb_act_bwd_f32(const float* g_rgb, const float* y_rgb, const float* w, const float* s, float clamp_rgb,
                          const float* g_next, const float* y, float* du, int n, int cin, int cout, int h, int w_,
                          const smc_conv_epilogue* epi, void* stream);

/* IDLoss face crop (id_loss.py:20-23): y[p] = adaptive_avg_pool(crop(adaptive_avg_pool(x[p], (pool_h, pool_w)),
 * [crop_y0 : crop_y0+crop_h, crop_x0 : crop_x0+crop_w]), (out_h, out_w)) for `planes` planes; the first pool
 * must be an integer factor (in = pool * k, else SMC_ERR_UNSUPPORTED).  The backward writes the whole input
 * gradient dx [planes][in_h][in_w] (zeros outside the crop). */
int smc_face_crop_f32(const float* x, int64_t planes, int in_h, int in_w, int pool_h, int pool_w, int crop_y0,
                      int crop_x0, int crop_h, int crop_w, int out_h, int out_w, float* y, void* stream);
int smc_face_crop_bwd_f32(const float* dy, int64_t planes, int in_h, int in_w, int pool_h, int pool_w, int crop_y0,
                          int crop_x0, int crop_h, int crop_w, int out_h, int out_w, float* dx, void* stream);

/* CLIP input preprocessing (find_direction.py:49-52): y = (bicubic(clamp(img*127.5+128, 0, 255), out) / 255
 * - mean[c]) / std[c], bicubic = F.interpolate(mode='bicubic', align_corners=False) (A = -0.75).  img
 * [n][channels][in_h][in_w] -> y [n][channels][out_h][out_w]; mean/std: `channels` floats on the device.
 * The backward writes the whole image gradient dimg (downsampling, in >= out, only). */
int smc_clip_unprocess_f32(const float* img, int n, int channels, int in_h, int in_w, int out_h, int out_w,
                           const float* mean, const float* std_, float* y, void* stream);
int smc_clip_unprocess_bwd_f32(const float* img, const float* dy, int n, int channels, int in_h, int in_w, int out_h,
                               int out_w, const float* mean, const float* std_, float* dimg, void* stream);
/* StyleGAN-NADA CLIP preprocessing (clip_loss_nada.py:72-75 `preprocess`, applied at :109-111 and :225):
 * torchvision Normalize(mean=-1, std=2) -> Resize(out, BICUBIC) -> CenterCrop(out) -> Normalize(CLIP mean, std),
 * no clamp: y = (bicubic((img + 1) / 2, out) - mean[c]) / std[c].  Same shapes / backward contract as
 * smc_clip_unprocess_f32 (square input, so the crop is the identity). */
int smc_clip_preprocess_nada_f32(const float* img, int n, int channels, int in_h, int in_w, int out_h, int out_w,
                                 const float* mean, const float* std_, float* y, void* stream);
int smc_clip_preprocess_nada_bwd_f32(const float* img, const float* dy, int n, int channels, int in_h, int in_w,
                                     int out_h, int out_w, const float* mean, const float* std_, float* dimg,
                                     void* stream);

/* ---------------------------------------------------------------------------------------------
 * CLIP ViT image tower (replaces the third-party openai/CLIP VisionTransformer that the reference
 * calls through CLIPLoss.encode_image, clip_loss.py:21,25-26; weights frozen -> data gradient only).
 *
 * smc_linear_f32: C[M][N] = epi(A[M][K] . B[K][N]) on fp32 MFMA (row-major, leading dimensions in
 * floats; K % 32 == 0, N % 4 == 0, A and B 16-B aligned).  B is the frozen weight stored K-major
 * (nn.Linear weight^T for a forward product, the weight itself for its data gradient).
 * Epilogue order: + bias[n]; * act'(dact_pre[m][n]); pre_save = v, v = act(v); + residual[m][n]
 * (residual may alias C).  Workspace: smc_linear_workspace_size() bytes (split-K partial tiles).
 */
#define SMC_LIN_ACT_NONE 0
#define SMC_LIN_ACT_QUICKGELU 1 /* x * sigmoid(1.702 x), CLIP's QuickGELU */

typedef struct {
    const float* bias;      /* [N] or NULL                                                    */
    const float* dact_pre;  /* multiply by QuickGELU'(dact_pre[m*ld_dact+n]) or NULL           */
    int ld_dact;
    int act;                /* SMC_LIN_ACT_*                                                   */
    float* pre_save;        /* pre-activation store when act != NONE, may be NULL              */
    int ld_pre;
    const float* residual;  /* added last, may be NULL or alias C                              */
    int ld_res;
} smc_linear_epilogue;

int64_t smc_linear_workspace_size(int M, int N, int K);
int smc_linear_f32(const float* a, int lda, const float* b, int ldb, float* c, int ldc, int M, int N, int K,
                   const smc_linear_epilogue* epi, float* workspace, int64_t workspace_bytes, void* stream);

/* LayerNorm over the last dim (nn.LayerNorm: biased variance, y = (x-mean)*rstd*w + b), one row per
 * wave; dim % 64 == 0, dim <= 1024.  mean/rstd [rows] may be NULL.  Row strides in floats. */
int smc_layernorm_fwd_f32(const float* x, int64_t ldx, const float* w, const float* b, float* y, int64_t ldy,
                          float* mean, float* rstd, int rows, int dim, float eps, void* stream);
/* dx = LN'(dy) (+ dres if not NULL); dx may alias dres. */
int smc_layernorm_bwd_f32(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* mean,
                          const float* rstd, const float* w, const float* dres, int64_t ldres, float* dx,
                          int64_t lddx, int rows, int dim, void* stream);

/* Multi-head softmax attention over qkv [batch*tokens][3*heads*64] (q | k | v, nn.MultiheadAttention
 * in_proj order) -> out [batch*tokens][heads*64]; p_save [batch][heads][tokens][tokens] may be NULL.
 * head_dim must be 64.  The backward writes dqkv [batch*tokens][3*heads*64] and needs qkv and dout 16-byte
 * aligned. */
int smc_attention_fwd_f32(const float* qkv, float* out, float* p_save, int batch, int tokens, int heads,
                          int head_dim, float scale, void* stream);
int smc_attention_bwd_f32(const float* dout, const float* qkv, const float* p_save, float* dqkv, int batch,
                          int tokens, int heads, int head_dim, float scale, void* stream);
/* The same forward with the causal mask of CLIP's text transformer (openai/CLIP model.py
 * build_attention_mask: -inf above the diagonal), used once per prompt by the CLIPLoss text side
 * (clip_loss.py:15-18 encode_text).  Forward only. */
int smc_attention_causal_fwd_f32(const float* qkv, float* out, int batch, int tokens, int heads, int head_dim,
                                 float scale, void* stream);

/* Non-overlapping patch extraction (conv kernel == stride): img [batch][channels][grid*patch]^2 <->
 * patches [batch*grid*grid][channels*patch*patch]; inverse = 1 writes img from patches. */
int smc_patch_im2col_f32(const float* img, float* patches, int batch, int channels, int grid, int patch,
                         int inverse, void* stream);

typedef struct {
    int width, layers, heads, patch, grid, out_dim, in_ch; /* ViT-B/32: 768, 12, 12, 32, 7, 512, 3 */
    float ln_eps;                                          /* 1e-5 (nn.LayerNorm default)          */
    int products;  /* 0: exact-fp32 MFMA; 1: split-bf16 (three bf16 terms per fp32 operand, the six products above
                      2^-23 |a b|; the packed buffer then ends with every projection's planes, smc_vit_pack_x3) */
} smc_vit_config;

/* Packed frozen weights: one fp32 buffer, segments in this order, each padded to 64 floats:
 *   conv_wt [C*p*p][D], conv_w [D][C*p*p], class_embedding [D], positional_embedding [L][D],
 *   ln_pre.{w,b} [D],
 *   per layer: ln_1.{w,b}, in_proj_weight^T [D][3D], in_proj_weight [3D][D], in_proj_bias [3D],
 *              out_proj.weight^T [D][D], out_proj.weight [D][D], out_proj.bias [D], ln_2.{w,b},
 *              c_fc.weight^T [D][4D], c_fc.weight [4D][D], c_fc.bias [4D],
 *              c_proj.weight^T [4D][D], c_proj.weight [D][4D], c_proj.bias [D],
 *   ln_post.{w,b} [D], proj [D][E], proj^T [E][D]
 * (the segment sizes of one layer are padded individually; see stylemc_amd/vit_hip.py). */
int64_t smc_vit_packed_floats(const smc_vit_config* cfg);
/* Activations the backward needs, per batch size (floats). */
int64_t smc_vit_saved_floats(const smc_vit_config* cfg, int batch);
/* products = 1: fill the planes region at the end of `packed` from its fp32 segments (after they are written). */
int smc_vit_pack_x3(const smc_vit_config* cfg, float* packed, void* stream);
int64_t smc_vit_workspace_bytes(const smc_vit_config* cfg, int batch);
/* image [batch][in_ch][grid*patch][grid*patch] -> out [batch][out_dim]; saved may be NULL (no backward). */
int smc_vit_forward_f32(const smc_vit_config* cfg, const float* packed, const float* image, int batch, float* out,
                        float* saved, float* workspace, int64_t workspace_bytes, void* stream);
/* dimage = d out / d image applied to dout, from the forward's saved activations (laid out for `batch`
 * images); only the leading batch_run <= batch images are differentiated: dout [batch_run][out_dim],
 * dimage [batch_run][in_ch][..][..] (the original-image half of a batched pair needs no gradient). */
int smc_vit_backward_f32(const smc_vit_config* cfg, const float* packed, const float* dout, int batch, int batch_run,
                         const float* saved, float* dimage, float* workspace, int64_t workspace_bytes,
                         void* stream);

/* ---------------------------------------------------------------------------------------------
 * ArcFace IR-SE50 (id_loss/model_irse.py:10-49, helpers.py:56-119; run by IDLoss.extract_feats,
 * id_loss/id_loss.py:20-24): forward and input gradient (frozen, eval-mode weights).
 * The caller describes the network once (packed conv phases as for smc_conv_gemm_f32, eval-mode
 * BatchNorms as per-channel scale a / shift b); see stylemc_amd/irse_hip.py for the packing.
 */
typedef struct {
    int cin, depth, stride, in_h, in_w;  /* unit input [n][cin][in_h][in_w] -> [n][depth][in_h/s][in_w/s]   */
    const float* bn1_a;                  /* [cin] res_layer BatchNorm2d (before conv1) as x*a + b              */
    const float* bn1_b;
    smc_conv_phase c1_fwd;               /* 3x3 stride 1, cin -> depth                                         */
    smc_conv_phase c1_bwd;               /* its adjoint depth -> cin, bn1_a folded into the weights            */
    const float* prelu;                  /* [depth]                                                            */
    smc_conv_phase c2_fwd;               /* 3x3 stride s, depth -> depth                                       */
    smc_conv_phase c2_bwd[4];            /* its adjoint (4 polyphase phases when s == 2), bn2_a folded         */
    int c2_bwd_nphases;
    const float* bn2_a;                  /* [depth]                                                            */
    const float* bn2_b;
    const float* se_w1;                  /* SE fc1 [hidden][depth]                                             */
    const float* se_w2;                  /* SE fc2 [depth][hidden]                                             */
    int se_hidden;
    int sc_conv;                         /* shortcut: 0 = MaxPool2d(1, s) (cin == depth), 1 = conv1x1(s) + BN  */
    smc_conv_phase sc_fwd;               /* 1 tap, in_stride s                                                 */
    smc_conv_phase sc_bwd;               /* adjoint on the compact grid, sc_a folded                          */
    const float* sc_a;
    const float* sc_b;
} smc_irse_unit;

typedef struct {
    int n_units;
    const smc_irse_unit* units;
    int in_h, in_w;                      /* 112 x 112                                                          */
    int img_ch;                          /* 3                                                                  */
    int stem_cin;                        /* img_ch padded to a multiple of 16 (zero channels / weights)        */
    int stem_cout;                       /* 64                                                                 */
    smc_conv_phase stem_fwd;             /* input_layer conv3x3                                                */
    smc_conv_phase stem_bwd;             /* its adjoint, stem_bn_a folded                                      */
    const float* stem_bn_a;
    const float* stem_bn_b;
    const float* stem_prelu;
    int feat;                            /* 512                                                                */
    int flat;                            /* 512*7*7                                                            */
    const float* fc_wt;                  /* [flat][feat]: output BatchNorm2d + Linear + BatchNorm1d folded     */
    const float* fc_w;                   /* [feat][flat] (data gradient)                                       */
    const float* fc_b;                   /* [feat]                                                             */
} smc_irse_net;

int64_t smc_irse_saved_floats(const smc_irse_net* net, int n);
int64_t smc_irse_workspace_bytes(const smc_irse_net* net, int n);
/* img [n][img_ch][in_h][in_w] -> feat [n][feat] (before the l2 normalisation); saved may be NULL. */
int smc_irse_forward_f32(const smc_irse_net* net, const float* img, int n, float* feat, float* saved,
                         float* workspace, int64_t workspace_bytes, void* stream);
/* input gradient of the leading n <= n_saved faces of a forward that ran (and saved) n_saved faces:
 * dfeat [n][feat] -> dimg [n][img_ch][in_h][in_w]. */
int smc_irse_backward_f32(const smc_irse_net* net, const float* dfeat, int n_saved, int n, const float* saved,
                          float* dimg, float* workspace, int64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* STYLEMC_HIP_H */
