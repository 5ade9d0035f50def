"""Modulated convolution on gfx950: forward + analytic backward through the C ABI.

Replaces [upstream] ``modulated_conv2d`` + the bias_act / noise epilogue of ``SynthesisLayer`` /
``ToRGBLayer`` (the per-layer work of utils.py:32,39-40,47).  The computation is the non-fused form

    u  = conv(x * s[n, i], W)                (one shared-weight implicit GEMM on MFMA, whole batch)
    y  = clamp(act(u * d[n, o] + noise * strength + b) * gain),   d = rsqrt(s^2 . Wsq + 1e-8)

which is mathematically identical to the reference's fused per-sample grouped convolution
(conv2d_resample.py:125-147 with groups = batch) and needs no per-sample weights.  up=2 layers run
the stride-2 transposed conv as 4 polyphase GEMM phases, then the [1,3,3,1] blur fused with the
epilogue (conv2d_resample.py:125-139 semantics: transposed conv, FIR pad 1, gain 4).

Backward (G is frozen, so no weight gradients):
    dz  = bias_act'(g; y)                      (CUDA-kernel clamp semantics, bias_act.cu:136-141)
    du  = dz * d,   dd[n,o] = sum_p dz * u
    dxs = conv^T(du, W)  [up=2: through the blur adjoint + stride-2 gather conv]
    dx  = dxs * s,  ds[n,i] = sum_p dxs * x  -  s[n,i] * sum_o dd * d^3 * Wsq[o,i]
"""
import ctypes

import torch

from . import _hip


def _phase(taps, in_stride, out_h, out_w, out_oy, out_ox, out_sy, out_sx, wk, wk_x3=None):
    ph = _hip.ConvPhase()
    ph.ntaps = len(taps)
    for t, (dy, dx) in enumerate(taps):
        ph.tap_dy[t] = dy
        ph.tap_dx[t] = dx
    ph.in_stride = in_stride
    ph.out_h, ph.out_w, ph.out_oy, ph.out_ox, ph.out_sy, ph.out_sx = out_h, out_w, out_oy, out_ox, out_sy, out_sx
    ph.wk = wk.data_ptr()
    ph.wk_x3 = wk_x3.data_ptr() if wk_x3 is not None else None
    return ph


# Split-bf16 products for the direct implicit-GEMM convs (include/stylemc_hip.h smc_conv_phase.wk_x3): every fp32
# operand split exactly into three bf16 terms, the six products above 2^-23 |a b| on the bf16 matrix core.  Module
# switch (tests / tools compare it against the exact-fp32 MFMA kernels).
X3 = True


def x3_planes(wk, cin, cout, enabled=None):
    """The split-bf16 planes (smc_conv_weights_x3) of [ntaps][cin][cout] GEMM weights, or None where the kernel has
    no split form (cin % 16), the weights are not on the GPU or split products are off (``enabled``; default: this
    module's X3 -- the IR-SE50 executor passes its own switch)."""
    if not ((X3 if enabled is None else enabled) and wk.is_cuda):
        return None
    lib = _hip.load()
    nb = lib.smc_conv_weights_x3_bytes(wk.shape[0], cin, cout)
    if nb <= 0:
        return None
    out = torch.empty((nb + 15) // 16 * 8, device=wk.device, dtype=torch.int16)
    _hip.call("smc_conv_weights_x3", wk.data_ptr(), wk.shape[0], cin, cout, out.data_ptr(), _hip.stream())
    return out


class PackedConv:
    """Frozen conv weights repacked for the gather GEMM (K = tap-major x channel, N contiguous)."""

    def __init__(self, weight, up):
        W = weight.detach().to(torch.float32).contiguous()
        self.cout, self.cin, kh, kw = W.shape
        self.k = kh
        self.up = up
        if not (kh == kw and kh in (1, 3)) or up not in (1, 2) or (up == 2 and kh != 3):
            raise NotImplementedError(f"modulated conv: kernel {kh}x{kw} with up={up} has no gfx950 kernel")
        self.wsq = W.square().sum(dim=[2, 3]).contiguous()                           # [O, I]
        taps = [(ky, kx) for ky in range(kh) for kx in range(kw)]
        self.wk_bwd = W.permute(2, 3, 0, 1).reshape(kh * kw, self.cout, self.cin).contiguous()  # [t][o][i]
        if up == 1:
            c = kh // 2
            self.fwd_taps = [(ky - c, kx - c) for ky, kx in taps]
            self.bwd_taps = [(c - ky, c - kx) for ky, kx in taps]
            self.wk_fwd = W.permute(2, 3, 1, 0).reshape(kh * kw, self.cin, self.cout).contiguous()  # [t][i][o]
        else:
            # polyphase transposed conv: T[o, 2a+py, 2b+px] += x[i, a-(ky-py)/2, b-(kx-px)/2] W[o,i,ky,kx]
            self.phases = []
            for py in (0, 1):
                for px in (0, 1):
                    sel = [(ky, kx) for ky, kx in taps if ky % 2 == py and kx % 2 == px]
                    wk = torch.stack([W[:, :, ky, kx].t() for ky, kx in sel]).contiguous()  # [t][i][o]
                    self.phases.append((py, px, [(-(ky - py) // 2, -(kx - px) // 2) for ky, kx in sel], wk))
            self.bwd_taps = [(ky, kx) for ky, kx in taps]  # stride-2 gather over dT
        # split-bf16 planes of the direct GEMMs' weights, built on first use (x3_fwd / x3_bwd / x3_phases): a layer
        # whose forward or data gradient always takes a Winograd kernel never builds (1.5x the fp32 bytes of) that
        # direction's planes.  The switch is read once, here.
        self.use_x3 = X3
        self._x3 = {}
        self._cache = {}
        self._wino = {}
        self._wino4 = {}

    def _planes(self, key, wk, cin, cout):
        if key not in self._x3:
            p = x3_planes(wk, cin, cout, enabled=self.use_x3)
            if p is not None:   # built on this stream, read from any: wait once (LayerSpec builds the expected ones
                torch.cuda.current_stream(wk.device).synchronize()   # up front; this is the fallback for others)
            self._x3[key] = p
        return self._x3[key]

    @property
    def x3_fwd(self):
        return self._planes("f", self.wk_fwd, self.cin, self.cout) if self.up == 1 else None

    @property
    def x3_bwd(self):
        return self._planes("b", self.wk_bwd, self.cout, self.cin)

    @property
    def x3_phases(self):
        if self.up != 2:
            return None
        return [self._planes(("p", i), wk, self.cin, self.cout) for i, (_, _, _, wk) in enumerate(self.phases)]

    def wino_weights(self, flip):
        """Winograd F(2x2, 3x3) transformed taps (smc_wino_weights_f32) of the 3x3 'same' conv, built once on the
        weights' device: flip 0 = the forward, 1 = the data gradient.  LayerSpec builds both eagerly for the layers
        that take the Winograd path; a transform built here later is waited for before it is returned (the first
        caller may be on a side stream while the next launch that reads it is on another one)."""
        if flip not in self._wino:
            W = self.wk_bwd  # [t][o][i] -> back to [o][i][3][3] on the same device
            w = W.reshape(3, 3, self.cout, self.cin).permute(2, 3, 0, 1).contiguous()
            uw = torch.empty(16 * self.cin * self.cout, device=w.device, dtype=torch.float32)
            _hip.call("smc_wino_weights_f32", w.data_ptr(), self.cout, self.cin, flip, uw.data_ptr(), _hip.stream())
            torch.cuda.current_stream(w.device).synchronize()
            self._wino[flip] = uw
        return self._wino[flip]

    def wino4_weights(self, flip):
        """Winograd F(4x4, 3x3) transformed taps (smc_wino4_weights_f32, 36 per channel pair), same contract as
        wino_weights."""
        if flip not in self._wino4:
            W = self.wk_bwd
            w = W.reshape(3, 3, self.cout, self.cin).permute(2, 3, 0, 1).contiguous()
            uw = torch.empty(36 * self.cin * self.cout, device=w.device, dtype=torch.float32)
            _hip.call("smc_wino4_weights_f32", w.data_ptr(), self.cout, self.cin, flip, uw.data_ptr(), _hip.stream())
            torch.cuda.current_stream(w.device).synchronize()
            self._wino4[flip] = uw
        return self._wino4[flip]

    def fwd_phases(self, h, w):
        key = ("f", h, w)
        if key not in self._cache:
            if self.up == 1:
                arr = (_hip.ConvPhase * 1)(_phase(self.fwd_taps, 1, h, w, 0, 0, 1, 1, self.wk_fwd, self.x3_fwd))
                self._cache[key] = (arr, 1, h, w)
            else:
                th, tw = 2 * h + 1, 2 * w + 1
                ph = [_phase(t, 1, (th - py + 1) // 2, (tw - px + 1) // 2, py, px, 2, 2, wk, wx)
                      for (py, px, t, wk), wx in zip(self.phases, self.x3_phases)]
                self._cache[key] = ((_hip.ConvPhase * 4)(*ph), 4, th, tw)
        return self._cache[key]

    def bwd_phases(self, h, w):
        key = ("b", h, w)
        if key not in self._cache:
            stride = 1 if self.up == 1 else 2
            self._cache[key] = ((_hip.ConvPhase * 1)(_phase(self.bwd_taps, stride, h, w, 0, 0, 1, 1, self.wk_bwd,
                                                            self.x3_bwd)), 1)
        return self._cache[key]


def conv_flops(n, cin, cout, h_out, w_out, taps):
    return 2.0 * n * cin * cout * h_out * w_out * taps


def gemm(x, y, phases, nph, cin, cout, s=None, epi=None, alg_flops=0.0, alg_bytes=0):
    """One smc_conv_gemm_f32 launch.  alg_flops / alg_bytes: the conv's dense MACs x 2 and its compulsory HBM
    bytes (input and output activations once, weights once, plus the saved u / scaled-input planes) -- only
    recorded by the bench's KernelTimer."""
    n, _, ih, iw = x.shape
    yh, yw = y.shape[2], y.shape[3]
    lib = _hip.load()
    ws_bytes = lib.smc_conv_gemm_workspace_size(n, cin, cout, yh, yw, phases, nph)
    ws = torch.empty(max(ws_bytes // 4, 1), device=x.device, dtype=torch.float32) if ws_bytes > 0 else None
    tm = _hip.timer()
    tok = tm.wrap(alg_flops, alg_bytes, kind="direct") if tm is not None else None
    _hip.call("smc_conv_gemm_f32", x.data_ptr(), n, cin, ih, iw, y.data_ptr(), cout, yh, yw, phases, nph,
              _hip.ptr(s), ctypes.byref(epi) if epi is not None else None, _hip.ptr(ws), ws_bytes, _hip.stream())
    if tok is not None:
        # the product form the library actually launched (split-bf16 only where the LDS-DMA kernels took the call)
        tm.finish(tok, kind="direct_x3" if lib.smc_conv_gemm_last_x3() else "direct")


# Winograd F(2x2, 3x3) for the 3x3 stride-1 convs wherever smc_conv3x3_wino_supported() has a kernel (module
# switch, not an environment knob: tests / tools flip it to compare against the direct implicit GEMM).
WINOGRAD = True


def wino_ok(n, cin, cout, h, w):
    return WINOGRAD and bool(_hip.load().smc_conv3x3_wino_supported(n, cin, cout, h, w))


# Split K for the grids of fewer than 512 work items (the 32 x 32 convs: smc_conv3x3_wino_workspace_size).
WINO_SPLIT = True


def wino(x, y, uw, cin, cout, s=None, epi=None, alg_flops=0.0, alg_bytes=0):
    """One smc_conv3x3_wino_f32 launch (3x3, stride 1, pad 1).  alg_flops: the MFMA FLOPs it executes
    (16 / 36 of the direct conv's; the timer also records the direct-equivalent count)."""
    n, _, h, w = x.shape
    ws_bytes = _hip.load().smc_conv3x3_wino_workspace_size(n, cin, cout, h, w) if WINO_SPLIT else 0
    ws = torch.empty(ws_bytes // 4, device=x.device, dtype=torch.float32) if ws_bytes > 0 else None
    tm = _hip.timer()
    tok = tm.wrap(alg_flops, alg_bytes, kind="wino", equiv_flops=alg_flops * 36 / 16) if tm is not None else None
    _hip.call("smc_conv3x3_wino_ws_f32", x.data_ptr(), n, cin, h, w, y.data_ptr(), cout, uw.data_ptr(), _hip.ptr(s),
              ctypes.byref(epi) if epi is not None else None, _hip.ptr(ws), ws_bytes, _hip.stream())
    if tok is not None:
        tm.finish(tok)


def wino4_ok(n, cin, cout, h, w):
    return WINOGRAD and bool(_hip.load().smc_conv3x3_wino4_supported(n, cin, cout, h, w))


# F(4x4) where it measured faster than F(2x2) (tools/bench_wino.py, FFHQ-1024 batch 4, profiles/r03_wino4/bench_wino_v2.txt):
# 1.32-1.35x at cin 512 (r = 64), 1.25-1.27x at 256, 1.14-1.16x at 128, 0.99-1.01x at 64 in round 3.  Round 6
# (profiles/r06/wino4_64/): the r = 512 / 64-channel conv1 now 1.05-1.07x (415 -> 390 us forward, 400 -> 383 data
# gradient) and the step +1.3 % images/s (three interleaved rounds), so 64-channel inputs take F(4x4) too; the
# 32-channel r = 1024 layer has no F(4x4) kernel.  Module switch.
WINO4 = True
WINO4_MIN_CIN = 64


def wino4_pick(n, cin, cout, h, w):
    return WINO4 and cin >= WINO4_MIN_CIN and wino4_ok(n, cin, cout, h, w)


def wino4(x, y, uw, cin, cout, s=None, epi=None, alg_flops=0.0, alg_bytes=0):
    """One smc_conv3x3_wino4_f32 launch (F(4x4, 3x3)).  alg_flops: the MFMA FLOPs it executes (36 / 144 of the
    direct conv's; the timer also records the direct-equivalent count)."""
    n, _, h, w = x.shape
    tm = _hip.timer()
    tok = tm.wrap(alg_flops, alg_bytes, kind="wino4", equiv_flops=alg_flops * 4) if tm is not None else None
    _hip.call("smc_conv3x3_wino4_f32", x.data_ptr(), n, cin, h, w, y.data_ptr(), cout, uw.data_ptr(), _hip.ptr(s),
              ctypes.byref(epi) if epi is not None else None, _hip.stream())
    if tok is not None:
        tm.finish(tok)


def wino4_flops(n, cin, cout, h, w):
    """MFMA FLOPs of one F(4x4, 3x3) launch: 36 multiplies per 4x4 tile and channel pair."""
    return 2.0 * n * cin * cout * (h // 4) * (w // 4) * 36


def wino_flops(n, cin, cout, h, w):
    return 2.0 * n * cin * cout * (h // 2) * (w // 2) * 16


def _epilogue(mode, d=None, noise=None, noise_nstride=0, strength=None, bias=None, act="linear", alpha=0.0,
              gain=1.0, clamp=-1.0, u_save=None):
    e = _hip.ConvEpilogue()
    e.mode = mode
    e.d = _hip.ptr(d)
    e.noise = _hip.ptr(noise)
    e.noise_nstride = noise_nstride
    e.noise_strength = _hip.ptr(strength)
    e.bias = _hip.ptr(bias)
    e.act = _hip.ACT_CODES[act]
    e.alpha, e.gain, e.clamp = float(alpha), float(gain), float(clamp)
    e.u_save = _hip.ptr(u_save)
    return e


class LayerSpec:
    """Everything the modconv kernels need about one frozen layer (built once per SynthesisLayer)."""

    def __init__(self, weight, bias, up, resample_filter, demodulate=True, act="lrelu", alpha=0.2, resolution=None):
        self.packed = PackedConv(weight, up)
        self.bias = bias.detach().float().contiguous() if bias is not None else None
        self.up = up
        self.filter = resample_filter.detach().float().contiguous() if resample_filter is not None else None
        # the synthesis' setup_filter([1,3,3,1]): the FIR forward kernel takes it as compile-time taps (f = NULL)
        k = torch.tensor([1.0, 3.0, 3.0, 1.0])
        self.std_filter = self.filter is not None and tuple(self.filter.shape) == (4, 4) and torch.equal(
            self.filter.detach().cpu(), torch.outer(k, k) / 64.0)
        self.demodulate = demodulate
        self.act = act
        self.alpha = alpha
        P = self.packed
        if weight.is_cuda:
            # the spec is built lazily, on whichever stream first reaches the layer (find_direction's first step
            # runs the original-image synthesis on a side stream): build the Winograd transforms of a Winograd
            # layer now, and let every packing kernel finish before another stream can read the packed weights
            direct = [True, True]   # forward, data gradient on the direct implicit GEMM (split-bf16 planes)
            if resolution is not None and up == 1 and P.k == 3:
                for flip, (ci, co) in enumerate([(P.cin, P.cout), (P.cout, P.cin)]):
                    if wino4_pick(1, ci, co, resolution, resolution):
                        P.wino4_weights(flip)
                        direct[flip] = False
                    elif wino_ok(1, ci, co, resolution, resolution):
                        P.wino_weights(flip)
                        direct[flip] = False
            # the split-bf16 planes of the directions that take the direct GEMM, built here (one wait below) rather than
            # on first use inside a step, where the build's host wait would stall whichever stream reached it first
            if resolution is not None:
                if direct[0]:
                    P.x3_fwd if up == 1 else P.x3_phases
                if direct[1]:
                    P.x3_bwd
            torch.cuda.current_stream(weight.device).synchronize()


def _noise_args(noise):
    if noise is None:
        return None, 0
    noise = noise.contiguous()
    if noise.ndim == 2:
        return noise, 0
    assert noise.ndim == 4 and noise.shape[1] == 1, "noise must be [H, W] or [N, 1, H, W]"
    return noise, noise.shape[2] * noise.shape[3]


def _modconv_fwd(ctx, x, styles, spec, noise, strength, gain, clamp, need_dx, need_ds):
    """The modconv forward (GEMM + fused epilogue); sets ctx's backward state, returns y and the tensors the
    backward needs (x, styles, d, and u -- or y itself where the styles need no gradient)."""
    x = x.contiguous()
    styles = styles.contiguous()
    P = spec.packed
    n, cin, h, w = x.shape
    assert cin == P.cin and styles.shape == (n, cin), (x.shape, styles.shape, P.cin)
    r_h, r_w = h * spec.up, w * spec.up
    d = None
    if spec.demodulate:
        d = torch.empty(n, P.cout, device=x.device, dtype=torch.float32)
        _hip.call("smc_modconv_demod_f32", _hip.ptr(styles), _hip.ptr(P.wsq), _hip.ptr(d), n, cin, P.cout, 1e-8,
                  _hip.stream())
    save = need_dx or need_ds
    # the activation mask of the backward needs only y; u is kept only where the style gradient needs
    # dd = sum dz * u (the trainable layers): every other layer skips the u store (grad_from_y backward)
    from_y = save and not need_ds
    y = torch.empty(n, P.cout, r_h, r_w, device=x.device, dtype=torch.float32)
    u = torch.empty_like(y) if save and not from_y else None
    nz, nstride = _noise_args(noise)
    epi = _epilogue(_hip.EPI_MODACT, d, nz, nstride, strength, spec.bias, spec.act, spec.alpha, gain, clamp, u)
    phases, nph, th, tw = P.fwd_phases(h, w)
    wbytes = 4 * P.k * P.k * cin * P.cout
    if spec.up == 1 and P.k == 3 and wino4_pick(n, cin, P.cout, h, w):
        wino4(x, y, P.wino4_weights(0), cin, P.cout, s=styles, epi=epi, alg_flops=wino4_flops(n, cin, P.cout, h, w),
              alg_bytes=4 * x.numel() + 4 * y.numel() * (2 if u is not None else 1) + 36 * 4 * cin * P.cout)
    elif spec.up == 1 and P.k == 3 and wino_ok(n, cin, P.cout, h, w):
        wino(x, y, P.wino_weights(0), cin, P.cout, s=styles, epi=epi, alg_flops=wino_flops(n, cin, P.cout, h, w),
             alg_bytes=4 * x.numel() + 4 * y.numel() * (2 if u is not None else 1) + 16 * 4 * cin * P.cout)
    elif spec.up == 1:
        gemm(x, y, phases, nph, cin, P.cout, s=styles, epi=epi,
             alg_flops=conv_flops(n, cin, P.cout, r_h, r_w, P.k * P.k),
             alg_bytes=4 * x.numel() + 4 * y.numel() * (2 if u is not None else 1) + wbytes)
    else:
        t = torch.empty(n, P.cout, th, tw, device=x.device, dtype=torch.float32)
        gemm(x, t, phases, nph, cin, P.cout, s=styles, epi=_epilogue(_hip.EPI_STORE),
             alg_flops=conv_flops(n, cin, P.cout, h, w, 9), alg_bytes=4 * x.numel() + 4 * t.numel() + wbytes)
        f = None if spec.std_filter else spec.filter.to(x.device)
        _hip.call("smc_modconv_blur_act_f32", t.data_ptr(), 1, 0, y.data_ptr(), n, P.cout, th, tw, 0, r_h, r_w,
                  _hip.ptr(f), 4 if f is None else f.shape[0], 4 if f is None else f.shape[1], 1, 1, 4.0, 0,
                  ctypes.byref(epi), _hip.stream())
    ctx.spec, ctx.gain, ctx.clamp = spec, gain, clamp
    ctx.noise, ctx.nstride, ctx.strength = nz, nstride, strength
    ctx.from_y = from_y
    return y, (x, styles, d, y if from_y else u)


def _modconv_epi_bwd(ctx, d):
    """conv's MODACT epilogue as its backward kernels see it (grad_from_y: their `u` is the saved y)."""
    spec = ctx.spec
    epi = _epilogue(_hip.EPI_MODACT, d, ctx.noise, ctx.nstride, ctx.strength, spec.bias, spec.act, spec.alpha,
                    ctx.gain, ctx.clamp)
    epi.grad_from_y = 1 if ctx.from_y else 0
    return epi


def _dd_workspace(dd, nbytes, device):
    """The dd-partials workspace of the epilogue backward kernels (torch's caching allocator, not the library)."""
    if dd is None or nbytes <= 0:
        return None
    return torch.empty(nbytes // 4, device=device, dtype=torch.float32)


def _nbytes(t):
    return 0 if t is None else 4 * t.numel()


def _modconv_bwd(ctx, saved, gy, need_dx, need_ds, g=None):
    """The modconv backward from the output gradient gy -- or from g, the epilogue's backward already applied
    (du = act'(gy; y) * d, a 1:1 layer whose styles need no gradient).  Returns (dx, ds)."""
    x, styles, d, u = saved
    spec = ctx.spec
    P = spec.packed
    n, cin, h, w = x.shape
    dd = torch.zeros(n, P.cout, device=x.device, dtype=torch.float32) if (need_ds and spec.demodulate) else None
    assert dd is None or not ctx.from_y
    if g is None:
        gy = gy.contiguous()
        epi = _modconv_epi_bwd(ctx, d)
        if spec.up == 1:
            g = torch.empty_like(u)
            ws = _dd_workspace(dd, _hip.load().smc_modconv_act_bwd_workspace_size(n, P.cout, u.shape[2], u.shape[3]),
                               x.device)
            _hip.call("smc_modconv_act_bwd_f32", gy.data_ptr(), u.data_ptr(), g.data_ptr(), _hip.ptr(dd), n, P.cout,
                      u.shape[2], u.shape[3], ctypes.byref(epi), _hip.ptr(ws), _nbytes(ws), _hip.stream())
        else:
            # fused: epilogue backward + adjoint of FIR(pad 1, gain 4) (pad fw-1-1 = 2, correlation) + dd
            f = None if spec.std_filter else spec.filter.to(x.device)
            fh, fw = (4, 4) if f is None else f.shape
            # dT rows padded to a multiple of 4 floats (aligned 16-B row starts for the FIR's stores and the gather
            # GEMM's loads); the stride-2 gather reads columns <= 2w only, so the pad columns are never read.
            th, tw = 2 * h + 1, 2 * w + 1
            pitch = (tw + 3) // 4 * 4
            g = torch.empty(n, P.cout, th, pitch, device=x.device, dtype=torch.float32)
            ws = _dd_workspace(dd, _hip.load().smc_modconv_blur_act_bwd_workspace_size(n, P.cout, u.shape[2],
                                                                                        u.shape[3], th, tw), x.device)
            _hip.call("smc_modconv_blur_act_bwd_f32", gy.data_ptr(), u.data_ptr(), g.data_ptr(), _hip.ptr(dd), n,
                      P.cout, u.shape[2], u.shape[3], th, tw, pitch, _hip.ptr(f), fh, fw, fw - 2, fh - 2, 4.0, 1,
                      ctypes.byref(epi), _hip.ptr(ws), _nbytes(ws), _hip.stream())
    else:
        assert spec.up == 1 and dd is None
    dx = torch.empty_like(x) if need_dx else None
    dxs = torch.empty_like(x) if need_ds else None
    if need_dx:
        ebw = _epilogue(_hip.EPI_MODACT, d=styles, act="linear", u_save=dxs)
        out = dx
    else:
        ebw = _epilogue(_hip.EPI_STORE)
        out = dxs
    g_bytes = 4 * g.numel() if spec.up == 1 else 4 * n * P.cout * (2 * h + 1) * (2 * w + 1)
    out_bytes = 4 * out.numel() * (2 if (need_dx and need_ds) else 1)
    if spec.up == 1 and P.k == 3 and wino4_pick(n, P.cout, cin, h, w):
        wino4(g, out, P.wino4_weights(1), P.cout, cin, epi=ebw, alg_flops=wino4_flops(n, P.cout, cin, h, w),
              alg_bytes=g_bytes + out_bytes + 36 * 4 * cin * P.cout)
    elif spec.up == 1 and P.k == 3 and wino_ok(n, P.cout, cin, h, w):
        wino(g, out, P.wino_weights(1), P.cout, cin, epi=ebw, alg_flops=wino_flops(n, P.cout, cin, h, w),
             alg_bytes=g_bytes + out_bytes + 16 * 4 * cin * P.cout)
    else:
        phases, nph = P.bwd_phases(h, w)
        gemm(g, out, phases, nph, P.cout, cin, epi=ebw, alg_flops=conv_flops(n, P.cout, cin, h, w, P.k * P.k),
             alg_bytes=g_bytes + out_bytes + 4 * P.k * P.k * cin * P.cout)
    ds = None
    if need_ds:
        ds = torch.empty(n, cin, device=x.device, dtype=torch.float32)
        _hip.call("smc_channel_dot_f32", dxs.data_ptr(), x.data_ptr(), None, ds.data_ptr(), None, n * cin, h * w, 0,
                  _hip.stream())
        if spec.demodulate:
            _hip.call("smc_modconv_demod_bwd_f32", styles.data_ptr(), d.data_ptr(), dd.data_ptr(),
                      P.wsq.data_ptr(), ds.data_ptr(), n, cin, P.cout, _hip.stream())
    return dx, ds


class ModConvFn(torch.autograd.Function):
    """y = modconv_epilogue(conv(x * s, W)); grads w.r.t. x and s only."""

    @staticmethod
    def forward(ctx, x, styles, spec, noise, strength, gain, clamp):
        y, saved = _modconv_fwd(ctx, x, styles, spec, noise, strength, gain, clamp, ctx.needs_input_grad[0],
                                ctx.needs_input_grad[1])
        ctx.save_for_backward(*saved)
        return y

    @staticmethod
    def backward(ctx, gy):
        need_dx, need_ds = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if not (need_dx or need_ds):
            return None, None, None, None, None, None, None
        dx, ds = _modconv_bwd(ctx, ctx.saved_tensors, gy, need_dx, need_ds)
        return dx, ds, None, None, None, None, None


def _torgb_fwd(x, styles, w2d, bias, clamp):
    n, cin, h, w = x.shape
    cout = w2d.shape[0]
    y = torch.empty(n, cout, h, w, device=x.device, dtype=torch.float32)
    _hip.call("smc_torgb_fwd_f32", x.data_ptr(), _hip.ptr(w2d), styles.data_ptr(), _hip.ptr(bias), y.data_ptr(), n,
              cin, cout, h, w, clamp, _hip.stream())
    return y


def _torgb_style_grad(gy, y, x, styles, w2d, clamp):
    n, cin, h, w = x.shape
    dxs = torch.empty_like(x)
    _hip.call("smc_torgb_bwd_f32", gy.data_ptr(), y.data_ptr(), w2d.data_ptr(), styles.data_ptr(), dxs.data_ptr(), n,
              cin, w2d.shape[0], h, w, clamp, 0, 0, _hip.stream())
    ds = torch.empty(n, cin, device=x.device, dtype=torch.float32)
    _hip.call("smc_channel_dot_f32", dxs.data_ptr(), x.data_ptr(), None, ds.data_ptr(), None, n * cin, h * w, 0,
              _hip.stream())
    return ds


class ModConvToRGBFn(torch.autograd.Function):
    """A synthesis block's conv1 (3x3 modconv) and the ToRGB layer reading its output y, as one Function:
    returns (y, rgb).  y also feeds the next block's conv0, so its gradient is g_next + ToRGB^T(g_rgb); where
    conv1's styles need no gradient the backward forms it and conv1's epilogue backward in one pass
    (smc_torgb_act_bwd_f32) instead of a ToRGB data-gradient kernel, autograd's sum and the act backward
    (utils.py:47 + [upstream] SynthesisBlock.forward; same numbers bit for bit)."""

    @staticmethod
    def forward(ctx, x, styles, spec, noise, strength, gain, clamp, s_rgb, w_rgb, b_rgb, clamp_rgb):
        ctx.set_materialize_grads(False)
        y, saved = _modconv_fwd(ctx, x, styles, spec, noise, strength, gain, clamp, ctx.needs_input_grad[0],
                                ctx.needs_input_grad[1])
        s_rgb = s_rgb.contiguous()
        rgb = _torgb_fwd(y, s_rgb, w_rgb, b_rgb, clamp_rgb)
        ctx.clamp_rgb = clamp_rgb
        ctx.save_for_backward(*saved, y, s_rgb, w_rgb, rgb)
        return y, rgb

    @staticmethod
    def backward(ctx, gy, grgb):
        x, styles, d, u, y, s_rgb, w_rgb, rgb = ctx.saved_tensors
        need_dx, need_ds, need_ds_rgb = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[7]
        ds_rgb = None
        if need_ds_rgb and grgb is not None:
            ds_rgb = _torgb_style_grad(grgb.contiguous(), rgb, y, s_rgb, w_rgb, ctx.clamp_rgb)
        dx = ds = None
        if (need_dx or need_ds) and (gy is not None or grgb is not None):
            saved = (x, styles, d, u)
            n, c, h, w = y.shape
            if grgb is not None and ctx.from_y and ctx.spec.up == 1:
                g = torch.empty_like(y)
                _hip.call("smc_torgb_act_bwd_f32", grgb.contiguous().data_ptr(), rgb.data_ptr(), w_rgb.data_ptr(),
                          s_rgb.data_ptr(), ctx.clamp_rgb, _hip.ptr(gy.contiguous() if gy is not None else None),
                          y.data_ptr(), g.data_ptr(), n, c, w_rgb.shape[0], h, w,
                          ctypes.byref(_modconv_epi_bwd(ctx, d)), _hip.stream())
                dx, ds = _modconv_bwd(ctx, saved, None, need_dx, need_ds, g=g)
            else:
                gtot = gy.contiguous().clone() if gy is not None else torch.zeros_like(y)
                if grgb is not None:
                    _hip.call("smc_torgb_bwd_f32", grgb.contiguous().data_ptr(), rgb.data_ptr(), w_rgb.data_ptr(),
                              s_rgb.data_ptr(), gtot.data_ptr(), n, c, w_rgb.shape[0], h, w, ctx.clamp_rgb, 1, 1,
                              _hip.stream())
                dx, ds = _modconv_bwd(ctx, saved, gtot, need_dx, need_ds)
        return dx, ds, None, None, None, None, None, ds_rgb, None, None, None


class ToRGBFn(torch.autograd.Function):
    """y = clamp(sum_i W[c,i] s[n,i] x[n,i,p] + b[c]) (1x1 modconv, demodulate=False, linear bias_act)."""

    @staticmethod
    def forward(ctx, x, styles, weight2d, bias, clamp):
        x = x.contiguous()
        styles = styles.contiguous()
        y = _torgb_fwd(x, styles, weight2d, bias, clamp)
        ctx.clamp = clamp
        ctx.save_for_backward(x, styles, weight2d, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, styles, w2, y = ctx.saved_tensors
        n, cin, h, w = x.shape
        gy = gy.contiguous()
        dx = ds = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _hip.call("smc_torgb_bwd_f32", gy.data_ptr(), y.data_ptr(), w2.data_ptr(), styles.data_ptr(),
                      dx.data_ptr(), n, cin, w2.shape[0], h, w, ctx.clamp, 1, 0, _hip.stream())
        if ctx.needs_input_grad[1]:
            ds = _torgb_style_grad(gy, y, x, styles, w2, ctx.clamp)
        return dx, ds, None, None, None


def modulated_conv2d(x, weight, styles, noise=None, up=1, down=1, padding=0, resample_filter=None, demodulate=True,
                     flip_weight=True, fused_modconv=True, spec=None):
    """[upstream] modulated_conv2d signature, without bias/activation (gain 1, linear, no clamp).

    ``fused_modconv`` is accepted for signature compatibility; both forms compute the same function.
    Only the synthesis-network shapes are supported: 3x3 (up 1 or 2, padding 1, flip_weight = (up == 1))
    and 1x1 (up 1, padding 0).
    """
    if down != 1:
        raise NotImplementedError("modulated_conv2d: down > 1 is not on the synthesis path")
    k = weight.shape[-1]
    if k == 1 and up == 1 and not demodulate and noise is None and weight.shape[0] <= 4:
        return ToRGBFn.apply(x, styles, weight[:, :, 0, 0].detach().float().contiguous(), None, -1.0)
    if padding != k // 2 or flip_weight != (up == 1):
        raise NotImplementedError("modulated_conv2d: only padding=k//2 with flip_weight=(up==1) is supported")
    if spec is None:
        spec = LayerSpec(weight, None, up, resample_filter, demodulate=demodulate, act="linear")
    if noise is not None:
        strength = torch.ones([], device=x.device, dtype=torch.float32)
    else:
        strength = None
    return ModConvFn.apply(x, styles, spec, noise, strength, 1.0, -1.0)
