"""ArcFace IR-SE50 on the gfx950 kernel library (BASELINE config 4: "id_loss IR-SE50 on HIP").

Drop-in for ``Backbone(112, 50, 'ir_se')`` of the reference (id_loss/model_irse.py:10-49,
helpers.py:56-119) as IDLoss.extract_feats runs it (id_loss/id_loss.py:20-24): same state_dict
(``input_layer``, ``body.{k}.{shortcut_layer,res_layer}``, ``output_layer``), eval mode, frozen.
The network is described to the native executor (``smc_irse_forward_f32`` / ``smc_irse_backward_f32``)
once: every convolution packed for the MFMA gather GEMM (forward taps [t][cin][cout]; adjoint taps
[t][cout][cin], stride-2 adjoints as 4 polyphase phases), eval BatchNorms as per-channel (a, b) --
folded into the adjoint weights, and for the output layer into the final Linear (BatchNorm2d ->
flatten -> Linear -> BatchNorm1d becomes one affine map, folded in float64).
"""
import ctypes

import torch
from torch import nn

from . import _hip, rowops
from .id_loss.model_irse import Backbone
from . import modconv
from .modconv import _phase

P = ctypes.c_void_p
# The 3x3 stride-1 convs of the <= 16x16 stages (14x14 x 256, 7x7 x 512) and their adjoints run as small-plane
# Winograd F(2x2, 3x3) with split-K (csrc/wino_sp.hip); module switch (tests / tools flip it for the direct GEMM).
WINO_SP = True


class IrseUnit(ctypes.Structure):
    _fields_ = [("cin", ctypes.c_int), ("depth", ctypes.c_int), ("stride", ctypes.c_int), ("in_h", ctypes.c_int),
                ("in_w", ctypes.c_int), ("bn1_a", P), ("bn1_b", P), ("c1_fwd", _hip.ConvPhase),
                ("c1_bwd", _hip.ConvPhase), ("prelu", P), ("c2_fwd", _hip.ConvPhase),
                ("c2_bwd", _hip.ConvPhase * 4), ("c2_bwd_nphases", ctypes.c_int), ("bn2_a", P), ("bn2_b", P),
                ("se_w1", P), ("se_w2", P), ("se_hidden", ctypes.c_int), ("sc_conv", ctypes.c_int),
                ("sc_fwd", _hip.ConvPhase), ("sc_bwd", _hip.ConvPhase), ("sc_a", P), ("sc_b", P)]


class IrseNet(ctypes.Structure):
    _fields_ = [("n_units", ctypes.c_int), ("units", P), ("in_h", ctypes.c_int), ("in_w", ctypes.c_int),
                ("img_ch", ctypes.c_int), ("stem_cin", ctypes.c_int), ("stem_cout", ctypes.c_int),
                ("stem_fwd", _hip.ConvPhase), ("stem_bwd", _hip.ConvPhase), ("stem_bn_a", P), ("stem_bn_b", P),
                ("stem_prelu", P), ("feat", ctypes.c_int), ("flat", ctypes.c_int), ("fc_wt", P), ("fc_w", P),
                ("fc_b", P)]


def bn_affine(bn):
    """Eval-mode BatchNorm as y = x * a + b (float64 math, fp32 result)."""
    rv, rm = bn.running_var.detach().double().cpu(), bn.running_mean.detach().double().cpu()
    w = bn.weight.detach().double().cpu() if bn.weight is not None else torch.ones_like(rv)
    b = bn.bias.detach().double().cpu() if bn.bias is not None else torch.zeros_like(rv)
    a = w / torch.sqrt(rv + bn.eps)
    return a, b - rm * a


def fwd_taps(W):
    """[t][cin][cout] packing and tap offsets of a same-padded k x k conv (k = 1 or 3)."""
    cout, cin, k, _ = W.shape
    c = k // 2
    taps = [(ky - c, kx - c) for ky in range(k) for kx in range(k)]
    return taps, W.permute(2, 3, 1, 0).reshape(k * k, cin, cout)


def adj_weight(W, ky, kx, in_scale=None, out_scale=None):
    """Adjoint tap [cout_fwd][cin_fwd] = W[:, :, ky, kx] scaled by the BN that follows (out) / precedes (in)."""
    w = W[:, :, ky, kx].double()
    if out_scale is not None:
        w = w * out_scale[:, None]
    if in_scale is not None:
        w = w * in_scale[None, :]
    return w


# Split-bf16 products for the executor's direct GEMMs (include/stylemc_hip.h smc_conv_phase.wk_x3).  Off: the IR-SE50
# input gradient of these seeded weights is ill-conditioned (PReLU kinks: the fp32 CPU path itself is 6.4e-3 of the max
# away from fp64 at 4 / 8 faces), and the split products move which kinks flip -- x3 1e-6 / 3e-3 / 6e-3 against fp32
# 1e-4 / 8e-5 / 9e-7 at 4 / 1 / 8 faces, cosine >= 0.9999994 either way (profiles/r04/irse_x3_diag.txt) -- for a
# 0.1 ms / step kernel-time gain (r05: +0.7 % images/s, profiles/r05/ab5/).  Round 5 showed the flips are the gradient's
# own: the fp64 gradient at an input one fp32 rounding away moves by up to 4.9e-3 of the max
# (profiles/r05/x3_accuracy/irse_x3_conditioning.txt).  The reference-pinned tolerances stay those of the exact-fp32
# products.
X3 = False


class _Packed:
    """Device tensors + ctypes descriptors of one IR-SE50 (kept alive together)."""

    def __init__(self, net: Backbone, device, in_hw=112):
        self.keep = []
        dev = torch.device(device)

        def d(t):
            t = t.detach().to(dev, torch.float32).contiguous()
            self.keep.append(t)
            return t

        def ptr(t):
            return d(t).data_ptr()

        def phase(taps, stride, oh, ow, wk, oy=0, ox=0, sy=1, sx=1):
            wk = d(wk)
            # split-bf16 planes for the direct GEMMs (X3 below; kept alive with the packed weights)
            wx = modconv.x3_planes(wk, wk.shape[1], wk.shape[2], enabled=X3)
            if wx is not None:
                self.keep.append(wx)
            return _phase(taps, stride, oh, ow, oy, ox, sy, sx, wk, wx)

        def same_adjoint(W, h, w, in_scale=None, out_scale=None):
            k = W.shape[2]
            c = k // 2
            taps, wks = [], []
            for ky in range(k):
                for kx in range(k):
                    taps.append((c - ky, c - kx))
                    wks.append(adj_weight(W, ky, kx, in_scale, out_scale))
            return phase(taps, 1, h, w, torch.stack(wks))

        lib = _hip.load()

        def wino(ph, cin, cout, hw):
            """Small-plane Winograd taps (smc_wino_taps_f32) for a 9-tap 3x3 stride-1 'same' phase whose planes
            (hw x hw) the smc_conv3x3_wino_sp_f32 kernel takes: the executor then runs that conv as F(2x2, 3x3)."""
            if not WINO_SP or dev.type != "cuda" or not lib.smc_wino_sp_supported(1, cin, cout, hw, hw):
                return ph  # (a host-side descriptor build keeps the implicit-GEMM phases; the taps are device data)
            uw = torch.empty(16 * cin * cout, device=dev, dtype=torch.float32)
            _hip.call("smc_wino_taps_f32", ctypes.byref(ph), cin, cout, uw.data_ptr(), _hip.stream())
            self.keep.append(uw)
            ph.wino_u = uw.data_ptr()
            return ph

        def stride2_adjoint(W, oh, ow, out_scale):
            # forward out[a] = sum_k W[k] x[2a + k - 1]  ->  d x[2a+p] gathers (p=0: k=1 at a; p=1: k=2 at a, k=0 at a+1)
            sel = {0: [(0, 1)], 1: [(0, 2), (1, 0)]}
            phases = []
            for py in (0, 1):
                for px in (0, 1):
                    taps, wks = [], []
                    for oy, ky in sel[py]:
                        for ox, kx in sel[px]:
                            taps.append((oy, ox))
                            wks.append(adj_weight(W, ky, kx, None, out_scale))
                    phases.append(phase(taps, 1, oh, ow, torch.stack(wks), py, px, 2, 2))
            return phases

        # ---- stem: Conv2d(3, 64, 3, 1, 1) + BN + PReLU; the face is padded to 16 channels
        conv, bn, prelu = net.input_layer[0], net.input_layer[1], net.input_layer[2]
        W = conv.weight.detach().double().cpu()
        cout, img_ch = W.shape[0], W.shape[1]
        cin_p = (img_ch + 15) // 16 * 16
        Wp = torch.zeros(cout, cin_p, 3, 3, dtype=torch.float64)
        Wp[:, :img_ch] = W
        a, b = bn_affine(bn)
        self.net = IrseNet()
        nt = self.net
        nt.in_h = nt.in_w = in_hw
        nt.img_ch, nt.stem_cin, nt.stem_cout = img_ch, cin_p, cout
        taps, wk = fwd_taps(Wp)
        nt.stem_fwd = phase(taps, 1, in_hw, in_hw, wk)
        nt.stem_bwd = same_adjoint(Wp, in_hw, in_hw, out_scale=a)
        nt.stem_bn_a, nt.stem_bn_b, nt.stem_prelu = ptr(a), ptr(b), ptr(prelu.weight)

        # ---- bottleneck units
        units = []
        hw = in_hw
        for blk in net.body:
            u = IrseUnit()
            res = blk.res_layer
            bn1, c1, pr, c2, bn2 = res[0], res[1], res[2], res[3], res[4]
            se = res[5]
            W1, W2 = c1.weight.detach().double().cpu(), c2.weight.detach().double().cpu()
            u.cin, u.depth = W1.shape[1], W1.shape[0]
            s = c2.stride[0]
            u.stride, u.in_h, u.in_w = s, hw, hw
            oh = hw // s
            a1, b1 = bn_affine(bn1)
            a2, b2 = bn_affine(bn2)
            u.bn1_a, u.bn1_b = ptr(a1), ptr(b1)
            taps, wk = fwd_taps(W1)
            u.c1_fwd = wino(phase(taps, 1, hw, hw, wk), u.cin, u.depth, hw)
            u.c1_bwd = wino(same_adjoint(W1, hw, hw, in_scale=a1), u.depth, u.cin, hw)
            u.prelu = ptr(pr.weight)
            taps, wk = fwd_taps(W2)
            u.c2_fwd = phase(taps, s, oh, oh, wk)
            if s == 1:
                u.c2_fwd = wino(u.c2_fwd, u.depth, u.depth, hw)
                u.c2_bwd[0] = wino(same_adjoint(W2, hw, hw, out_scale=a2), u.depth, u.depth, hw)
                u.c2_bwd_nphases = 1
            else:
                for i, ph in enumerate(stride2_adjoint(W2, oh, oh, a2)):
                    u.c2_bwd[i] = ph
                u.c2_bwd_nphases = 4
            u.bn2_a, u.bn2_b = ptr(a2), ptr(b2)
            u.se_w1 = ptr(se.fc1.weight.reshape(se.fc1.weight.shape[0], -1))
            u.se_w2 = ptr(se.fc2.weight.reshape(se.fc2.weight.shape[0], -1))
            u.se_hidden = se.fc1.weight.shape[0]
            if isinstance(blk.shortcut_layer, nn.Sequential):
                sconv, sbn = blk.shortcut_layer[0], blk.shortcut_layer[1]
                Ws = sconv.weight.detach().double().cpu()
                sa, sb = bn_affine(sbn)
                u.sc_conv = 1
                u.sc_fwd = phase([(0, 0)], sconv.stride[0], oh, oh, Ws[:, :, 0, 0].t().reshape(1, u.cin, u.depth))
                u.sc_bwd = phase([(0, 0)], 1, oh, oh, adj_weight(Ws, 0, 0, None, sa).reshape(1, u.depth, u.cin))
                u.sc_a, u.sc_b = ptr(sa), ptr(sb)
            else:
                u.sc_conv = 0
            units.append(u)
            hw = oh
        self.units = (IrseUnit * len(units))(*units)
        nt.n_units = len(units)
        nt.units = ctypes.cast(self.units, P)

        # ---- output layer: BatchNorm2d -> Dropout (eval: identity) -> flatten -> Linear -> BatchNorm1d
        bno, fc, bnf = net.output_layer[0], net.output_layer[3], net.output_layer[4]
        ao, bo = bn_affine(bno)
        af, bf = bn_affine(bnf)
        Wl = fc.weight.detach().double().cpu()                     # [feat][flat], flat index = c*hw*hw + p
        feat, flat = Wl.shape
        rep = flat // ao.numel()
        Wf = Wl * ao.repeat_interleave(rep)[None, :]
        fb = fc.bias.detach().double().cpu() + Wl @ bo.repeat_interleave(rep)
        Wf = Wf * af[:, None]
        fb = fb * af + bf
        nt.feat, nt.flat = feat, flat
        nt.fc_wt, nt.fc_w, nt.fc_b = ptr(Wf.t()), ptr(Wf), ptr(fb)
        if dev.type == "cuda":  # the packed weights (and Winograd taps) are complete before any stream reads them
            torch.cuda.current_stream(dev).synchronize()


class _IrseFn(torch.autograd.Function):
    """Backbone forward (features before the l2 norm) / input gradient of the leading n_grad faces."""

    @staticmethod
    def forward(ctx, x, mod, n_grad=None):
        if not x.is_cuda:
            raise RuntimeError("HipIRSE50 runs on the GPU only (got a CPU tensor)")
        x = x.to(torch.float32).contiguous()
        n = x.shape[0]
        pk = mod.packed_net()
        net = ctypes.byref(pk.net)
        if tuple(x.shape[1:]) != (pk.net.img_ch, pk.net.in_h, pk.net.in_w):
            raise ValueError(f"HipIRSE50 expects [n, {pk.net.img_ch}, {pk.net.in_h}, {pk.net.in_w}], got {tuple(x.shape)}")
        lib = _hip.load()
        feat = torch.empty(n, pk.net.feat, device=x.device, dtype=torch.float32)
        saved = None
        if ctx.needs_input_grad[0]:
            saved = torch.empty(lib.smc_irse_saved_floats(net, n), device=x.device, dtype=torch.float32)
        wsb = lib.smc_irse_workspace_bytes(net, n)
        ws = torch.empty(wsb // 4, device=x.device, dtype=torch.float32)
        _hip.call("smc_irse_forward_f32", net, x.data_ptr(), n, feat.data_ptr(), _hip.ptr(saved), ws.data_ptr(), wsb,
                  _hip.stream())
        ctx.mod, ctx.saved_buf, ctx.shape = mod, saved, x.shape
        ctx.n_grad = n if n_grad is None else int(n_grad)
        if not 1 <= ctx.n_grad <= n:
            raise ValueError(f"n_grad {n_grad} not in [1, {n}]")
        return feat

    @staticmethod
    def backward(ctx, gfeat):
        pk = ctx.mod.packed_net()
        net = ctypes.byref(pk.net)
        n, nr = ctx.shape[0], ctx.n_grad
        gfeat = gfeat[:nr].to(torch.float32).contiguous()
        lib = _hip.load()
        dx = (torch.empty if nr == n else torch.zeros)(ctx.shape, device=gfeat.device, dtype=torch.float32)
        wsb = lib.smc_irse_workspace_bytes(net, nr)
        ws = torch.empty(wsb // 4, device=gfeat.device, dtype=torch.float32)
        _hip.call("smc_irse_backward_f32", net, gfeat.data_ptr(), n, nr, ctx.saved_buf.data_ptr(), dx.data_ptr(),
                  ws.data_ptr(), wsb, _hip.stream())
        ctx.saved_buf = None
        return dx, None, None


class HipIRSE50(nn.Module):
    """IR-SE50 (state_dict-compatible with the reference Backbone) executed by the gfx950 kernel library."""

    def __init__(self, input_size=112, num_layers=50, mode="ir_se", drop_ratio=0.6, affine=True):
        super().__init__()
        self.body_net = Backbone(input_size, num_layers, mode, drop_ratio, affine)
        self.input_size = input_size
        self._packed = None

    def state_dict(self, *args, **kwargs):
        return self.body_net.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        r = self.body_net.load_state_dict(state_dict, strict=strict, assign=assign)
        self._packed = None
        return r

    def _apply(self, fn, *args, **kwargs):
        super()._apply(fn, *args, **kwargs)
        self._packed = None
        return self

    def packed_net(self):
        if self._packed is None:
            dev = next(self.body_net.parameters()).device
            self._packed = _Packed(self.body_net.eval(), dev, self.input_size)
        return self._packed

    supports_partial_grad = True

    def forward(self, x, n_grad=None):
        """n_grad: back-propagate only the leading n_grad faces (the rest get a zero gradient)."""
        f = _IrseFn.apply(x, self, n_grad)
        return rowops.l2_normalize(f)          # model_irse.py:48 l2_norm (rows in a fixed order)


def build_irse50(state_dict=None, seed=3, device="cuda"):
    from . import synthetic
    net = HipIRSE50(input_size=112, num_layers=50, mode="ir_se", drop_ratio=0.6)
    net.body_net.load_state_dict(state_dict if state_dict is not None else
                                 synthetic.seeded_state_dict(net.body_net, seed=seed))
    net = net.eval().requires_grad_(False).to(device)
    net.packed_net()
    return net
