"""CPU restatement of the reference's resampling / activation ops (TEST ORACLE ONLY).

Each function restates the *semantics* of the reference's pure-torch ``_ref`` path (the path the
reference itself falls back to when its CUDA plugin is unavailable), written independently:

  setup_filter      <- torch_utils/ops/upfirdn2d.py:72-116
  upfirdn2d         <- torch_utils/ops/upfirdn2d.py:168-208   (_upfirdn2d_ref)
  upsample2d        <- torch_utils/ops/upfirdn2d.py:308-343
  downsample2d      <- torch_utils/ops/upfirdn2d.py:347-382
  filter2d          <- torch_utils/ops/upfirdn2d.py:272-304
  upfirdn2d_adjoint_padding <- torch_utils/ops/upfirdn2d.py:247-261 (backward padding rule)
  bias_act          <- torch_utils/ops/bias_act.py:93-123     (_bias_act_ref)
  bias_act_grad     <- torch_utils/ops/bias_act.cu:23-147     (grad=1 semantics: the clamp mask
                       zeroes the gradient at |y| == clamp, unlike torch's clamp backward)
  conv2d_resample   <- torch_utils/ops/conv2d_resample.py:58-154 (+ _conv2d_wrapper 29-54)
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

# name -> (function(x, alpha), default alpha, default gain, which saved tensor the grad needs)
_ACTS = {
    "linear": (lambda x, a: x, 0.0, 1.0, ""),
    "relu": (lambda x, a: F.relu(x), 0.0, math.sqrt(2.0), "y"),
    "lrelu": (lambda x, a: F.leaky_relu(x, a), 0.2, math.sqrt(2.0), "y"),
    "tanh": (lambda x, a: torch.tanh(x), 0.0, 1.0, "y"),
    "sigmoid": (lambda x, a: torch.sigmoid(x), 0.0, 1.0, "y"),
    "elu": (lambda x, a: F.elu(x), 0.0, 1.0, "y"),
    "selu": (lambda x, a: F.selu(x), 0.0, 1.0, "y"),
    "softplus": (lambda x, a: F.softplus(x), 0.0, 1.0, "y"),
    "swish": (lambda x, a: torch.sigmoid(x) * x, 0.0, math.sqrt(2.0), "x"),
}


def act_defaults(act):
    fn, alpha, gain, _ = _ACTS[act]
    return alpha, gain


def _pair(v):
    if isinstance(v, int):
        return v, v
    a, b = v
    return int(a), int(b)


def _pad4(p):
    if isinstance(p, int):
        return p, p, p, p
    p = list(p)
    if len(p) == 2:
        return p[0], p[0], p[1], p[1]
    return tuple(int(v) for v in p)


def filter_size(f):
    if f is None:
        return 1, 1
    return int(f.shape[-1]), int(f.shape[0])


def setup_filter(f, normalize=True, flip_filter=False, gain=1, separable=None):
    """2-D FIR taps as float32 (upfirdn2d.py:72-116)."""
    t = torch.as_tensor(1 if f is None else f, dtype=torch.float32)
    if t.ndim == 0:
        t = t.reshape(1)
    if separable is None:
        separable = t.ndim == 1 and t.numel() >= 8
    if t.ndim == 1 and not separable:
        t = torch.outer(t, t)
    if normalize:
        t = t / t.sum()
    if flip_filter:
        t = torch.flip(t, dims=list(range(t.ndim)))
    return t * (gain ** (t.ndim / 2))


def upfirdn2d(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1):
    """zero-insert upsample -> pad/crop -> FIR (convolution unless flip_filter) -> decimate."""
    if f is None:
        f = torch.ones(1, 1, dtype=torch.float32)
    ux, uy = _pair(up)
    dx, dy = _pair(down)
    px0, px1, py0, py1 = _pad4(padding)
    n, c, h, w = x.shape
    # 1. zero insertion: place x at every (uy, ux)-th sample.
    if ux > 1 or uy > 1:
        z = x.new_zeros(n, c, h * uy, w * ux)
        z[:, :, ::uy, ::ux] = x
        x = z
    # 2. pad with zeros (positive) / crop (negative).
    x = F.pad(x, [max(px0, 0), max(px1, 0), max(py0, 0), max(py1, 0)])
    x = x[:, :, max(-py0, 0): x.shape[2] - max(-py1, 0), max(-px0, 0): x.shape[3] - max(-px1, 0)]
    # 3. FIR.  conv2d correlates, so flip the taps to convolve (the reference default).
    taps = f.to(x.dtype) * (gain ** (f.ndim / 2))
    if not flip_filter:
        taps = torch.flip(taps, dims=list(range(taps.ndim)))
    if taps.ndim == 2:
        x = F.conv2d(x, taps.expand(c, 1, *taps.shape).contiguous(), groups=c)
    else:
        x = F.conv2d(x, taps.reshape(1, 1, 1, -1).expand(c, 1, 1, -1).contiguous(), groups=c)
        x = F.conv2d(x, taps.reshape(1, 1, -1, 1).expand(c, 1, -1, 1).contiguous(), groups=c)
    # 4. keep every (dy, dx)-th sample.
    return x[:, :, ::dy, ::dx]


def upfirdn2d_out_size(in_h, in_w, fh, fw, up, down, padding):
    ux, uy = _pair(up)
    dx, dy = _pair(down)
    px0, px1, py0, py1 = _pad4(padding)
    oh = (in_h * uy + py0 + py1 - fh + dy) // dy
    ow = (in_w * ux + px0 + px1 - fw + dx) // dx
    return oh, ow


def upfirdn2d_adjoint_padding(in_h, in_w, out_h, out_w, fh, fw, up, down, padding):
    """Padding of the adjoint upfirdn2d (up<->down swapped, filter flipped): upfirdn2d.py:251-256."""
    ux, uy = _pair(up)
    dx, dy = _pair(down)
    px0, px1, py0, py1 = _pad4(padding)
    return [fw - px0 - 1, in_w * ux - out_w * dx + px0 - ux + 1,
            fh - py0 - 1, in_h * uy - out_h * dy + py0 - uy + 1]


def upsample2d(x, f, up=2, padding=0, flip_filter=False, gain=1):
    ux, uy = _pair(up)
    px0, px1, py0, py1 = _pad4(padding)
    fw, fh = filter_size(f)
    pad = [px0 + (fw + ux - 1) // 2, px1 + (fw - ux) // 2, py0 + (fh + uy - 1) // 2, py1 + (fh - uy) // 2]
    return upfirdn2d(x, f, up=up, padding=pad, flip_filter=flip_filter, gain=gain * ux * uy)


def downsample2d(x, f, down=2, padding=0, flip_filter=False, gain=1):
    dx, dy = _pair(down)
    px0, px1, py0, py1 = _pad4(padding)
    fw, fh = filter_size(f)
    pad = [px0 + (fw - dx + 1) // 2, px1 + (fw - dx) // 2, py0 + (fh - dy + 1) // 2, py1 + (fh - dy) // 2]
    return upfirdn2d(x, f, down=down, padding=pad, flip_filter=flip_filter, gain=gain)


def filter2d(x, f, padding=0, flip_filter=False, gain=1):
    px0, px1, py0, py1 = _pad4(padding)
    fw, fh = filter_size(f)
    pad = [px0 + fw // 2, px1 + (fw - 1) // 2, py0 + fh // 2, py1 + (fh - 1) // 2]
    return upfirdn2d(x, f, padding=pad, flip_filter=flip_filter, gain=gain)


def _resolve(act, alpha, gain, clamp):
    fn, a0, g0, _ = _ACTS[act]
    alpha = float(a0 if alpha is None else alpha)
    gain = float(g0 if gain is None else gain)
    clamp = float(-1 if clamp is None else clamp)
    return fn, alpha, gain, clamp


def bias_act(x, b=None, dim=1, act="linear", alpha=None, gain=None, clamp=None):
    """y = clamp(act(x + b) * gain, -clamp, clamp)  (bias_act.py:93-123)."""
    fn, alpha, gain, clamp = _resolve(act, alpha, gain, clamp)
    if b is not None:
        shape = [1] * x.ndim
        shape[dim] = -1
        x = x + b.reshape(shape)
    x = fn(x, alpha)
    if gain != 1:
        x = x * gain
    if clamp >= 0:
        x = x.clamp(-clamp, clamp)
    return x


def bias_act_grad(dy, y, act="lrelu", alpha=None, gain=None, clamp=None):
    """dx of bias_act for the y-referenced activations, CUDA-kernel semantics (bias_act.cu:51-142).

    Only the activations whose gradient is a function of the output y (linear/relu/lrelu) are
    needed on the hot path.  dx = dy * gain * act'(y / gain), zeroed where |y| >= clamp.
    """
    _, alpha, gain, clamp = _resolve(act, alpha, gain, clamp)
    if act == "linear":
        dx = dy * gain
    elif act == "relu":
        dx = torch.where(y > 0, dy, torch.zeros_like(dy)) * gain
    elif act == "lrelu":
        dx = torch.where(y > 0, dy, dy * alpha) * gain
    else:
        raise NotImplementedError(act)
    if clamp >= 0:
        dx = torch.where((y > -clamp) & (y < clamp), dx, torch.zeros_like(dx))
    return dx


def conv2d_resample(x, w, f=None, up=1, down=1, padding=0, groups=1, flip_weight=True, flip_filter=False):
    """Convolution with fused FIR up/down-sampling (conv2d_resample.py:58-154).

    Only the routes the synthesis network uses are restated: plain conv (up=down=1, symmetric
    padding), the 1x1 fast paths, up>1 via stride-`up` transposed convolution followed by the
    FIR, and down>1 via FIR followed by a strided convolution.
    """
    oc, icpg, kh, kw = w.shape
    fw, fh = filter_size(f)
    px0, px1, py0, py1 = _pad4(padding)
    if up > 1:
        px0 += (fw + up - 1) // 2
        px1 += (fw - up) // 2
        py0 += (fh + up - 1) // 2
        py1 += (fh - up) // 2
    if down > 1:
        px0 += (fw - down + 1) // 2
        px1 += (fw - down) // 2
        py0 += (fh - down + 1) // 2
        py1 += (fh - down) // 2

    def conv(x, w, stride=1, pad=0, transpose=False, flip=True):
        if not flip:  # F.conv2d correlates; a convolution needs the flipped kernel.
            w = torch.flip(w, [2, 3])
        if transpose:
            return F.conv_transpose2d(x, w, stride=stride, padding=pad, groups=groups)
        return F.conv2d(x, w, stride=stride, padding=pad, groups=groups)

    if kh == 1 and kw == 1 and down > 1 and up == 1:
        x = upfirdn2d(x, f, down=down, padding=[px0, px1, py0, py1], flip_filter=flip_filter)
        return conv(x, w, flip=flip_weight)
    if kh == 1 and kw == 1 and up > 1 and down == 1:
        x = conv(x, w, flip=flip_weight)
        return upfirdn2d(x, f, up=up, padding=[px0, px1, py0, py1], gain=up * up, flip_filter=flip_filter)
    if down > 1 and up == 1:
        x = upfirdn2d(x, f, padding=[px0, px1, py0, py1], flip_filter=flip_filter)
        return conv(x, w, stride=down, flip=flip_weight)
    if up > 1:
        # [groups*oc/g, icpg, kh, kw] -> [groups*icpg, oc/g, kh, kw] for conv_transpose2d.
        wt = w.reshape(groups, oc // groups, icpg, kh, kw).transpose(1, 2).reshape(groups * icpg, oc // groups, kh, kw)
        px0 -= kw - 1
        px1 -= kw - up
        py0 -= kh - 1
        py1 -= kh - up
        pxt = max(min(-px0, -px1), 0)
        pyt = max(min(-py0, -py1), 0)
        x = conv(x, wt, stride=up, pad=[pyt, pxt], transpose=True, flip=not flip_weight)
        x = upfirdn2d(x, f, padding=[px0 + pxt, px1 + pxt, py0 + pyt, py1 + pyt], gain=up * up, flip_filter=flip_filter)
        if down > 1:
            x = upfirdn2d(x, f, down=down, flip_filter=flip_filter)
        return x
    if px0 == px1 and py0 == py1 and px0 >= 0 and py0 >= 0:
        return conv(x, w, pad=[py0, px0], flip=flip_weight)
    x = upfirdn2d(x, None, padding=[px0, px1, py0, py1])
    return conv(x, w, flip=flip_weight)


def fma(a, b, c):
    """a * b + c  (fma.py:15-16)."""
    return torch.addcmul(c, a, b)


_ = np  # numpy kept for callers that pass arrays to setup_filter
