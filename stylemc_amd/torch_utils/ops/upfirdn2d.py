"""FIR resampling on gfx950 -- drop-in for the reference's torch_utils/ops/upfirdn2d.py.

Public surface kept: ``setup_filter`` (upfirdn2d.py:72-116), ``upfirdn2d`` (:120-164) with gradients of
any order (the backward is again upfirdn2d with up/down swapped and the taps flipped, :245-264),
``filter2d`` (:272-304), ``upsample2d`` (:308-343), ``downsample2d`` (:347-382).  Runs the HIP kernel
``smc_upfirdn2d_f32``; CPU tensors / ``impl='ref'`` raise instead of falling back.
"""
import numpy as np
import torch

from ... import _hip


def _parse_scaling(scaling):
    if isinstance(scaling, int):
        scaling = [scaling, scaling]
    sx, sy = scaling
    assert sx >= 1 and sy >= 1
    return int(sx), int(sy)


def _parse_padding(padding):
    if isinstance(padding, int):
        padding = [padding, padding]
    padding = list(padding)
    if len(padding) == 2:
        padx, pady = padding
        padding = [padx, padx, pady, pady]
    return tuple(int(p) for p in padding)


def _get_filter_size(f):
    if f is None:
        return 1, 1
    assert isinstance(f, torch.Tensor) and f.ndim in (1, 2)
    return int(f.shape[-1]), int(f.shape[0])


def setup_filter(f, device=torch.device("cpu"), normalize=True, flip_filter=False, gain=1, separable=None):
    if f is None:
        f = 1
    f = torch.as_tensor(f, dtype=torch.float32)
    assert f.ndim in (0, 1, 2) and f.numel() > 0
    if f.ndim == 0:
        f = f[np.newaxis]
    if separable is None:
        separable = f.ndim == 1 and f.numel() >= 8
    if f.ndim == 1 and not separable:
        f = torch.outer(f, f)
    assert f.ndim == (1 if separable else 2)
    if normalize:
        f = f / f.sum()
    if flip_filter:
        f = f.flip(list(range(f.ndim)))
    f = f * (gain ** (f.ndim / 2))
    return f.to(device=device)


def _launch(x, f, upx, upy, downx, downy, padx0, padx1, pady0, pady1, flip, gain):
    x = x.contiguous()
    f = f.to(device=x.device, dtype=torch.float32).contiguous()
    n, c, ih, iw = x.shape
    fh, fw = f.shape
    oh = (ih * upy + pady0 + pady1 - fh + downy) // downy
    ow = (iw * upx + padx0 + padx1 - fw + downx) // downx
    assert oh >= 1 and ow >= 1, "upfirdn2d: empty output"
    y = torch.empty([n, c, oh, ow], device=x.device, dtype=x.dtype)
    _hip.call("smc_upfirdn2d_f32", _hip.ptr(x), _hip.ptr(f), _hip.ptr(y), n * c, ih, iw, oh, ow, fh, fw, upx, upy,
              downx, downy, padx0, padx1, pady0, pady1, int(bool(flip)), float(gain), _hip.stream())
    return y


_cache = {}


def _upfirdn2d_fn(up=1, down=1, padding=0, flip_filter=False, gain=1):
    upx, upy = _parse_scaling(up)
    downx, downy = _parse_scaling(down)
    padx0, padx1, pady0, pady1 = _parse_padding(padding)
    key = (upx, upy, downx, downy, padx0, padx1, pady0, pady1, bool(flip_filter), float(gain))
    if key in _cache:
        return _cache[key]

    class Upfirdn2dHip(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, f):
            assert x.ndim == 4
            if f is None:
                f = torch.ones([1, 1], dtype=torch.float32, device=x.device)
            if f.ndim == 2:
                y = _launch(x, f, upx, upy, downx, downy, padx0, padx1, pady0, pady1, flip_filter, gain)
            else:
                g = float(np.sqrt(gain))
                y = _launch(x, f.unsqueeze(0), upx, 1, downx, 1, padx0, padx1, 0, 0, flip_filter, g)
                y = _launch(y, f.unsqueeze(1), 1, upy, 1, downy, 0, 0, pady0, pady1, flip_filter, g)
            ctx.save_for_backward(f)
            ctx.x_shape = x.shape
            return y

        @staticmethod
        def backward(ctx, dy):
            (f,) = ctx.saved_tensors
            _, _, ih, iw = ctx.x_shape
            _, _, oh, ow = dy.shape
            fw, fh = _get_filter_size(f)
            p = [fw - padx0 - 1, iw * upx - ow * downx + padx0 - upx + 1,
                 fh - pady0 - 1, ih * upy - oh * downy + pady0 - upy + 1]
            dx = None
            if ctx.needs_input_grad[0]:
                dx = _upfirdn2d_fn(up=[downx, downy], down=[upx, upy], padding=p, flip_filter=not flip_filter,
                                   gain=gain).apply(dy, f)
            assert not ctx.needs_input_grad[1], "gradients w.r.t. the filter are not supported"
            return dx, None

    _cache[key] = Upfirdn2dHip
    return Upfirdn2dHip


def upfirdn2d(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1, impl="cuda"):
    assert isinstance(x, torch.Tensor)
    if impl != "cuda":
        raise NotImplementedError("stylemc_amd.upfirdn2d: only the HIP implementation ships (impl='cuda')")
    if not x.is_cuda:
        raise RuntimeError("stylemc_amd.upfirdn2d: x must be a GPU tensor (no CPU fallback)")
    return _upfirdn2d_fn(up=up, down=down, padding=padding, flip_filter=flip_filter, gain=gain).apply(x, f)


def filter2d(x, f, padding=0, flip_filter=False, gain=1, impl="cuda"):
    padx0, padx1, pady0, pady1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    p = [padx0 + fw // 2, padx1 + (fw - 1) // 2, pady0 + fh // 2, pady1 + (fh - 1) // 2]
    return upfirdn2d(x, f, padding=p, flip_filter=flip_filter, gain=gain, impl=impl)


def upsample2d(x, f, up=2, padding=0, flip_filter=False, gain=1, impl="cuda"):
    upx, upy = _parse_scaling(up)
    padx0, padx1, pady0, pady1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    p = [padx0 + (fw + upx - 1) // 2, padx1 + (fw - upx) // 2, pady0 + (fh + upy - 1) // 2, pady1 + (fh - upy) // 2]
    return upfirdn2d(x, f, up=up, padding=p, flip_filter=flip_filter, gain=gain * upx * upy, impl=impl)


def downsample2d(x, f, down=2, padding=0, flip_filter=False, gain=1, impl="cuda"):
    downx, downy = _parse_scaling(down)
    padx0, padx1, pady0, pady1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    p = [padx0 + (fw - downx + 1) // 2, padx1 + (fw - downx) // 2, pady0 + (fh - downy + 1) // 2,
         pady1 + (fh - downy) // 2]
    return upfirdn2d(x, f, down=down, padding=p, flip_filter=flip_filter, gain=gain, impl=impl)
