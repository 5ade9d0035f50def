"""Fused bias + activation on gfx950 -- drop-in for the reference's torch_utils/ops/bias_act.py.

Same public surface: ``activation_funcs`` (bias_act.py:23-33), ``bias_act(x, b, dim, act, alpha, gain,
clamp, impl)`` (bias_act.py:55-89) with 1st/2nd-order gradients.  ``impl='cuda'`` (the default, kept as
the name callers pass) runs the HIP kernel ``smc_bias_act_f32``; there is no silent fallback: CPU
tensors or ``impl='ref'`` raise (the pure-torch semantics live in the test oracle only).
"""
import math

import torch

from ... import _hip


class _Spec:
    def __init__(self, def_alpha, def_gain, cuda_idx, ref, has_2nd_grad):
        self.def_alpha, self.def_gain, self.cuda_idx, self.ref, self.has_2nd_grad = (
            def_alpha, def_gain, cuda_idx, ref, has_2nd_grad)


activation_funcs = {
    "linear": _Spec(0, 1, 1, "", False),
    "relu": _Spec(0, math.sqrt(2), 2, "y", False),
    "lrelu": _Spec(0.2, math.sqrt(2), 3, "y", False),
    "tanh": _Spec(0, 1, 4, "y", True),
    "sigmoid": _Spec(0, 1, 5, "y", True),
    "elu": _Spec(0, 1, 6, "y", True),
    "selu": _Spec(0, 1, 7, "y", True),
    "softplus": _Spec(0, 1, 8, "y", True),
    "swish": _Spec(0, math.sqrt(2), 9, "x", True),
}


def bias_act(x, b=None, dim=1, act="linear", alpha=None, gain=None, clamp=None, impl="cuda"):
    assert isinstance(x, torch.Tensor)
    if impl != "cuda":
        raise NotImplementedError("stylemc_amd.bias_act: only the HIP implementation ships (impl='cuda')")
    if not x.is_cuda:
        raise RuntimeError("stylemc_amd.bias_act: x must be a GPU tensor (no CPU fallback)")
    return _bias_act_fn(dim=dim, act=act, alpha=alpha, gain=gain, clamp=clamp).apply(x, b)


def _launch(x, b, xref, yref, dy, grad, dim, spec, alpha, gain, clamp):
    y = torch.empty_like(x, memory_format=torch.contiguous_format)
    size_b = b.numel() if b is not None else 0
    step_b = x.stride(dim) if b is not None else 1
    _hip.call("smc_bias_act_f32", _hip.ptr(x), _hip.ptr(b), _hip.ptr(xref), _hip.ptr(yref), _hip.ptr(dy),
              _hip.ptr(y), x.numel(), size_b, step_b, grad, spec.cuda_idx, alpha, gain, clamp, _hip.stream())
    return y


_cache = {}


def _bias_act_fn(dim=1, act="linear", alpha=None, gain=None, clamp=None):
    assert clamp is None or clamp >= 0
    spec = activation_funcs[act]
    alpha = float(alpha if alpha is not None else spec.def_alpha)
    gain = float(gain if gain is not None else spec.def_gain)
    clamp = float(clamp if clamp is not None else -1)
    key = (dim, act, alpha, gain, clamp)
    if key in _cache:
        return _cache[key]

    class BiasActHip(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, b):
            x = x.contiguous()
            b = b.contiguous() if b is not None else None
            if b is not None:
                assert b.ndim == 1 and b.shape[0] == x.shape[dim], "bias shape must match x.shape[dim]"
            y = x
            if act != "linear" or gain != 1 or clamp >= 0 or b is not None:
                y = _launch(x, b, None, None, None, 0, dim, spec, alpha, gain, clamp)
            keep_x = "x" in spec.ref or spec.has_2nd_grad
            # y is also kept for a clamped linear act so the backward masks like _bias_act_ref (the reference's
            # CUDA plugin saves no y for 'linear' and so ignores the clamp in its backward, bias_act.py:154-157).
            keep_y = "y" in spec.ref or (clamp >= 0 and y is not x)
            ctx.save_for_backward(x if keep_x else None, b if keep_x else None, y if keep_y else None)
            return y

        @staticmethod
        def backward(ctx, dy):
            dy = dy.contiguous()
            x, b, y = ctx.saved_tensors
            dx = db = None
            if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
                dx = dy
                if act != "linear" or gain != 1 or clamp >= 0:
                    dx = BiasActHipGrad.apply(dy, x, b, y)
            if ctx.needs_input_grad[1]:
                db = dx.sum([i for i in range(dx.ndim) if i != dim])
            return dx, db

    class BiasActHipGrad(torch.autograd.Function):
        @staticmethod
        def forward(ctx, dy, x, b, y):
            dx = _launch(dy, b, x, y, None, 1, dim, spec, alpha, gain, clamp)
            ctx.save_for_backward(dy if spec.has_2nd_grad else None, x, b, y)
            return dx

        @staticmethod
        def backward(ctx, d_dx):
            d_dx = d_dx.contiguous()
            dy, x, b, y = ctx.saved_tensors
            d_dy = d_x = d_b = None
            if ctx.needs_input_grad[0]:
                d_dy = BiasActHipGrad.apply(d_dx, x, b, y)
            if spec.has_2nd_grad and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2]):
                d_x = _launch(d_dx, b, x, y, dy, 2, dim, spec, alpha, gain, clamp)
            if spec.has_2nd_grad and ctx.needs_input_grad[2]:
                d_b = d_x.sum([i for i in range(d_x.ndim) if i != dim])
            return d_dy, d_x, d_b, None

    _cache[key] = BiasActHip
    return BiasActHip
