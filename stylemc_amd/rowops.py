"""Batch-invariant row reductions of the loss heads (csrc/heads.hip).

The loss heads of find_direction reduce embedding rows -- norms, cosines, dot products (clip_loss.py:28-34,
id_loss/id_loss.py:26-39, model_irse.py:48).  ATen's row reduction chooses its block shape from the number of rows,
so the same row summed in a batch of 2 and in a batch of 4 can differ in the last bit; a data-parallel shard would
then not reproduce the single-process gradient exactly.  These ops reduce each row on one wave in a fixed order
(``smc_row_dot_f32`` / ``smc_direction_head_f32``), whatever the batch.  GPU tensors only; the CPU tensors of the
host-logic tests take the torch expressions.
"""
import torch

from . import _hip


def row_dot(a, b):
    """[R, L] x [R or 1, L] -> [R] (no autograd)."""
    if not a.is_cuda:
        return (a * b).sum(1)
    a = a.contiguous().float()
    b = b.contiguous().float()
    rows, L = a.shape
    if b.ndim != 2 or b.shape[1] != L or b.shape[0] not in (1, rows):
        raise ValueError(f"row_dot: b {tuple(b.shape)} must be [1 or {rows}, {L}]")
    out = torch.empty(rows, device=a.device, dtype=torch.float32)
    if rows == 0:
        return out
    ldb = 0 if b.shape[0] == 1 and rows > 1 else L
    _hip.call("smc_row_dot_f32", _hip.ptr(a), L, _hip.ptr(b), ldb, out.data_ptr(), rows, L, _hip.stream())
    return out


class _RowDot(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return row_dot(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = g[:, None] * b if ctx.needs_input_grad[0] else None
        gb = None
        if ctx.needs_input_grad[1]:
            gb = g[:, None] * a
            if b.shape[0] == 1 and a.shape[0] > 1:
                gb = gb.sum(0, keepdim=True)
        return ga, gb


def dot(a, b):
    """sum(a * b, dim=1) with autograd; batch-invariant on the GPU."""
    if not a.is_cuda:
        return (a * b).sum(1)
    return _RowDot.apply(a, b)


class _L2Normalize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f):
        nrm = row_dot(f, f).sqrt_()[:, None]
        y = f / nrm
        ctx.save_for_backward(y, nrm)
        return y

    @staticmethod
    def backward(ctx, g):
        y, nrm = ctx.saved_tensors
        return (g - y * row_dot(g, y)[:, None]) / nrm


def l2_normalize(f):
    """f / ||f||_2 per row (model_irse.py:48 l2_norm) with autograd; batch-invariant on the GPU."""
    if not f.is_cuda:
        return f / torch.norm(f, 2, 1, True)
    return _L2Normalize.apply(f)


def direction_head(e, src, t, eps=1e-8):
    """(1 - cos(normalize(e - src), t), d/de) per row in one launch (smc_direction_head_f32); e, src: [R, D], t: [1, D]."""
    if e.dtype != torch.float32 or src.dtype != torch.float32 or t.dtype != torch.float32:
        raise ValueError("direction_head: fp32 tensors only")
    if e.ndim != 2 or src.shape != e.shape or t.shape != (1, e.shape[1]):
        raise ValueError(f"direction_head: e {tuple(e.shape)}, src {tuple(src.shape)} (same), t {tuple(t.shape)} "
                         f"(1 x D)")
    e = e if e.stride(-1) == 1 else e.contiguous()
    src = src if src.stride(-1) == 1 else src.contiguous()
    t = t.contiguous()
    rows, D = e.shape
    loss = torch.empty(rows, device=e.device, dtype=torch.float32)
    grad = torch.empty(rows, D, device=e.device, dtype=torch.float32)
    if rows == 0:
        return loss, grad
    _hip.call("smc_direction_head_f32", _hip.ptr(e), e.stride(0), _hip.ptr(src), src.stride(0), _hip.ptr(t),
              loss.data_ptr(), grad.data_ptr(), rows, D, float(eps), _hip.stream())
    return loss, grad
