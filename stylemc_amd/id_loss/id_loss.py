"""Identity loss (id_loss/id_loss.py:7-39): 1 - <ArcFace(y_hat), ArcFace(y).detach()>, batch mean.

``extract_feats``: adaptive-avg-pool to 256 (4x4 mean at 1024 px), crop [35:223, 32:220], adaptive pool
to 112, IR-SE50, l2-normalised.  IR-SE50 runs on the gfx950 kernel library (``impl='hip'``, default:
stylemc_amd.irse_hip, BASELINE config 4) or on PyTorch-ROCm/MIOpen (``impl='torch'``, config 2).  The target image's features are computed under no_grad (the reference detaches them, :32), so the
backbone backward runs for y_hat only; the per-sample dot loop (id_loss.py:34-37) is a batched row dot.
"""
import os

import torch
import torch.nn.functional as F
from torch import nn

from .. import rowops
from .model_irse import build_irse50


# id_loss.py:20-23 geometry: pool to 256, crop [35:223, 32:220] (188 x 188), pool to 112
_POOL, _CROP, _OUT = 256, (35, 32, 188, 188), 112


class FaceCropFn(torch.autograd.Function):
    """The face crop as one gfx950 kernel each way (smc_face_crop_f32 / _bwd_f32)."""

    @staticmethod
    def forward(ctx, x):
        from .. import _hip
        x = x.contiguous()
        n, c, h, w = x.shape
        y = torch.empty(n, c, _OUT, _OUT, device=x.device, dtype=torch.float32)
        _hip.call("smc_face_crop_f32", _hip.ptr(x), n * c, h, w, _POOL, _POOL, *_CROP, _OUT, _OUT, y.data_ptr(),
                  _hip.stream())
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        from .. import _hip
        gy = gy.contiguous()
        n, c, h, w = ctx.shape
        dx = torch.empty(ctx.shape, device=gy.device, dtype=torch.float32)
        _hip.call("smc_face_crop_bwd_f32", _hip.ptr(gy), n * c, h, w, _POOL, _POOL, *_CROP, _OUT, _OUT, dx.data_ptr(),
                  _hip.stream())
        return dx


class IDLoss(nn.Module):
    def __init__(self, opts=None, facenet=None, weights="id_loss/model_ir_se50.pth", device="cuda", seed=3,
                 impl="hip"):
        super().__init__()
        if facenet is None:
            # like the reference (id_loss.py:12) a missing weights file is an error; weights=None asks for the
            # seeded synthetic IR-SE50 explicitly (tests, bench, --network synthetic)
            sd = None
            if weights is not None:
                if not os.path.exists(weights):
                    raise FileNotFoundError(f"{weights}: IR-SE50 ArcFace weights not found (the reference loads "
                                            f"id_loss/model_ir_se50.pth, id_loss.py:12); pass --id_weights, or "
                                            f"weights=None for seeded synthetic weights")
                sd = torch.load(weights, map_location="cpu", weights_only=True)
            if impl == "hip":
                from ..irse_hip import build_irse50 as build_hip
                facenet = build_hip(sd, seed=seed, device=device)
            elif impl == "torch":
                facenet = build_irse50(sd, seed=seed, device=device)
            else:
                raise ValueError(f"impl must be 'hip' or 'torch', got {impl!r}")
        self.facenet = facenet.eval()
        self.opts = opts
        self.fused_crop = impl == "hip"

    def face_crop(self, x):
        """id_loss.py:20-23: pool to 256, crop [35:223, 32:220], pool to 112 (one HIP kernel each way on the
        hip path when the input is an integer multiple of 256 px; the PyTorch ops otherwise)."""
        if (self.fused_crop and x.is_cuda and x.dtype == torch.float32 and x.shape[2] % _POOL == 0
                and x.shape[3] % _POOL == 0 and x.shape[3] // _POOL in (1, 2, 4)):
            return FaceCropFn.apply(x)
        if x.shape[2] != 256:
            x = F.adaptive_avg_pool2d(x, (256, 256))
        x = x[:, :, 35:223, 32:220]
        return F.adaptive_avg_pool2d(x, (112, 112))

    def extract_feats(self, x):
        return self.facenet(self.face_crop(x))

    def per_sample_pair(self, y_hat, y):
        """per_sample(y_hat, y) with both faces in ONE backbone batch [y_hat; y]: the backward runs for
        the y_hat half only (y's features are detached in the reference, id_loss.py:32)."""
        n = y_hat.shape[0]
        a = self.face_crop(y_hat)
        with torch.no_grad():
            b = self.face_crop(y)
        x = torch.cat([a, b])
        f = self.facenet(x, n_grad=n) if getattr(self.facenet, "supports_partial_grad", False) else self.facenet(x)
        return 1 - rowops.dot(f[:n], f[n:].detach())

    @torch.no_grad()
    def target_feats(self, y):
        """Features of the original image (detached in the reference, id_loss.py:32)."""
        return self.extract_feats(y)

    def per_sample_with(self, y_hat, y_feats):
        return 1 - rowops.dot(self.extract_feats(y_hat), y_feats)

    def per_sample(self, y_hat, y):
        """(1 - <f(y_hat_i), f(y_i)>) for each i; y's features are detached."""
        return self.per_sample_with(y_hat, self.target_feats(y))

    def forward(self, y_hat, y):
        return self.per_sample(y_hat, y).mean(), 0.0
