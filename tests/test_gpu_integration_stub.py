"""INTEGRATION.md section 3 executed: the ctypes `_plugin` stub a maintainer would drop into the reference's
torch_utils/ops, called exactly the way the reference's op modules call their plugin
(bias_act.py:153,182 and upfirdn2d.py:237-240, 245-264), against the golden vectors the reference's own ops
produced (tests/golden/ops_bias_act.npz, ops_upfirdn2d.npz).  Catches any drift between the documented
binding (argument order, types, activation codes) and the C ABI in include/stylemc_hip.h.

Tolerances as tests/test_gpu_ops.py: 1e-5 of the tensor's max magnitude.
"""
import os
import re

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = "cuda"
# reference bias_act.py:24-32: name -> (cuda_idx, def_alpha, def_gain, ref, has_2nd_grad)
ACTS = {"linear": (1, 0.0, 1.0, "", False), "relu": (2, 0.0, np.sqrt(2), "y", False),
        "lrelu": (3, 0.2, np.sqrt(2), "y", False), "tanh": (4, 0.0, 1.0, "y", True),
        "sigmoid": (5, 0.0, 1.0, "y", True), "elu": (6, 0.0, 1.0, "y", True), "selu": (7, 0.0, 1.0, "y", True),
        "softplus": (8, 0.0, 1.0, "y", True), "swish": (9, 0.0, np.sqrt(2), "x", True)}


@pytest.fixture(scope="module")
def plugin():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from stylemc_amd import _hip
    _hip.load()
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = text[text.index("## 3. Plugin-level binding"):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    assert 'ctypes.CDLL("stylemc_amd/_lib/libstylemc_hip.so")' in code
    code = code.replace('"stylemc_amd/_lib/libstylemc_hip.so"', repr(_hip.LIB_PATH))
    ns = {}
    exec(compile(code, "INTEGRATION.md#3", "exec"), ns)
    return ns["plugin"]


def close(a, b, tol, what):
    a = a.detach().double().cpu()
    b = torch.from_numpy(np.asarray(b)).double()
    scale = max(b.abs().max().item(), 1e-12)
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"{what}: max err {err:.3e} > {tol:.1e} * {scale:.3e}"


@pytest.mark.parametrize("act", list(ACTS))
@pytest.mark.parametrize("clamp", [None, 0.7])
def test_stub_bias_act_vs_reference_golden(plugin, golden, act, clamp):
    g = golden("ops_bias_act.npz")
    name = f"{act}_c{'none' if clamp is None else clamp}"
    idx, alpha, gain, ref, has2 = ACTS[act]
    cl = -1.0 if clamp is None else float(clamp)
    x = torch.from_numpy(g[f"{name}/x"]).to(DEV)
    b = torch.from_numpy(g[f"{name}/b"]).to(DEV)
    null = torch.empty([0], device=DEV)
    # forward (bias_act.py:153)
    y = plugin.bias_act(x, b, null, null, null, 0, 1, idx, alpha, gain, cl)
    close(y, g[f"{name}/y"], 1e-5, f"{name} y")
    # first-order gradient (bias_act.py:170-182): dx = dy for linear without gain/clamp, else the grad=1 kernel on
    # the saved references.  'linear' saves no y, so the CUDA plugin ignores the clamp there (DESIGN.md section 5
    # item 5); the golden is the reference's _bias_act_ref, which masks it -- compare only the unclamped case.
    if act == "linear" and clamp is not None:
        return
    dy = torch.from_numpy(g[f"{name}/dy"]).to(DEV)
    xs = x if ("x" in ref or has2) else null     # ctx.save_for_backward, bias_act.py:154-157
    bs = b if ("x" in ref or has2) else null
    ys = y if "y" in ref else null
    if act == "linear" and gain == 1.0:
        dx = dy
    else:
        dx = plugin.bias_act(dy, bs, xs, ys, null, 1, 1, idx, alpha, gain, cl)
    close(dx, g[f"{name}/dx"], 1e-5, f"{name} dx")
    close(dx.sum(dim=[0, 2, 3]), g[f"{name}/db"], 1e-5, f"{name} db")


def _ufd(plugin, x, f, up, down, pad, flip, gain):
    """upfirdn2d.py:228-241: one 2-D call, or two 1-D passes for a separable (1-D) filter."""
    upx, upy = up
    downx, downy = down
    padx0, padx1, pady0, pady1 = pad
    if f.ndim == 2:
        return plugin.upfirdn2d(x, f, upx, upy, downx, downy, padx0, padx1, pady0, pady1, flip, gain)
    y = plugin.upfirdn2d(x, f.unsqueeze(0), upx, 1, downx, 1, padx0, padx1, 0, 0, flip, float(np.sqrt(gain)))
    return plugin.upfirdn2d(y, f.unsqueeze(1), 1, upy, 1, downy, 0, 0, pady0, pady1, flip, float(np.sqrt(gain)))


@pytest.mark.parametrize("case", ["blur_conv0", "up2_img", "down2_adj", "blur_adj", "rect_up2_down1", "crop_neg_pad",
                                  "odd_filter", "sep_filter8", "up4_down3", "single_pixel"])
def test_stub_upfirdn2d_vs_reference_golden(plugin, golden, case):
    g = golden("ops_upfirdn2d.npz")
    p = lambda k: g[f"{case}/{k}"]
    x = torch.from_numpy(p("x")).to(DEV)
    f = torch.from_numpy(p("f")).to(DEV)
    up = [int(v) for v in p("up")]
    down = [int(v) for v in p("down")]
    pad = [int(v) for v in p("pad")]
    flip, gain = bool(p("flip")), float(p("gain"))
    y = _ufd(plugin, x, f, up, down, pad, flip, gain)
    close(y, p("y"), 1e-5, f"{case} y")
    # backward (upfirdn2d.py:245-264): the adjoint upfirdn2d with up/down swapped, the filter flipped
    ih, iw = x.shape[2:]
    oh, ow = y.shape[2:]
    fw, fh = (f.shape[-1], f.shape[0]) if f.ndim == 2 else (f.shape[0], f.shape[0])
    padx0, padx1, pady0, pady1 = pad
    pg = [fw - padx0 - 1, iw * up[0] - ow * down[0] + padx0 - up[0] + 1,
          fh - pady0 - 1, ih * up[1] - oh * down[1] + pady0 - up[1] + 1]
    dx = _ufd(plugin, torch.from_numpy(p("dy")).to(DEV), f, down, up, pg, not flip, gain)
    assert tuple(dx.shape) == tuple(x.shape)
    close(dx, p("dx"), 1e-5, f"{case} dx")
