"""HBM-bound synthesis kernels in isolation at the FFHQ-1024 shapes (batch 4): achieved GB/s of
algorithmic bytes for blur_act fwd/bwd, act_bwd, torgb fwd/bwd, channel_dot.

    python tools/bench_membound.py [--res 1024 512 256]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, modconv  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--res", type=int, nargs="+", default=[1024, 512, 256])
    p.add_argument("--n", type=int, default=4)
    a = p.parse_args()
    _hip.load()
    dev = "cuda"
    n = a.n
    f = torch.tensor([1., 3., 3., 1.], device=dev)
    f = (f[:, None] * f[None, :])
    f = (f / f.sum()).contiguous()
    for r in a.res:
        c = min(32768 // r, 512)
        h = r // 2
        th = 2 * h + 1
        t = torch.randn(n, c, th, th, device=dev)
        y = torch.empty(n, c, r, r, device=dev)
        u = torch.empty_like(y)
        d = torch.rand(n, c, device=dev) + 0.5
        noise = torch.randn(r, r, device=dev)
        strength = torch.tensor(0.1, device=dev)
        bias = torch.randn(c, device=dev) * 0.1
        epi = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 256.0, u)
        st = _hip.stream()

        def blur():
            _hip.call("smc_modconv_blur_act_f32", t.data_ptr(), 1, 0, y.data_ptr(), n, c, th, th, 0, r, r, f.data_ptr(),
                      4, 4, 1, 1, 4.0, 0, ctypes.byref(epi), st)
        us = timeit(blur)
        byt = 4 * (t.numel() + 2 * y.numel())
        print(f"r={r:5d} c={c:4d} blur_act_fwd  {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s  ({byt / 1e6:.0f} MB)")
        g = torch.randn_like(y)
        dt = torch.empty_like(t)
        dd = torch.zeros(n, c, device=dev)
        epib = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 256.0)
        lib = _hip.load()
        wsb = max(lib.smc_modconv_blur_act_bwd_workspace_size(n, c, r, r, th, th),
                  lib.smc_modconv_act_bwd_workspace_size(n, c, r, r))
        ws = torch.empty(max(wsb // 4, 1), device=dev)

        def blur_b():
            _hip.call("smc_modconv_blur_act_bwd_f32", g.data_ptr(), u.data_ptr(), dt.data_ptr(), dd.data_ptr(), n, c,
                      r, r, th, th, 0, f.data_ptr(), 4, 4, 2, 2, 4.0, 1, ctypes.byref(epib), ws.data_ptr(), wsb, st)
        us = timeit(blur_b)
        byt = 4 * (2 * y.numel() + t.numel())
        print(f"r={r:5d} c={c:4d} blur_act_bwd  {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s")
        tp = (th + 3) // 4 * 4
        dtp = torch.empty(n, c, th, tp, device=dev)

        def blur_bp():
            _hip.call("smc_modconv_blur_act_bwd_f32", g.data_ptr(), u.data_ptr(), dtp.data_ptr(), dd.data_ptr(), n, c,
                      r, r, th, th, tp, f.data_ptr(), 4, 4, 2, 2, 4.0, 1, ctypes.byref(epib), ws.data_ptr(), wsb, st)
        us = timeit(blur_bp)
        print(f"r={r:5d} c={c:4d} blur_act_bwd_pitch{tp} {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s")
        epiy = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 256.0)
        epiy.grad_from_y = 1

        def blur_by():
            _hip.call("smc_modconv_blur_act_bwd_f32", g.data_ptr(), y.data_ptr(), dtp.data_ptr(), None, n, c,
                      r, r, th, th, tp, f.data_ptr(), 4, 4, 2, 2, 4.0, 1, ctypes.byref(epiy), None, 0, st)
        us = timeit(blur_by)
        print(f"r={r:5d} c={c:4d} blur_act_bwd_from_y {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s")
        du = torch.empty_like(y)

        def actb():
            _hip.call("smc_modconv_act_bwd_f32", g.data_ptr(), u.data_ptr(), du.data_ptr(), dd.data_ptr(), n, c, r, r,
                      ctypes.byref(epib), ws.data_ptr(), wsb, st)
        us = timeit(actb)
        byt = 4 * 3 * y.numel()
        print(f"r={r:5d} c={c:4d} act_bwd       {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s")
        w2 = torch.randn(3, c, device=dev)
        s = torch.randn(n, c, device=dev)
        b3 = torch.randn(3, device=dev)
        rgb = torch.empty(n, 3, r, r, device=dev)

        def trgb():
            _hip.call("smc_torgb_fwd_f32", y.data_ptr(), w2.data_ptr(), s.data_ptr(), b3.data_ptr(), rgb.data_ptr(), n,
                      c, 3, r, r, 256.0, st)
        us = timeit(trgb)
        byt = 4 * (y.numel() + rgb.numel())
        print(f"r={r:5d} c={c:4d} torgb_fwd     {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s")
        grgb = torch.randn_like(rgb)

        def trgb_b():
            _hip.call("smc_torgb_bwd_f32", grgb.data_ptr(), rgb.data_ptr(), w2.data_ptr(), s.data_ptr(), du.data_ptr(),
                      n, c, 3, r, r, 256.0, 1, 0, st)
        us = timeit(trgb_b)
        byt = 4 * (y.numel() + 2 * rgb.numel())
        print(f"r={r:5d} c={c:4d} torgb_bwd     {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s")
        out = torch.empty(n * c, device=dev)

        def cdot():
            _hip.call("smc_channel_dot_f32", du.data_ptr(), y.data_ptr(), None, out.data_ptr(), None, n * c, r * r, 0, st)
        us = timeit(cdot)
        byt = 4 * 2 * y.numel()
        print(f"r={r:5d} c={c:4d} channel_dot   {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s")
        img = torch.randn(n, 3, h, h, device=dev)
        img2 = torch.empty(n, 3, r, r, device=dev)
        print(f"r={r:5d} copy ref      {timeit(lambda: y.copy_(u)):8.1f} us  "
              f"{8 * y.numel() / timeit(lambda: y.copy_(u)) / 1e3:7.0f} GB/s (torch copy_)")
        del t, y, u, g, dt, du
        torch.cuda.empty_cache()




def ufd_main():
    """upsample2d / downsample2d of the 3-channel skip image (the skip-architecture img path)."""
    from stylemc_amd.torch_utils.ops import upfirdn2d
    f = upfirdn2d.setup_filter([1, 3, 3, 1], device="cuda")
    for r in (1024, 512, 256):
        img = torch.randn(4, 3, r // 2, r // 2, device="cuda")
        us = timeit(lambda: upfirdn2d.upsample2d(img, f))
        byt = 4 * (img.numel() + 4 * img.numel())
        print(f"r={r:5d} upsample2d    {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s")
        big = torch.randn(4, 3, r, r, device="cuda")
        us = timeit(lambda: upfirdn2d.downsample2d(big, f))
        byt = 4 * (big.numel() + big.numel() // 4)
        print(f"r={r:5d} downsample2d  {us:8.1f} us  {byt / us / 1e3:7.0f} GB/s")


if __name__ == "__main__":
    if "--ufd" in sys.argv:
        ufd_main()
    else:
        main()
