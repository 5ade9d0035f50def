"""conv0's FIR + modconv epilogue forward (smc_modconv_blur_act_f32) at the FFHQ-1024 batch-4 shapes in the step's
form (MODACT, const [r, r] noise, no u store: the r >= 128 layers' styles need no gradient), plus a y checksum so
library variants (tools/ab_libs.sh) can be compared bit for bit.

    python tools/bench_blur.py
"""
import ctypes
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, modconv  # noqa: E402


# f = NULL: the built-in [1,3,3,1] taps, as modconv passes for the synthesis' resample filter (--file-taps: f given)
BUILTIN = "--file-taps" not in sys.argv


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    _hip.load()
    dev = "cuda"
    n = 4
    f1 = torch.tensor([1., 3., 3., 1.], device=dev)
    f = (f1[:, None] * f1[None, :] / 64.0).contiguous()
    g = torch.Generator(device=dev).manual_seed(0)
    total = 0.0
    for r, c in ((1024, 32), (512, 64), (256, 128), (128, 256), (64, 512)):
        h = r // 2
        th = 2 * h + 1
        t = torch.randn(n, c, th, th, device=dev, generator=g)
        y = torch.empty(n, c, r, r, device=dev)
        d = torch.rand(n, c, device=dev, generator=g) + 0.5
        noise = torch.randn(r, r, device=dev, generator=g)
        strength = torch.tensor(0.1, device=dev)
        bias = torch.randn(c, device=dev, generator=g) * 0.1
        epi = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 256.0)
        st = _hip.stream()

        def blur():
            _hip.call("smc_modconv_blur_act_f32", t.data_ptr(), 1, 0, y.data_ptr(), n, c, th, th, 0, r, r,
                      None if BUILTIN else f.data_ptr(), 4, 4, 1, 1, 4.0, 0, ctypes.byref(epi), st)
        us = timeit(blur)
        total += us
        byt = 4 * (t.numel() + y.numel())
        digest = hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest()[:12]
        print(f"r={r:5d} c={c:4d} blur_act_fwd {us:8.1f} us {byt / us / 1e3:7.0f} GB/s ({byt / 1e6:.0f} MB) y {digest}",
              flush=True)
        del t, y
        torch.cuda.empty_cache()
    print(f"total {total:.1f} us")


if __name__ == "__main__":
    main()
