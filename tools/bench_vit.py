"""Time the CLIP ViT tower (forward with saved activations + data backward, and a no-grad forward) on the
HIP kernel library vs the PyTorch-ROCm tower, batch B (default 4).  python tools/bench_vit.py [B] [name]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stylemc_amd import build, clip_model, vit_hip  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    name = sys.argv[2] if len(sys.argv) > 2 else "ViT-B/32"
    build.build(verbose=False)
    torch.backends.cuda.matmul.allow_tf32 = False
    x = torch.randn(B, 3, 224, 224, device="cuda")
    cot = torch.randn(B, 512, device="cuda")
    for label, m in [("hip", vit_hip.build_visual(name, seed=4)), ("torch", clip_model.build_visual(name, seed=4))]:
        gflop = m.flops_per_image() * B / 1e9

        def fwd():
            with torch.no_grad():
                m(x)

        def fwdbwd():
            xx = x.clone().requires_grad_(True)
            torch.autograd.grad(m(xx), xx, cot)

        tf = timeit(fwd)
        tb = timeit(fwdbwd)
        print(f"{name} B={B} {label}: no-grad fwd {tf:.3f} ms ({gflop / tf:.1f} TF/s), fwd+bwd {tb:.3f} ms "
              f"({3 * gflop / tb:.1f} TF/s alg)", flush=True)


if __name__ == "__main__":
    main()
