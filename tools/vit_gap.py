"""Wall time per CLIP ViT forward + data backward (the HIP tower, batch B) -- run under rocprofv3 --kernel-trace to set
it against the sum of its kernels' durations (the gaps between launches).  python tools/vit_gap.py [B] [iters]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stylemc_amd import build, vit_hip  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    build.build(verbose=False)
    m = vit_hip.build_visual("ViT-B/32", seed=4)
    x = torch.randn(B, 3, 224, 224, device="cuda")
    cot = torch.randn(B, 512, device="cuda")

    def fwdbwd():
        xx = x.clone().requires_grad_(True)
        torch.autograd.grad(m(xx), xx, cot)

    for _ in range(5):
        fwdbwd()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fwdbwd()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / iters * 1e3
    print(f"ViT-B/32 B={B} fwd+bwd wall {t:.3f} ms per iteration over {iters}", flush=True)


if __name__ == "__main__":
    main()
