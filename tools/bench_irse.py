"""Time IR-SE50 (forward with saved activations + input backward, and a no-grad forward) on the HIP kernel
library vs PyTorch-ROCm/MIOpen, batch n (default 4).  python tools/bench_irse.py [n]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stylemc_amd import build, irse_hip  # noqa: E402
from stylemc_amd.id_loss import model_irse  # noqa: E402


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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    build.build(verbose=False)
    torch.backends.cudnn.allow_tf32 = False
    x = torch.randn(n, 3, 112, 112, device="cuda")
    cot = torch.randn(n, 512, device="cuda")
    gflop = 12.59 * n
    for label, m in [("hip", irse_hip.build_irse50(seed=3)), ("torch", model_irse.build_irse50(seed=3))]:
        def fwd():
            with torch.no_grad():
                m(x)

        def fwdbwd():
            xx = x.clone().requires_grad_(True)
            torch.autograd.grad(m(xx), xx, cot)

        tf = timeit(fwd)
        tb = timeit(fwdbwd)
        print(f"IR-SE50 n={n} {label}: no-grad fwd {tf:.3f} ms ({gflop / tf:.1f} TF/s), fwd+bwd {tb:.3f} ms "
              f"({3 * gflop / tb:.1f} TF/s alg)", flush=True)


if __name__ == "__main__":
    main()
