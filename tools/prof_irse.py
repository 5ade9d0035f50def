"""IR-SE50 in the find_direction pair pattern (forward of [edited; original] = 2n faces, input gradient of
the leading n) repeated `iters` times -- run under rocprofv3 --kernel-trace, then summarise with
tools/trace_grid.py.   python tools/prof_irse.py [n] [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stylemc_amd import irse_hip  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    m = irse_hip.build_irse50(seed=3)
    x = torch.randn(2 * n, 3, 112, 112, device="cuda")
    cot = torch.randn(2 * n, 512, device="cuda")
    for _ in range(iters + 2):
        xx = x.clone().requires_grad_(True)
        torch.autograd.grad(m(xx, n_grad=n), xx, cot)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        xx = x.clone().requires_grad_(True)
        torch.autograd.grad(m(xx, n_grad=n), xx, cot)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"IR-SE50 pair fwd({2 * n}) + bwd({n}): {ev[0].elapsed_time(ev[1]) / iters:.3f} ms/iter")


if __name__ == "__main__":
    main()
