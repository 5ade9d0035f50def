"""K sweep of smc_linear_f32 at the ViT token counts (M = 200 / 400), N = 768 / 3072: time = fixed + per-K part?
Cold weights: every call reads a different copy of B (a ring of copies larger than the MALL), as the tower does.
Diagnostic only.   python tools/lin_sweep.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stylemc_amd import _hip, build  # noqa: E402


def main():
    build.build(verbose=False)
    lib = _hip.load()
    reps = 40
    for M in (200, 400):
        for N in (768, 3072):
            for K in (64, 256, 768, 3072):
                a = torch.randn(M, K, device="cuda")
                nb = max(2, int(600e6 // (K * N * 4)))  # > 256 MB of B copies
                nb = min(nb, reps)
                ws_ = [torch.randn(K, N, device="cuda") for _ in range(nb)]
                c = torch.empty(M, N, device="cuda")
                wsb = lib.smc_linear_workspace_size(M, N, K)
                ws = torch.empty(max(wsb // 4, 1), device="cuda")
                e = _hip.LinearEpilogue()

                def call(w):
                    _hip.call("smc_linear_f32", a.data_ptr(), K, w.data_ptr(), N, c.data_ptr(), N, M, N, K,
                              ctypes.byref(e), ws.data_ptr(), wsb, _hip.stream())
                for w in ws_[:3]:
                    call(w)
                torch.cuda.synchronize()
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
                for i in range(reps):
                    call(ws_[i % nb])
                t1.record()
                torch.cuda.synchronize()
                us = t0.elapsed_time(t1) / reps * 1e3
                f = 2.0 * M * N * K
                print(f"M={M:4d} N={N:4d} K={K:4d} {us:7.1f} us {f / us / 1e6:6.1f} TF/s", flush=True)
                del ws_


if __name__ == "__main__":
    main()
