"""TFLOP/s of smc_linear_f32 on the CLIP ViT-B/32 GEMM shapes (M = 50 x batch tokens) vs torch.mm (hipBLASLt).

    python tools/bench_linear.py [batch ...]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stylemc_amd import _hip, build  # noqa: E402


def shapes(B):
    M, D = 50 * B, 768
    return [("qkv", M, 3 * D, D), ("out", M, D, D), ("fc", M, 4 * D, D), ("proj", M, D, 4 * D),
            ("fc^T", M, D, 4 * D), ("proj^T", M, 4 * D, D), ("qkv^T", M, D, 3 * D), ("patch", 49 * B, D, 3072)]


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    build.build(verbose=False)
    torch.backends.cuda.matmul.allow_tf32 = False
    lib = _hip.load()
    batches = [int(a) for a in sys.argv[1:]] or [4, 8]
    for B in batches:
        tot_h = tot_t = tot_f = 0.0
        for name, M, N, K in shapes(B):
            a = torch.randn(M, K, device="cuda")
            w = torch.randn(K, N, device="cuda")
            c = torch.empty(M, N, device="cuda")
            wsb = lib.smc_linear_workspace_size(M, N, K)
            ws = torch.empty(max(wsb // 4, 1), device="cuda")
            e = _hip.LinearEpilogue()

            def hip():
                _hip.call("smc_linear_f32", a.data_ptr(), K, w.data_ptr(), N, c.data_ptr(), N, M, N, K,
                          ctypes.byref(e), ws.data_ptr(), wsb, _hip.stream())

            th = timeit(hip)
            tt = timeit(lambda: torch.mm(a, w, out=c))
            f = 2.0 * M * N * K
            tot_h += th
            tot_t += tt
            tot_f += f
            print(f"B={B} {name:7s} M={M:4d} N={N:4d} K={K:4d}  hip {th * 1e6:7.1f} us {f / th / 1e12:6.1f} TF/s   "
                  f"torch {tt * 1e6:7.1f} us {f / tt / 1e12:6.1f} TF/s", flush=True)
        print(f"B={B} TOTAL hip {tot_h * 1e6:.1f} us ({tot_f / tot_h / 1e12:.1f} TF/s)  torch {tot_t * 1e6:.1f} us "
              f"({tot_f / tot_t / 1e12:.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
