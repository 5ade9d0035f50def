"""Winograd F(2x2, 3x3) and F(4x4, 3x3) vs the direct implicit GEMM on the synthesis conv1 shapes (FFHQ-1024, batch 4).

    python tools/bench_wino.py [--batch 4] [--reps 10]
Per shape: us per launch of each path, the direct-equivalent TFLOP/s (dense 3x3 MACs x 2 / time) and the Winograd
kernel's MFMA fraction (its own 16-multiply FLOPs / time vs 157.3 TF/s).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, build, modconv  # noqa: E402

PEAK = 157.3e12


def timeit(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e-3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-split", action="store_true", help="F(2x2) without split K (modconv.WINO_SPLIT off)")
    ap.add_argument("--res", type=int, nargs="+", default=[32, 64, 128, 256, 512, 1024])
    ap.add_argument("--x3", type=int, default=0, help="smc_set_wino_x3 mode (the split-bf16 F(2x2) for 32 channels)")
    ap.add_argument("--modact", action="store_true",
                    help="the synthesis epilogues (conv1 forward: demod, noise, bias, lrelu, gain, clamp, u store; "
                         "data gradient: x s) instead of plain stores")
    args = ap.parse_args()
    build.build(verbose=False)
    modconv.WINO_SPLIT = not args.no_split
    _hip.load().smc_set_wino_x3(args.x3)
    n, dev = args.batch, "cuda"
    tot = {"direct": 0.0, "wino": 0.0, "wino4": 0.0}
    for r in args.res:
        c = min(32768 // r, 512)
        W = torch.randn(c, c, 3, 3, device=dev) / (3 * c ** 0.5)
        P = modconv.PackedConv(W, 1)
        x = torch.randn(n, c, r, r, device=dev)
        s = torch.rand(n, c, device=dev) + 0.5
        y = torch.empty_like(x)
        phases, nph, _, _ = P.fwd_phases(r, r)
        bph, bnph = P.bwd_phases(r, r)
        uf, ub = P.wino_weights(0), P.wino_weights(1)
        has4 = modconv.wino4_ok(n, c, c, r, r)
        if has4:
            uf4, ub4 = P.wino4_weights(0), P.wino4_weights(1)
        st = stb = modconv._epilogue(_hip.EPI_STORE)
        if args.modact:
            d = torch.rand(n, c, device=dev) + 0.5
            noise = torch.randn(n, 1, r, r, device=dev)
            strength, bias, u = torch.tensor([0.3], device=dev), torch.randn(c, device=dev), torch.empty_like(x)
            st = modconv._epilogue(_hip.EPI_MODACT, d, noise, r * r, strength, bias, "lrelu", 0.2, 2 ** 0.5, 256.0, u)
            stb = modconv._epilogue(_hip.EPI_MODACT, s, None, 0, None, None, "linear", 0.0, 1.0, -1.0, None)
        runs = {
            ("fwd", "direct"): lambda: modconv.gemm(x, y, phases, nph, c, c, s=s, epi=st),
            ("fwd", "wino"): lambda: modconv.wino(x, y, uf, c, c, s=s, epi=st),
            ("bwd", "direct"): lambda: modconv.gemm(x, y, bph, bnph, c, c, epi=stb),
            ("bwd", "wino"): lambda: modconv.wino(x, y, ub, c, c, epi=stb),
        }
        if has4:
            runs[("fwd", "wino4")] = lambda: modconv.wino4(x, y, uf4, c, c, s=s, epi=st)
            runs[("bwd", "wino4")] = lambda: modconv.wino4(x, y, ub4, c, c, epi=stb)
        flops = modconv.conv_flops(n, c, c, r, r, 9)
        wfl = modconv.wino_flops(n, c, c, r, r)
        wfl4 = modconv.wino4_flops(n, c, c, r, r)
        for kind in ("fwd", "bwd"):
            td = timeit(runs[(kind, "direct")], args.reps)
            tw = timeit(runs[(kind, "wino")], args.reps)
            tot["direct"] += td
            tot["wino"] += tw
            print(f"r={r:5d} c={c:4d} {kind}: direct {td * 1e6:8.1f} us ({flops / td / 1e12:6.1f} TF/s, "
                  f"{flops / td / PEAK:.3f})  wino {tw * 1e6:8.1f} us (eq {flops / tw / 1e12:6.1f} TF/s, "
                  f"MFMA frac {wfl / tw / PEAK:.3f})  speedup {td / tw:.2f}x", flush=True)
            if has4:
                t4 = timeit(runs[(kind, "wino4")], args.reps)
                tot["wino4"] += t4
                print(f"            {kind}: wino4 {t4 * 1e6:8.1f} us (eq {flops / t4 / 1e12:6.1f} TF/s, "
                      f"MFMA frac {wfl4 / t4 / PEAK:.3f})  vs wino {tw / t4:.2f}x", flush=True)
            else:
                tot["wino4"] += tw
    print(f"total: direct {tot['direct'] * 1e3:.3f} ms, wino {tot['wino'] * 1e3:.3f} ms, "
          f"speedup {tot['direct'] / tot['wino']:.2f}x; best-of wino4/wino {tot['wino4'] * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
