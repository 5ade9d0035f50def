"""Per-layer timing of the modconv GEMM at FFHQ-1024 shapes (fwd 3x3, fwd convT, bwd 3x3, bwd stride-2).

    python tools/bench_gemm.py [--batch 4] [--reps 10]
Prints TFLOP/s per shape (algorithmic FLOPs) and the FLOP-weighted total.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, build, modconv  # noqa: E402


def shapes(n):
    ch = {r: min(32768 // r, 512) for r in [4, 8, 16, 32, 64, 128, 256, 512, 1024]}
    out = []
    for r in [8, 16, 32, 64, 128, 256, 512, 1024]:
        cin, cout = ch[r // 2], ch[r]
        out.append(("fwd_conv0", r, cin, cout, 2, "fwd"))
        out.append(("fwd_conv1", r, cout, cout, 1, "fwd"))
        out.append(("bwd_conv1", r, cout, cout, 1, "bwd"))
        out.append(("bwd_conv0", r, cin, cout, 2, "bwd"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="", help="comma-separated name filters, e.g. fwd_conv0 or fwd_conv0:128")
    ap.add_argument("--fp32", action="store_true", help="exact-fp32 MFMA products (modconv.X3 = False)")
    args = ap.parse_args()
    modconv.X3 = not args.fp32
    only = [f for f in args.only.split(",") if f]
    build.build(verbose=False)
    dev = "cuda"
    n = args.batch
    tot_f = tot_t = 0.0
    for name, r, cin, cout, up, kind in shapes(n):
        if only and not any(f == name or f == f"{name}:{r}" for f in only):
            continue
        W = torch.randn(cout, cin, 3, 3, device=dev)
        P = modconv.PackedConv(W, up)
        h = r // up
        if kind == "fwd":
            x = torch.randn(n, cin, h, h, device=dev)
            s = torch.randn(n, cin, device=dev)
            phases, nph, th, tw = P.fwd_phases(h, h)
            y = torch.empty(n, cout, th, tw, device=dev)
            run = lambda: modconv.gemm(x, y, phases, nph, cin, cout, s=s, epi=modconv._epilogue(_hip.EPI_STORE))
            flops = modconv.conv_flops(n, cin, cout, h * up if up == 1 else h, h * up if up == 1 else h, 9)
        else:
            gin = torch.randn(n, cout, r if up == 1 else 2 * h + 1, r if up == 1 else 2 * h + 1, device=dev)
            phases, nph = P.bwd_phases(h, h)
            y = torch.empty(n, cin, h, h, device=dev)
            run = lambda: modconv.gemm(gin, y, phases, nph, cout, cin, epi=modconv._epilogue(_hip.EPI_STORE))
            flops = modconv.conv_flops(n, cout, cin, h, h, 9)
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(args.reps):
            run()
        s1.record()
        torch.cuda.synchronize()
        t = s0.elapsed_time(s1) / 1e3 / args.reps
        tot_f += flops
        tot_t += t
        print(f"{name:10s} r={r:5d} cin={cin:4d} cout={cout:4d}  {t * 1e6:9.1f} us  {flops / t / 1e12:7.2f} TF/s")
    print(f"TOTAL {tot_t * 1e3:.2f} ms  {tot_f / tot_t / 1e12:.2f} TF/s (FLOP-weighted)")


if __name__ == "__main__":
    main()
