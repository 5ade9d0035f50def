"""Loss-network phases of a find_direction step in isolation: IR-SE50 forward(4) + input backward(4) (the edited
images; the original image's features are prefetched) and the CLIP ViT-B/32 forward(8) + backward(4) ([edited;
original] with the edited half differentiated).  Diagnostic only.

    python tools/loss_trace.py run [iters]          wall ms per phase iteration (HIP events, unprofiled)
    python tools/loss_trace.py analyze trace.csv    per phase: launches, sum of kernel durations, wall span, idle
Phases are separated by a 50 ms host sleep, so the analysis splits the kernel trace at gaps > 20 ms.
"""
import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(iters):
    import torch
    from stylemc_amd import build, irse_hip, vit_hip
    build.build(verbose=False)
    dev = "cuda"
    irse = irse_hip.build_irse50(seed=3)
    vit = vit_hip.build_visual("ViT-B/32", seed=4)
    face = torch.randn(4, 3, 112, 112, device=dev)
    img = torch.randn(8, 3, 224, 224, device=dev)
    cot_i, cot_c = torch.randn(4, 512, device=dev), torch.randn(8, 512, device=dev)

    def irse_fb():
        xx = face.clone().requires_grad_(True)
        torch.autograd.grad(irse(xx), xx, cot_i)

    def clip_fb():
        xx = img.clone().requires_grad_(True)
        f = vit(xx, n_grad=4) if "n_grad" in vit.forward.__code__.co_varnames else vit(xx)
        torch.autograd.grad(f, xx, cot_c)

    for name, fn in [("irse_f4b4", irse_fb), ("clip_f8b4", clip_fb)]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        time.sleep(0.05)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(f"{name}: {s.elapsed_time(e) / iters:.3f} ms/iter (wall, {iters} iters)", flush=True)
        time.sleep(0.05)


def analyze(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    groups, cur = [], [iv[0]]
    for a, b in zip(iv, iv[1:]):
        if b[0] - a[1] > 20e6:
            groups.append(cur)
            cur = []
        cur.append(b)
    groups.append(cur)
    for gi, g in enumerate(groups):
        busy = sum(b - a for a, b, _ in g)
        span = g[-1][1] - g[0][0]
        # union of intervals (several streams may overlap)
        u, end = 0, 0
        for a, b, _ in g:
            if b > end:
                u += b - max(a, end)
                end = b
        print(f"group {gi}: {len(g)} launches, kernel sum {busy / 1e6:.3f} ms, union {u / 1e6:.3f} ms, "
              f"span {span / 1e6:.3f} ms, idle {(span - u) / 1e6:.3f} ms ({(span - u) / max(len(g) - 1, 1) / 1e3:.2f} "
              f"us per gap)")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 20)
    else:
        analyze(sys.argv[2])
