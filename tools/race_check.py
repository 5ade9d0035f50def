"""Which component is not bit-reproducible when another stream shares the CUs?  Each test runs one piece REPS times
on the main stream while a disturbing workload runs on a second stream (a different amount of it each rep), and
compares every rep's output with the first bit for bit.  Diagnostic only.   python tools/race_check.py [reps] [piece:disturber,...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from stylemc_amd import _hip, build, synthetic, utils
    from stylemc_amd.find_direction import DirectionFinder, initial_delta
    from tests import dist_gpu_worker as W
    build.build(verbose=False)
    _hip.load()
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = torch.device("cuda", 0)
    G, clip, idl, shapes = W.problem(dev)
    cl = clip[0][0]
    styles = synthetic.synthetic_styles(4, seed=5).to(dev)
    f = DirectionFinder(G, styles, clip, idl, resolution=W.RES, batch_size=4, global_batch=4, n_epochs=4, seed=1,
                        init_delta=initial_delta(0, 0.01), temp_shapes=shapes)
    delta = initial_delta(0, 0.01).to(dev)
    gen = torch.Generator().manual_seed(9)
    x224 = torch.randn(8, 3, 224, 224, generator=gen).to(dev)
    x112 = torch.randn(4, 3, 112, 112, generator=gen).to(dev)
    other = torch.cuda.Stream(dev)

    def synth_fb():
        d = delta.expand(4, -1, -1).clone().requires_grad_(True)
        img = utils.generate_image_rows(G, f.until_k, styles, shapes, "const", delta=d)
        (gd,) = torch.autograd.grad(img, d, torch.ones_like(img))
        return [img.detach(), gd]

    def synth_f():
        with torch.no_grad():
            return [utils.generate_image_rows(G, f.until_k, styles, shapes, "const")]

    def irse_f():
        with torch.no_grad():
            return [idl.facenet(x112)]

    def irse_fb():
        x = x112.clone().requires_grad_(True)
        y = idl.facenet(x)
        (gx,) = torch.autograd.grad(y, x, torch.ones_like(y))
        return [y.detach(), gx]

    def clip_fb():
        x = x224.clone().requires_grad_(True)
        e = cl.visual(x, n_grad=4)
        (gx,) = torch.autograd.grad(e[:4], x, torch.ones_like(e[:4]))
        return [e.detach(), gx]

    pieces = {"synth_fb": synth_fb, "synth_f": synth_f, "irse_f": irse_f, "irse_fb": irse_fb, "clip_fb": clip_fb}
    pairs = [("synth_fb", "irse_f"), ("synth_f", "clip_fb"), ("irse_f", "synth_fb"), ("irse_fb", "synth_f"),
             ("clip_fb", "synth_f")]
    if len(sys.argv) > 2:
        pairs = [tuple(pr.split(":")) for pr in sys.argv[2].split(",")]
    for name, dname in pairs:
        fn = pieces[name]
        disturb = {name: pieces[dname]}
        ref = fn()
        torch.cuda.synchronize()
        bad = []
        for r in range(reps):
            other.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(other):
                for _ in range(r % 3):
                    disturb[name]()
            out = fn()
            torch.cuda.synchronize()
            for i, (a, b) in enumerate(zip(out, ref)):
                if not torch.equal(a, b):
                    bad.append((r, i, (a - b).abs().max().item()))
        print(f"{name} beside {disturb[name].__name__}: {'bit-equal' if not bad else bad}", flush=True)


if __name__ == "__main__":
    main()
