"""Stress the CLIP ViT backward beside a concurrent synthesis (round 6 nondeterminism hunt).

tools/det_stage.py located the run-to-run difference of the pipelined find_direction step in the ViT backward: the
gradient at the tower's input differs while the gradient at its output does not.  Here the ViT forward + partial
backward of a fixed [8, 3, 224, 224] batch (n_grad 4, as in the step) runs `reps` times on the main stream while a
FFHQ synthesis forward runs on a second stream (the prefetch's overlap), and every input gradient is compared with
the first one computed alone.  SMC_HIP_LIB selects an A/B build of the library.
    python tools/vit_race.py reps [res] [mode]
mode: overlap (default) | alone
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    res = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    mode = sys.argv[3] if len(sys.argv) > 3 else "overlap"
    from stylemc_amd import _hip, networks, synthetic, utils, vit_hip
    _hip.load()
    dev = torch.device("cuda", 0)
    cfg = synthetic.generator_config(resolution=res)
    G = networks.build_generator(cfg, synthetic.generator_state_dict(cfg, seed=0), device=dev)
    shapes = utils.get_temp_shapes(G)
    until_k = res.bit_length() - 3
    styles = synthetic.synthetic_styles(4, seed=5).to(dev)
    vis = vit_hip.build_visual("ViT-B/32", None, seed=4, device=dev)
    g = torch.Generator(device="cpu").manual_seed(1)
    x0 = torch.randn(8, 3, 224, 224, generator=g).to(dev)
    w = torch.randn(4, 512, generator=g).to(dev)

    def fb():
        x = x0.clone().requires_grad_(True)
        e = vis(x, n_grad=4)
        (gx,) = torch.autograd.grad((e[:4] * w).sum(), x)
        return gx

    ref = fb()
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    outs = []
    for _ in range(reps):
        if mode == "overlap":
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side), torch.no_grad():
                img = utils.generate_image_rows(G, until_k, styles, shapes, "const")
            img.record_stream(torch.cuda.current_stream())
        outs.append(fb())
        if mode == "overlap":
            torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    bad = [(i, (o - ref).abs().max().item()) for i, o in enumerate(outs) if not torch.equal(o, ref)]
    print(f"lib {os.environ.get('SMC_HIP_LIB', 'default')} mode {mode} res {res}: {len(bad)} of {reps} differ"
          + (f"; first {bad[:5]}, rel {max(b for _, b in bad) / ref.abs().max().item():.1e}" if bad else ""),
          flush=True)


if __name__ == "__main__":
    main()
