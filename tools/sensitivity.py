"""Which chain bounds the find_direction step (FFHQ-1024, batch 4, HIP losses)?  Diagnostic only.

    python tools/sensitivity.py --variants default,no_clip,no_irse,no_losses,no_prefetch,irse_pair [--rounds 2]

Times the default three-stream step, then the same step with one piece replaced by a stand-in that costs ~nothing
(its loss term becomes sum(input) * 0, so autograd still reaches the synthesis): without CLIP, without IR-SE50,
without both, and without the next iteration's original-image prefetch.  The drop in ms/step when a piece is
removed is what speeding that piece up can gain at most.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Free(torch.nn.Module):
    """A loss with the per-sample interface that does no work."""

    def __init__(self, raw=False):
        super().__init__()
        self.takes_raw_images = raw

    def per_sample_pair(self, tgt, src):
        return tgt.flatten(1)[:, :1].sum(1) * 0.0

    def target_feats(self, y):
        return y

    def per_sample_with(self, e, tgt):
        return tgt.flatten(1)[:, :1].sum(1) * 0.0

    def encode_src(self, src):
        return src


def timed(f, steps):
    for _ in range(3):
        f.step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        f.step()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


def main():
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 10
    from stylemc_amd import _hip, synthetic, utils
    from stylemc_amd import find_direction as FD
    from stylemc_amd.id_loss import IDLoss
    _hip.load()
    dev = torch.device("cuda", 0)
    G = FD.load_generator("synthetic", 1024, dev)
    styles = synthetic.synthetic_styles(129, seed=0).to(dev)
    clip = FD.build_clip_losses("small", dev, "a", "b", synthetic_weights=True)
    idl = IDLoss("a", device=dev, weights=None)
    ts = utils.get_temp_shapes(G)
    free = _Free()

    def finder(clips, idloss, **kw):
        return FD.DirectionFinder(G, styles, clips, idloss, resolution=1024, batch_size=4, seed=0, temp_shapes=ts,
                                  init_delta=FD.initial_delta(0, 0.01), n_epochs=1000, **kw)

    variants = {"default": (clip, idl, {}), "no_clip": ([(free, 1.0)], idl, {}), "no_irse": (clip, free, {}),
                "no_losses": ([(free, 1.0)], free, {}), "no_prefetch": (clip, idl, dict(prefetch_orig=False)),
                "irse_pair": (clip, idl, dict(prefetch_id=False)),
                "side_hi": (clip, idl, {}), "unfused": (clip, idl, {}),
                "main_side_hi": (clip, idl, {})}
    name = sys.argv[sys.argv.index("--variant") + 1]
    clips, idloss, kw = variants[name]
    if name == "unfused":  # the loss head and composition through autograd's op-by-op graph
        from stylemc_amd import clip_loss
        clip_loss.FUSED_HEAD = False
        FD.FUSED_TOTAL = False
    f = finder(clips, idloss, **kw)
    # stream priority variants: the IR-SE50 (side) stream -- or it and the main stream (edited synthesis, CLIP,
    # backward) -- at high priority; the prefetch stream (next iteration's original image) stays normal
    if name in ("side_hi", "main_side_hi"):
        f._side = torch.cuda.Stream(device=dev, priority=-1)
    main = torch.cuda.Stream(device=dev, priority=-1) if name == "main_side_hi" else torch.cuda.current_stream()
    with torch.cuda.stream(main):
        ms = timed(f, steps)
    print(f"{name:12s} {ms:7.2f} ms/step", flush=True)


def driver():
    """Each variant in a fresh process, interleaved over rounds: a process's HIP streams map onto the hardware
    queues in creation order, so variants timed one after another in one process do not compare."""
    import subprocess
    steps = sys.argv[sys.argv.index("--steps") + 1] if "--steps" in sys.argv else "10"
    names = sys.argv[sys.argv.index("--variants") + 1].split(",")
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 2
    for r in range(rounds):
        for n in names:
            out = subprocess.run([sys.executable, "-u", __file__, "--variant", n, "--steps", steps],
                                 capture_output=True, text=True, timeout=300)
            line = [l for l in out.stdout.splitlines() if "ms/step" in l]
            print(f"round {r} {line[-1] if line else 'FAILED ' + out.stderr[-300:]}", flush=True)
            if out.returncode != 0:
                sys.exit(out.returncode)


if __name__ == "__main__":
    if "--variants" in sys.argv:
        driver()
    else:
        main()
