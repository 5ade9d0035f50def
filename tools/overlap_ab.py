"""Where the find_direction step's time goes across its three HIP streams (FFHQ-1024, batch 4, HIP losses).

    python tools/overlap_ab.py [--steps 10]

1. ms/step for the three stream schedules: all on one stream (overlap=False), original-image branch on a second
   stream without the next-iteration prefetch, and the default (second stream + prefetch on a third).
2. The serialised pieces, each timed alone on an idle GPU: edited synthesis forward (with the saved tensors), the
   original synthesis (no grad), CLIP ViT-B/32 and IR-SE50 forward on the [edited; original] pair of 8 images, their
   backward for the edited half, the synthesis backward.  Their sum against the schedules shows how much the
   streams overlap and which chain bounds the step.
"""
import os
import sys
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


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
    ts = utils.get_temp_shapes(G)   # before the first finder (its synthesis drops the affine layers)

    def finder(**kw):
        return FD.DirectionFinder(G, styles, clip, idl, resolution=1024, batch_size=4, seed=0, temp_shapes=ts,
                                  init_delta=FD.initial_delta(0, 0.01), n_epochs=1000, **kw)

    for name, kw in (("one stream", dict(overlap=False)), ("2 streams, no prefetch", dict(prefetch_orig=False)),
                     ("3 streams (default)", {})):
        f = finder(**kw)
        ms = timed(f.step, reps=steps)
        print(f"schedule {name:24s} {ms:7.2f} ms/step")

    # serialised pieces on one stream
    f = finder(overlap=False)
    tshape = f.temp_shapes
    s4 = styles[:4]
    d = f.delta.detach().clone().requires_grad_(True)
    T = FD.S_TRAINABLE_SPACE_CHANNELS
    pieces = {}
    pieces["synth edited fwd (saved)"] = timed(lambda: utils.generate_image_rows(G, f.until_k, s4, tshape, f.noise_mode,
                                                                                  delta=d))
    with torch.no_grad():
        pieces["synth original fwd (no grad)"] = timed(lambda: utils.generate_image_rows(G, f.until_k, s4, tshape,
                                                                                          f.noise_mode))
        orig = utils.generate_image_rows(G, f.until_k, s4, tshape, f.noise_mode)
    img = utils.generate_image_rows(G, f.until_k, s4, tshape, f.noise_mode, delta=d)
    imgd = img.detach().requires_grad_(True)
    cl = clip[0][0]

    def clip_fwd():
        tgt = FD.unprocess(imgd, f.mean, f.std)
        with torch.no_grad():
            src = FD.unprocess(orig, f.mean, f.std)
        return cl.per_sample_pair(tgt, src)

    def id_fwd():
        return idl.per_sample_pair(imgd, orig)

    pieces["CLIP fwd [8 images]"] = timed(lambda: clip_fwd())
    pieces["CLIP fwd + bwd (edited half)"] = timed(lambda: torch.autograd.grad(clip_fwd().sum(), imgd))
    pieces["IR-SE50 fwd [8 images]"] = timed(lambda: id_fwd())
    pieces["IR-SE50 fwd + bwd (edited half)"] = timed(lambda: torch.autograd.grad(id_fwd().sum(), imgd))
    gimg = torch.randn_like(img)

    def synth_bwd():
        im = utils.generate_image_rows(G, f.until_k, s4, tshape, f.noise_mode, delta=d)
        return torch.autograd.grad(im, d, gimg)

    pieces["synth fwd + bwd"] = timed(synth_bwd)
    for k, v in pieces.items():
        print(f"piece {k:34s} {v:7.2f} ms")
    fwd = pieces["synth edited fwd (saved)"]
    print(f"derived: synth bwd {pieces['synth fwd + bwd'] - fwd:.2f} ms; serial sum (edited fwd+bwd + original fwd + "
          f"CLIP f+b + ID f+b) {pieces['synth fwd + bwd'] + pieces['synth original fwd (no grad)'] + pieces['CLIP fwd + bwd (edited half)'] + pieces['IR-SE50 fwd + bwd (edited half)']:.2f} ms")


if __name__ == "__main__":
    main()
