"""GPU-timeline phase split of the find_direction step (HIP events on the main stream, no profiler):
synthesis forwards (edited on main + original on the side stream), loss-network forwards, backward, and the
rest (all-reduce + SGD).   python tools/phase_times.py [--steps 10]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 10
    from stylemc_amd import _hip, synthetic, utils
    from stylemc_amd import find_direction as FD
    from stylemc_amd.id_loss import IDLoss
    _hip.load()
    dev = torch.device("cuda", 0)
    ev = {}

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        ev.setdefault(name, []).append(e)

    orig_synth = utils.generate_image_rows
    calls = {"n": 0}

    def synth(*a, **k):
        out = orig_synth(*a, **k)
        if k.get("delta") is not None:   # the edited synthesis (main stream) just enqueued
            mark("synth_main_done")
        return out

    class F(FD.DirectionFinder):
        def _pair_terms(self, *a, **k):
            mark("start")
            r = super()._pair_terms(*a, **k)
            mark("losses_fwd_done")
            return r

        def _finish(self, *a):
            r = super()._finish(*a)
            mark("backward_done")
            return r

    G = FD.load_generator("synthetic", 1024, dev)
    styles = synthetic.synthetic_styles(129, seed=0).to(dev)
    f = F(G, styles, FD.build_clip_losses("small", dev, "a", "b", synthetic_weights=True), IDLoss("a", device=dev, weights=None),
          resolution=1024, batch_size=4, seed=0, init_delta=FD.initial_delta(0, 0.01), n_epochs=1000, synth_fn=synth)
    for _ in range(3):
        f.step()
    torch.cuda.synchronize()
    ev.clear()
    for _ in range(steps):
        f.step()
        mark("step_done")
    torch.cuda.synchronize()
    names = ["start", "synth_main_done", "losses_fwd_done", "backward_done", "step_done"]
    tot = {n: 0.0 for n in names[1:]}
    for i in range(steps):
        for a, b in zip(names, names[1:]):
            tot[b] += ev[a][i].elapsed_time(ev[b][i])
    step = sum(ev["step_done"][i - 1].elapsed_time(ev["step_done"][i]) for i in range(1, steps)) / (steps - 1)
    print(f"step {step:.2f} ms (GPU timeline); phases, ms/step (main-stream events):")
    for a, b in zip(names, names[1:]):
        print(f"  {a:>16s} -> {b:<16s} {tot[b] / steps:7.2f}")


if __name__ == "__main__":
    main()
