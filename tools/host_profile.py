"""cProfile of the host side of DirectionFinder.step() (GPU box): where the ~26 ms of Python/launch time goes.

    python tools/host_profile.py [--steps 5]
"""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 5
    from stylemc_amd import _hip, synthetic
    from stylemc_amd.find_direction import DirectionFinder, build_clip_losses, initial_delta, load_generator
    from stylemc_amd.id_loss import IDLoss
    _hip.load()
    dev = torch.device("cuda", 0)
    G = load_generator("synthetic", 1024, dev)
    styles = synthetic.synthetic_styles(129, seed=0).to(dev)
    f = DirectionFinder(G, styles, build_clip_losses("small", dev, "a", "b", synthetic_weights=True), IDLoss("a", device=dev, weights=None),
                        resolution=1024, batch_size=4, seed=0, init_delta=initial_delta(0, 0.01), n_epochs=1000)
    for _ in range(3):
        f.step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        f.step()
        torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
