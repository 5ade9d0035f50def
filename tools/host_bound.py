"""Is the find_direction step host-launch bound?  Times K steps' host enqueue (no sync) against the
synchronised wall time, and counts the kernel launches of one step (torch.profiler is not used: the
count comes from rocprofv3 when run under it).

    python tools/host_bound.py [--steps K] [--no-batch-losses]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--no-batch-losses", action="store_true")
    p.add_argument("--no-overlap", action="store_true")
    a = p.parse_args()
    from stylemc_amd import _hip, synthetic
    from stylemc_amd.find_direction import DirectionFinder, build_clip_losses, initial_delta, load_generator
    from stylemc_amd.id_loss import IDLoss
    _hip.load()
    dev = torch.device("cuda", 0)
    G = load_generator("synthetic", 1024, dev)
    styles = synthetic.synthetic_styles(129, seed=0).to(dev)
    clip = build_clip_losses("small", dev, "a", "b", synthetic_weights=True)
    f = DirectionFinder(G, styles, clip, IDLoss("a", device=dev, weights=None), resolution=1024, batch_size=4,
                        seed=0, init_delta=initial_delta(0, 0.01), n_epochs=1000,
                        batch_losses=not a.no_batch_losses, overlap=not a.no_overlap)
    for _ in range(3):
        f.step()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h0 = time.perf_counter()
        f.step()
        host.append(time.perf_counter() - h0)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    host.sort()
    print(f"steps {a.steps}: enqueue {1e3 * t_enq / a.steps:.2f} ms/step (median step() {1e3 * host[len(host) // 2]:.2f} ms, "
          f"max {1e3 * host[-1]:.2f}), wall {1e3 * t_all / a.steps:.2f} ms/step")
    # per-step host time with the GPU idle-waiting each step (the pure launch cost)
    iso = []
    for _ in range(5):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        f.step()
        iso.append(time.perf_counter() - h0)
        torch.cuda.synchronize()
    iso.sort()
    print(f"isolated step() host time: median {1e3 * iso[2]:.2f} ms")


if __name__ == "__main__":
    main()
