"""Look for host syncs in DirectionFinder.step(): torch's sync debug mode (.item() / blocking copies ...) and the
caching allocator's segment allocations (hipMalloc) per step after warm-up.
    python tools/sync_probe.py [--steps 6]"""
import os
import sys
import time
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 6
    from stylemc_amd import _hip, synthetic
    from stylemc_amd.find_direction import DirectionFinder, build_clip_losses, initial_delta, load_generator
    from stylemc_amd.id_loss import IDLoss
    _hip.load()
    dev = torch.device("cuda", 0)
    G = load_generator("synthetic", 1024, dev)
    styles = synthetic.synthetic_styles(129, seed=0).to(dev)
    clip = build_clip_losses("small", dev, "a", "b", synthetic_weights=True)
    f = DirectionFinder(G, styles, clip, IDLoss("a", device=dev, weights=None), resolution=1024, batch_size=4, seed=0,
                        init_delta=initial_delta(0, 0.01), n_epochs=1000)
    for _ in range(4):
        f.step()
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("warn")
    st0 = torch.cuda.memory_stats()
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        t = []
        for _ in range(steps):
            t0 = time.perf_counter()
            f.step()
            t.append(1e3 * (time.perf_counter() - t0))
        torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode(0)
    st1 = torch.cuda.memory_stats()
    print("host step() ms:", [round(x, 2) for x in t])
    print("sync warnings:", len(w))
    for x in w[:10]:
        print("  ", str(x.message)[:200], x.filename, x.lineno)
    for k in ["num_alloc_retries", "segment.all.allocated", "num_device_alloc", "num_device_free", "num_sync_all_streams"]:
        print(k, st1.get(k, 0) - st0.get(k, 0))


if __name__ == "__main__":
    main()
