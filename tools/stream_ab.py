"""A/B of how the find_direction step's HIP streams are created.

    python tools/stream_ab.py [--steps 10]

Round 2 measured 33 ms/step (against 21) for a tree whose streams were all created at an explicit priority 0
and did not explain it.  Each variant below runs the default 3-stream schedule (FFHQ-1024, batch 4, HIP losses)
and reports ms/step plus what the caching allocator did during the timed steps (device allocations / frees,
allocation retries, cross-stream syncs: a hipMalloc / hipFree inside a step synchronises the device) and the
stream handles, so a slowdown can be attributed to stream placement or to allocator behaviour.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KEYS = ("num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams",
        "segment.all.allocated", "segment.all.freed")


def stats():
    s = torch.cuda.memory_stats()
    return {k: s.get(k, 0) for k in KEYS}


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

    variants = [
        ("default: pool streams, default priority", None, None),
        ("side/prefetch Stream(priority=0)", lambda d: torch.cuda.Stream(device=d, priority=0), None),
        ("side/prefetch Stream(priority=-1)", lambda d: torch.cuda.Stream(device=d, priority=-1), None),
        ("main on a pool stream too", None, lambda d: torch.cuda.Stream(device=d)),
        ("main + side + prefetch priority=0", lambda d: torch.cuda.Stream(device=d, priority=0),
         lambda d: torch.cuda.Stream(device=d, priority=0)),
        ("main priority=-1, side/prefetch 0", lambda d: torch.cuda.Stream(device=d, priority=0),
         lambda d: torch.cuda.Stream(device=d, priority=-1)),
        ("default again", None, None),
    ]
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (None, None)
    print(f"priority range (least, greatest) = {lo}, {hi}; default stream {torch.cuda.current_stream().cuda_stream:#x}")
    for name, factory, main_factory in variants:
        f = FD.DirectionFinder(G, styles, clip, idl, resolution=1024, batch_size=4, seed=0, temp_shapes=ts,
                               init_delta=FD.initial_delta(0, 0.01), n_epochs=1000, stream_factory=factory)
        main = main_factory(dev) if main_factory else torch.cuda.current_stream()
        with torch.cuda.stream(main):
            for _ in range(3):
                f.step()
            torch.cuda.synchronize()
            a = stats()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(steps):
                f.step()
            e.record()
            torch.cuda.synchronize()
            b = stats()
        ms = s.elapsed_time(e) / steps
        handles = [main.cuda_stream, f._side.cuda_stream, f._pre.cuda_stream]
        delta = {k: b[k] - a[k] for k in KEYS if b[k] != a[k]}
        print(f"{name:40s} {ms:7.2f} ms/step  streams(main, side, pre) = "
              f"{', '.join(f'{h:#x}' for h in handles)}  priorities = {main.priority}, {f._side.priority}, "
              f"{f._pre.priority}  allocator during timed steps: {delta or 'no device alloc/free'}", flush=True)
        del f
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
