"""Single-run hazard probe for the pipelined find_direction step (round 6).

SMC_POISON=1: every torch allocation starts as NaN (torch.use_deterministic_algorithms + fill_uninitialized_memory):
a kernel that reads an element nobody wrote in this run, or a block the caching allocator handed to another stream
while a kernel still reads it, then shows up in that one run instead of ~1 run in 8.  Each run's per-step gradients
are saved (gpurun_out/r06/det_<tag>.pt) so that runs of different processes can be compared.
    python tools/det_nan.py res reps mode[,mode...] [tag]
modes: single_stream, no_prefetch, pipelined, pipelined_no_id_prefetch, pipelined_sync_step (device sync after every
step), pipelined_sync_pref (the prefetch waited for on the host right after it is enqueued)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    res = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["single_stream", "no_prefetch", "pipelined"]
    tag = sys.argv[4] if len(sys.argv) > 4 else "run"
    poison = os.environ.get("SMC_POISON", "1") == "1"
    if poison:
        torch.use_deterministic_algorithms(True, warn_only=True)
        from torch.utils import deterministic
        deterministic.fill_uninitialized_memory = True
    from stylemc_amd import _hip, build, synthetic
    from stylemc_amd import dist as sdist
    from stylemc_amd import find_direction as FD
    from tests import dist_gpu_worker as W
    W.RES = res
    build.build(verbose=False)
    _hip.load()
    dev = torch.device("cuda", 0)
    G, clip, idl, shapes = W.problem(dev)
    world = sdist.World(0, 1, 0, None, 0)
    gb, n_items, steps = 4, 8, 3
    kws = {"pipelined": {}, "no_prefetch": {"prefetch_orig": False}, "single_stream": {"overlap": False},
           "pipelined_no_id_prefetch": {"prefetch_id": False}, "pipelined_sync_step": {}, "pipelined_sync_pref": {}}
    orig_prefetch = FD.DirectionFinder._prefetch_next
    saved = {}
    print(f"res {res} poison {poison}", flush=True)
    for name in modes:
        def pref(self, _sync=name == "pipelined_sync_pref"):
            orig_prefetch(self)
            if _sync:
                torch.cuda.synchronize()
        FD.DirectionFinder._prefetch_next = pref
        for rep in range(reps):
            styles = synthetic.synthetic_styles(n_items, seed=5).to(dev)
            f = FD.DirectionFinder(G, styles, clip, idl, resolution=res, batch_size=gb, global_batch=gb, n_epochs=4,
                                   seed=1, world=world, init_delta=FD.initial_delta(0, 0.01), temp_shapes=shapes,
                                   **kws[name])
            grads = []
            for _ in range(steps):
                grads.append(f.step()["grad"].clone())
                if name == "pipelined_sync_step":
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            out = torch.stack(grads).cpu()
            saved[f"{name}/{rep}"] = out
            ref = saved[f"{name}/0"]
            fin = [bool(torch.isfinite(g).all()) for g in out]
            d = [(ref[s] - out[s]).abs().nan_to_num(float("inf")).max().item() for s in range(steps)]
            print(f"{name} rep {rep}: finite {fin}  max|d| per step vs rep 0 " + " ".join(f"{x:.2e}" for x in d),
                  flush=True)
    FD.DirectionFinder._prefetch_next = orig_prefetch
    os.makedirs("gpurun_out/r06", exist_ok=True)
    torch.save(saved, f"gpurun_out/r06/det_{tag}.pt")


if __name__ == "__main__":
    main()
