"""Run-to-run determinism of the find_direction step on one GPU (diagnostic for the flaky 2-rank == 1-rank test):
the first tests/dist_gpu_worker CASES problem (global batch 4, 8 codes, 3 steps) run 3 times per schedule --
pipelined (side stream + prefetch stream), side stream without the prefetch, single stream -- and compared bit for bit.
    python tools/det_check.py [mode,mode ...] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from stylemc_amd import _hip, build, synthetic
    from stylemc_amd import dist as sdist
    from stylemc_amd.find_direction import DirectionFinder, initial_delta
    from tests import dist_gpu_worker as W
    build.build(verbose=False)
    _hip.load()
    dev = torch.device("cuda", 0)
    G, clip, idl, shapes = W.problem(dev)
    world = sdist.World(0, 1, 0, None, 0)
    gb, n_items, steps = W.CASES[0]
    modes = {"pipelined": {}, "no_prefetch": {"prefetch_orig": False}, "single_stream": {"overlap": False},
             "pipelined_no_id_prefetch": {"prefetch_id": False}, "pipelined_id_after_bwd": {}, "pipelined_losses_on_main": {}}
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["pipelined", "no_prefetch", "single_stream"]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for name in names:
        kw = modes[name]
        outs = []
        for rep in range(reps):
            styles = synthetic.synthetic_styles(n_items, seed=5).to(dev)
            f = DirectionFinder(G, styles, clip, idl, resolution=W.RES, batch_size=gb, global_batch=gb, n_epochs=4,
                                seed=1, world=world, init_delta=initial_delta(0, 0.01), temp_shapes=shapes, **kw)
            f.diag_id_after_bwd = name == "pipelined_id_after_bwd"
            f.diag_losses_on_main = name == "pipelined_losses_on_main"
            rows = []
            for _ in range(steps):
                last = f.step()
                rows.append(last["parts"].clone())
            torch.cuda.synchronize()
            outs.append((f.delta.clone(), torch.stack(rows)))
        same = [torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1]) for o in outs[1:]]
        diff = max((outs[0][0] - o[0]).abs().max().item() for o in outs[1:])
        print(f"{name}: runs bit-equal to the first: {same}  max |d delta| {diff:.3e}", flush=True)


if __name__ == "__main__":
    main()
