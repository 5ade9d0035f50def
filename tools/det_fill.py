"""Deterministic stale-read probe (round 6): every torch.empty / torch.empty_like / Tensor.new_empty made from Python
(the outputs and workspaces handed to libstylemc_hip) is filled with a chosen value before the library sees it.  A
kernel that reads an element of its output or workspace that it did not write (in this launch or an earlier one of
the same call) then changes the result with the fill value, in one run, whatever the timing.
    python tools/det_fill.py res mode fill[,fill...] [module-filter]
module-filter: only allocations whose calling file path contains this string are filled (bisection).
"""
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

_FILL = {"v": None, "filter": None, "count": 0}
_empty, _empty_like = torch.empty, torch.empty_like


def _maybe_fill(t):
    v = _FILL["v"]
    if v is None or not t.is_cuda or not t.is_floating_point():
        return t
    flt = _FILL["filter"]
    if flt:
        caller = traceback.extract_stack(limit=3)[0].filename
        if flt not in caller:
            return t
    _FILL["count"] += 1
    return t.fill_(v)


def empty(*a, **k):
    return _maybe_fill(_empty(*a, **k))


def empty_like(*a, **k):
    return _maybe_fill(_empty_like(*a, **k))


def main():
    res = int(sys.argv[1])
    mode = sys.argv[2]
    fills = [float(x) for x in sys.argv[3].split(",")]
    _FILL["filter"] = sys.argv[4] if len(sys.argv) > 4 else None
    torch.empty, torch.empty_like = empty, empty_like
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
    kws = {"pipelined": {}, "no_prefetch": {"prefetch_orig": False}, "single_stream": {"overlap": False}}
    ref = None
    for v in [None] + fills:
        _FILL["v"], _FILL["count"] = v, 0
        styles = synthetic.synthetic_styles(8, seed=5).to(dev)
        f = FD.DirectionFinder(G, styles, clip, idl, resolution=res, batch_size=4, global_batch=4, n_epochs=4, seed=1,
                               world=world, init_delta=FD.initial_delta(0, 0.01), temp_shapes=shapes, **kws[mode])
        grads = [f.step()["grad"].clone() for _ in range(3)]
        torch.cuda.synchronize()
        out = torch.stack(grads).cpu()
        if ref is None:
            ref = out
        d = [(ref[s] - out[s]).abs().nan_to_num(float("inf")).max().item() for s in range(3)]
        print(f"{mode} fill {v}: filled {_FILL['count']} allocations; finite {bool(torch.isfinite(out).all())}; "
              f"max|d| per step vs unfilled " + " ".join(f"{x:.2e}" for x in d), flush=True)


if __name__ == "__main__":
    main()
