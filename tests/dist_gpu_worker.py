"""One rank of the multi-rank GPU find_direction test (tests/test_gpu_distributed.py).

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p SMC_DIST_BACKEND=gloo SMC_SHARE_GPU=1 \
        python -m tests.dist_gpu_worker OUT.npz

Runs `run_cases` (the same DirectionFinder problems the test runs single-process) with the default three-stream
schedule -- edited synthesis on the main stream, IR-SE50 beside CLIP on the side stream, the next iteration's
original image prefetched on the third stream -- and the rank's shard of every global batch; rank 0 writes the
results.  Started as a fresh process (never forked from a process that touched the GPU).
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

# (global batch, S codes, steps[, per-rank batch]): even shards (4 over 8), uneven 2 + 1 with a short last batch of 1
# that leaves rank 1 empty (3 over 7), and rank 1 empty on every step (1 over 3).  The per-rank batch (default: the
# global batch) is the finder's batch_size, i.e. the planning batch of every launch (smc_set_plan_batch).
CASES_BY_RES = {
    256: ((4, 8, 3), (3, 7, 4), (1, 3, 3)),
    # the headline configuration (BASELINE configs 2-3): FFHQ-1024 at a global batch of 4 split 2 + 2 (parity mode),
    # and 4 images per rank (throughput mode: global batch 8, the 1-rank run plans as for 4 images per launch)
    1024: ((4, 8, 2), (8, 16, 2, 4)),
}
RES = int(os.environ.get("SMC_DIST_RES", "256"))
CASES = CASES_BY_RES[RES]


def case(c):
    """(global batch, S codes, steps, per-rank batch) of a CASES entry."""
    return (c[0], c[1], c[2], c[3] if len(c) > 3 else c[0])


def problem(dev):
    from stylemc_amd import networks, synthetic, utils
    from stylemc_amd.clip_loss import CLIPLoss
    from stylemc_amd.id_loss import IDLoss
    cfg = synthetic.generator_config(resolution=RES)
    G = networks.build_generator(cfg, synthetic.generator_state_dict(cfg, seed=0), device=dev)
    text = synthetic.text_direction("a photo of a face of a feminine woman", "a photo of a face of a man")
    clip = [(CLIPLoss(dev, text_features=text, synthetic_weights=True, seed=4), 1.0)]
    # get_temp_shapes replaces every affine by Identity (utils.py:100-120): once per generator
    return G, clip, IDLoss(device=dev, weights=None, seed=3), utils.get_temp_shapes(G)


def _finder(world, dev, G, clip, idl, shapes, gb, n_items, bs=None):
    from stylemc_amd import synthetic
    from stylemc_amd.find_direction import DirectionFinder, initial_delta
    styles = synthetic.synthetic_styles(n_items, seed=5).to(dev)
    f = DirectionFinder(G, styles, clip, idl, resolution=RES, batch_size=bs or gb, global_batch=gb, n_epochs=4,
                        seed=1, world=world, init_delta=initial_delta(0, 0.01), temp_shapes=shapes)
    assert f.prefetch_orig and f.batch_losses and f._side_stream() is not None, "not the pipelined schedule"
    return f


def _record(out, gb, f, parts, picks):
    torch.cuda.synchronize()
    out[f"delta_{gb}"] = f.delta.cpu().numpy()
    out[f"sdir_{gb}"] = f.styles_direction.cpu().numpy()
    out[f"parts_{gb}"] = torch.stack(parts).numpy()
    out[f"picks_{gb}"] = np.array(picks)


def run_cases(world, dev, G, clip, idl, shapes):
    """Every CASES problem through DirectionFinder.step with `world` (the real N-rank run, or one rank)."""
    out = {}
    for c in CASES:
        gb, n_items, steps, bs = case(c)
        f = _finder(world, dev, G, clip, idl, shapes, gb, n_items, bs)
        parts, picks = [], []
        for _ in range(steps):
            last = f.step()
            parts.append(last["parts"].cpu())
            picks.append(last["batch"])
        _record(out, gb, f, parts, picks)
    return out


def run_cases_simulated(dev, G, clip, idl, shapes, world_size=2):
    """The N-rank run replayed in ONE process: a finder per rank view (World(rank=r, world_size=N)), in lockstep --
    each computes its shard's per-image rows (local_step, under its own plan scope), the rows are concatenated in rank
    order (what the all_gather assembles), every view applies their fixed-order sum (apply_step)."""
    from stylemc_amd import dist as sdist
    out = {}
    for c in CASES:
        gb, n_items, steps, bs = case(c)
        fs = [_finder(sdist.World(r, world_size, 0, None, 0), dev, G, clip, idl, shapes, gb, n_items, bs)
              for r in range(world_size)]
        parts, picks = [], []
        for _ in range(steps):
            rows = torch.cat([f.local_step() for f in fs])
            buf = rows.sum(0)
            lasts = [f.apply_step(buf.clone()) for f in fs]
            parts.append(lasts[0]["parts"].cpu())
            picks.append(lasts[0]["batch"])
        for f in fs[1:]:
            assert torch.equal(f.delta, fs[0].delta)
        _record(out, gb, fs[0], parts, picks)
    return out


def main(path):
    from stylemc_amd import _hip, build
    from stylemc_amd import dist as sdist
    world = sdist.init_from_env(use_cuda=True)
    dev = torch.device("cuda", world.device_index)
    build.build(verbose=False) if world.rank == 0 else None
    world.barrier()
    _hip.load()
    out = run_cases(world, dev, *problem(dev))
    world.barrier()
    if world.rank == 0:
        out["world_size"] = np.array(world.world_size)
        np.savez(path, **out)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
