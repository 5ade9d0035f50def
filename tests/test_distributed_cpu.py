"""world_size-2 gloo coverage of the data-parallel find_direction step (CPU, no GPU).

Each rank draws the same batch index, takes a contiguous slice of the global batch and the single
all_reduce(SUM) per step combines gradient + loss terms; the trajectory must equal the 1-process run
with the same global batch up to reduction order.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stylemc_amd import dist as sdist
from stylemc_amd import synthetic
from stylemc_amd.find_direction import DirectionFinder, initial_delta
from tests.fd_helpers import OracleCLIP, OracleID, TinyFace, oracle_generator, oracle_rows_synth, tiny_clip_visual


def _make(world, global_batch, n_items=5):
    torch.manual_seed(0)
    G = oracle_generator(16, 256)
    styles = synthetic.synthetic_styles(n_items, seed=1)
    clip = OracleCLIP(tiny_clip_visual(), synthetic.text_direction("a", "b", dim=32))
    return DirectionFinder(G, styles, [(clip, 1.0)], OracleID(TinyFace()), resolution=16, batch_size=global_batch,
                           global_batch=global_batch, learning_rate=1.5, n_epochs=2, seed=3, world=world,
                           init_delta=initial_delta(0, 0.01), synth_fn=oracle_rows_synth)


def _finder(world, global_batch, n_items=5, steps=3):
    f = _make(world, global_batch, n_items)
    losses = []
    for _ in range(steps):
        last = f.step()
        losses.append(last["parts"].clone())
    return f.delta.clone(), torch.stack(losses), f.styles_direction.clone()


def _worker(rank, world_size, port, global_batch, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        w = sdist.World(rank, world_size, 0, "gloo")
        delta, losses, sdir = _finder(w, global_batch)
        if rank == 0:
            torch.save({"delta": delta, "losses": losses, "sdir": sdir}, out)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("global_batch", [4, 3, 1])
def test_two_rank_matches_single_rank(tmp_path, global_batch):
    """B=4: even shards; B=3: uneven (2+1); B=1: rank 1 owns no rows but still joins the all_reduce."""
    torch.set_num_threads(2)
    ref_delta, ref_losses, ref_sdir = _finder(sdist.World(), global_batch)
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), global_batch, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    assert torch.isfinite(ref_delta).all()
    # fp32 reduction order + batch-size-dependent CPU conv algorithms differ at ~1e-7 relative; the
    # directional CLIP term's 1/|E(tgt)-E(src)| amplifies that over steps, hence max-norm tolerances.
    for key, ref in (("delta", ref_delta), ("losses", ref_losses), ("sdir", ref_sdir)):
        err = (got[key] - ref).abs().max().item()
        assert err <= 1e-4 * ref.abs().max().item() + 1e-7, (key, err)


def _simulated(global_batch, steps=3):
    """The 2-rank run replayed in one process: two rank views in lockstep, local_step each, buffers summed (what
    all_reduce(SUM) of two ranks computes), apply_step each."""
    fs = [_make(sdist.World(r, 2, 0, None), global_batch) for r in range(2)]
    losses = []
    for _ in range(steps):
        b0, b1 = (f.local_step() for f in fs)
        tot = b0 + b1
        lasts = [f.apply_step(tot.clone()) for f in fs]
        losses.append(lasts[0]["parts"].clone())
    assert torch.equal(fs[0].delta, fs[1].delta)
    return fs[0].delta.clone(), torch.stack(losses), fs[0].styles_direction.clone()


@pytest.mark.parametrize("global_batch", [4, 3, 1])
def test_two_rank_matches_lockstep_replay_exactly(tmp_path, global_batch):
    """The multi-process exchange adds nothing beyond the sum of the shard buffers: bit-equal to the replay."""
    torch.set_num_threads(1)
    ref = _simulated(global_batch)
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), global_batch, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    for key, r in zip(("delta", "losses", "sdir"), ref):
        assert torch.equal(got[key], r), key


def test_shard_rows_partition():
    for lo, hi in [(0, 4), (8, 9), (4, 11), (0, 0)]:
        for w in (1, 2, 3, 8):
            parts = [sdist.shard_rows(lo, hi, r, w) for r in range(w)]
            assert parts[0][0] == lo and parts[-1][1] == hi
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1
