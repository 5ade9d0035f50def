"""world_size-2 and world_size-8 gloo coverage of the data-parallel find_direction step (CPU, no GPU).

Each rank draws the same batch index, takes a contiguous slice of the global batch and computes one row per image
(its direction gradient and loss terms); one all_gather puts every row on every rank, which sums them over the
global batch in one fixed order.  The networks here run image by image (per_image_*), so every image's row is
independent of how the batch is sharded -- the CPU twin of the GPU path's batch-invariant kernel plans
(smc_set_plan_batch) -- and the N-rank trajectory must equal the 1-process run BIT FOR BIT.
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
from tests.fd_helpers import (OracleCLIP, OracleID, TinyFace, oracle_generator, per_image_module, per_image_synth,
                              tiny_clip_visual)


def _make(world, global_batch, n_items=5, seed=3, batch_size=None):
    torch.manual_seed(0)
    G = oracle_generator(16, 256)
    styles = synthetic.synthetic_styles(n_items, seed=1)
    clip = OracleCLIP(per_image_module(tiny_clip_visual()), synthetic.text_direction("a", "b", dim=32))
    return DirectionFinder(G, styles, [(clip, 1.0)], OracleID(per_image_module(TinyFace())), resolution=16,
                           batch_size=batch_size or global_batch, global_batch=global_batch, learning_rate=1.5,
                           n_epochs=2, seed=seed, world=world, init_delta=initial_delta(0, 0.01),
                           synth_fn=per_image_synth)


def _finder(world, global_batch, n_items=5, steps=3, seed=3, batch_size=None):
    f = _make(world, global_batch, n_items, seed, batch_size)
    losses, picks = [], []
    for _ in range(steps):
        last = f.step()
        losses.append(last["parts"].clone())
        picks.append(last["batch"])
    return {"delta": f.delta.clone(), "losses": torch.stack(losses), "sdir": f.styles_direction.clone(),
            "picks": torch.tensor(picks)}


def _worker(rank, world_size, port, kw, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        w = sdist.World(rank, world_size, 0, "gloo")
        res = _finder(w, **kw)
        if rank == 0:
            torch.save(res, out)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(tmp_path, world_size, kw):
    out = str(tmp_path / f"r0_{world_size}.pt")
    mp.spawn(_worker, args=(world_size, _free_port(), kw, out), nprocs=world_size, join=True)
    return torch.load(out, weights_only=True)


def _assert_equal(got, ref):
    assert torch.isfinite(ref["delta"]).all()
    assert not torch.equal(ref["delta"], initial_delta(0, 0.01).reshape(ref["delta"].shape)), "no update happened"
    for key in ("picks", "delta", "losses", "sdir"):
        assert torch.equal(got[key], ref[key]), key


@pytest.mark.parametrize("global_batch", [4, 3, 1])
def test_two_rank_matches_single_rank_exactly(tmp_path, global_batch):
    """B=4: even shards; B=3: uneven (2+1); B=1: rank 1 owns no rows but still joins the exchange.  Bit-equal to
    the single-process run of the same global batches."""
    torch.set_num_threads(1)
    ref = _finder(sdist.World(), global_batch)
    _assert_equal(_run_ranks(tmp_path, 2, dict(global_batch=global_batch)), ref)


def test_eight_rank_parity_mode_exact(tmp_path):
    """Config-3 partitioning, parity mode: global batch 4 over 8 ranks -- ranks 4..7 own no image on any step and
    still join every exchange.  Bit-equal to the single-process run."""
    torch.set_num_threads(1)
    ref = _finder(sdist.World(), 4, n_items=9)
    _assert_equal(_run_ranks(tmp_path, 8, dict(global_batch=4, n_items=9)), ref)


def test_eight_rank_throughput_mode_exact(tmp_path):
    """Config-3 partitioning, throughput mode (--per_gpu_batch): 4 seeds per rank, global batch 32, the 129 x 8
    schedule (33 batches, the last one 8 seeds = 1 per rank; seed 29 draws batches 21, 32, 24).  Bit-equal to one
    process running the global batches of 32."""
    torch.set_num_threads(1)
    kw = dict(global_batch=32, n_items=129 * 8, seed=29, batch_size=4)
    ref = _finder(sdist.World(), **kw)
    assert ref["picks"].tolist() == [21, 32, 24]
    _assert_equal(_run_ranks(tmp_path, 8, kw), ref)


def _simulated(global_batch, steps=3, world_size=2):
    """The N-rank run replayed in one process: the rank views in lockstep, local_step each, their rows concatenated
    in rank order (what the all_gather assembles), combine + apply_step each."""
    fs = [_make(sdist.World(r, world_size, 0, None), global_batch) for r in range(world_size)]
    losses = []
    for _ in range(steps):
        rows = torch.cat([f.local_step() for f in fs])
        lasts = [f.apply_step(rows.sum(0)) for f in fs]
        losses.append(lasts[0]["parts"].clone())
    assert torch.equal(fs[0].delta, fs[1].delta)
    return fs[0].delta.clone(), torch.stack(losses), fs[0].styles_direction.clone()


@pytest.mark.parametrize("global_batch", [4, 3, 1])
def test_two_rank_matches_lockstep_replay_exactly(tmp_path, global_batch):
    """The multi-process exchange adds nothing beyond gathering the shard rows: bit-equal to the replay."""
    torch.set_num_threads(1)
    ref = _simulated(global_batch)
    got = _run_ranks(tmp_path, 2, dict(global_batch=global_batch))
    for key, r in zip(("delta", "losses", "sdir"), ref):
        assert torch.equal(got[key], r), key


def test_gather_rows_single_process_is_identity():
    w = sdist.World()
    rows = torch.randn(3, 5)
    assert torch.equal(w.gather_rows(rows, 0, 3), rows)


def test_shard_rows_partition():
    for lo, hi in [(0, 4), (8, 9), (4, 11), (0, 0)]:
        for w in (1, 2, 3, 8):
            parts = [sdist.shard_rows(lo, hi, r, w) for r in range(w)]
            assert parts[0][0] == lo and parts[-1][1] == hi
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1
