"""The sharded find_direction step with the pipelined three-stream schedule, world_size 2 on the GPU.

Two fresh rank processes (tests/dist_gpu_worker.py, gloo, both ranks on device 0: a one-GPU box cannot give
RCCL two ranks) run DirectionFinder with the default schedule -- the next iteration's batch index drawn one step
early, its original image prefetched on the third stream, empty-shard ranks skipping the prefetch -- at global
batch 4 (2 + 2), 3 (2 + 1, and a short last batch of 1 that empties rank 1) and 1 (rank 1 empty every step).

Every launch of a shard is planned for the full batch (smc_set_plan_batch: split-K factors, tile configurations and
channel splits from the planning batch, not the shard), the loss heads reduce rows in a fixed order (rowops), each
image's gradient row comes back separately and the global batch's rows are summed in one fixed order after the
all_gather.  That makes every piece of a shard's step bit-equal to the full batch's (tests/test_gpu_batch_invariance.py)
and the 8-rank gloo runs bit-exact (tests/test_distributed_cpu.py).  The pipelined schedule is run-to-run reproducible
since round 6 (the attention backward's LDS staging), so the two-rank run must equal the
single-rank run and the lockstep replay BIT FOR BIT: batch picks, deltas, saved directions and loss terms.
The same holds at the headline configuration (FFHQ-1024, SMC_DIST_RES=1024): a global batch of 4 split 2 + 2, and
4 images per rank (global batch 8) against one process running the batch of 8 planned as 4 per launch.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from tests import dist_gpu_worker as W

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _two_ranks(out, res=256):
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SMC_DIST_BACKEND="gloo", SMC_SHARE_GPU="1", SMC_DIST_RES=str(res))
        procs.append(subprocess.Popen([sys.executable, "-u", "-m", "tests.dist_gpu_worker", out], cwd=REPO,
                                      env=env))
    codes = []
    try:
        for p in procs:
            codes.append(p.wait(timeout=240))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return codes


def _check_bit_equal(got, runs, cases):
    from stylemc_amd.find_direction import initial_delta
    for c in cases:
        gb = W.case(c)[0]
        assert np.isfinite(got[f"delta_{gb}"]).all()
        init = initial_delta(0, 0.01).numpy().reshape(got[f"delta_{gb}"].shape)
        assert not np.array_equal(got[f"delta_{gb}"], init), gb
        for key in ("picks", "delta", "sdir", "parts"):
            for other, what in runs:
                a, b = got[f"{key}_{gb}"], other[f"{key}_{gb}"]
                assert np.array_equal(a, b), (gb, key, what, float(np.abs(a.astype(np.float64) - b).max()))


def _run(tmp_path, res, replay):
    from stylemc_amd import _hip, build
    from stylemc_amd import dist as sdist
    build.build(verbose=False)
    _hip.load()
    out = str(tmp_path / "rank0.npz")
    codes = _two_ranks(out, res)
    assert codes == [0, 0], codes
    got = dict(np.load(out))
    assert int(got["world_size"]) == 2
    old_res, old_cases = W.RES, W.CASES
    W.RES, W.CASES = res, W.CASES_BY_RES[res]
    try:
        dev = torch.device("cuda", 0)
        prob = W.problem(dev)
        runs = [(W.run_cases(sdist.World(), dev, *prob), "vs the 1-rank run")]
        if replay:
            runs.append((W.run_cases_simulated(dev, *prob), "vs lockstep replay"))
        _check_bit_equal(got, runs, W.CASES)
    finally:
        W.RES, W.CASES = old_res, old_cases


def test_two_ranks_pipelined_match_single_rank(tmp_path):
    _run(tmp_path, 256, replay=True)


def test_two_ranks_pipelined_match_single_rank_ffhq1024(tmp_path):
    """Config 3's sharded step at its own size: FFHQ-1024, global batch 4 over 2 ranks and 4 images per rank."""
    _run(tmp_path, 1024, replay=False)
