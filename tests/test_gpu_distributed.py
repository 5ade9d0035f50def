"""The sharded find_direction step with the pipelined three-stream schedule, world_size 2 on the GPU.

Two fresh rank processes (tests/dist_gpu_worker.py, gloo, both ranks on device 0: a one-GPU box cannot give
RCCL two ranks) run DirectionFinder with the default schedule -- the next iteration's batch index drawn one step
early, its original image prefetched on the third stream, empty-shard ranks skipping the prefetch -- at global
batch 4 (2 + 2), 3 (2 + 1, and a short last batch of 1 that empties rank 1) and 1 (rank 1 empty every step).

Every launch of a shard is planned for the full batch (smc_set_plan_batch: split-K factors, tile configurations and
channel splits from the planning batch, not the shard), the loss heads reduce rows in a fixed order (rowops), each
image's gradient row comes back separately and the global batch's rows are summed in one fixed order after the
all_gather.  That makes every piece of a shard's step bit-equal to the full batch's (tests/test_gpu_batch_invariance.py)
and the 8-rank gloo runs bit-exact (tests/test_distributed_cpu.py).  This pipelined schedule itself, however, is not
run-to-run reproducible on the GPU (round 5, tools/det_check.py: about one run in eight differs from the others, up to
5e-4 (absolute) in delta after three steps, within one process too -- root cause open),
so the two-rank run is compared with the single-rank run and with the lockstep replay at tolerance: batch picks
exact, delta / saved direction / loss terms within 1e-2 of their max and cosine >= 0.9999.
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


def _two_ranks(out):
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SMC_DIST_BACKEND="gloo", SMC_SHARE_GPU="1")
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


def test_two_ranks_pipelined_match_single_rank(tmp_path):
    from stylemc_amd import _hip, build
    from stylemc_amd import dist as sdist
    build.build(verbose=False)
    _hip.load()
    out = str(tmp_path / "rank0.npz")
    codes = _two_ranks(out)
    assert codes == [0, 0], codes
    got = dict(np.load(out))
    assert int(got["world_size"]) == 2
    dev = torch.device("cuda", 0)
    prob = W.problem(dev)
    sim = W.run_cases_simulated(dev, *prob)
    ref = W.run_cases(sdist.World(), dev, *prob)
    from stylemc_amd.find_direction import initial_delta
    for gb, _, steps in W.CASES:
        assert np.isfinite(got[f"delta_{gb}"]).all()
        init = initial_delta(0, 0.01).numpy().reshape(got[f"delta_{gb}"].shape)
        assert not np.array_equal(got[f"delta_{gb}"], init), gb
        assert np.array_equal(got[f"picks_{gb}"], sim[f"picks_{gb}"]), (gb, "vs lockstep replay")
        assert np.array_equal(got[f"picks_{gb}"], ref[f"picks_{gb}"]), (gb, "vs the 1-rank run")
        for key in ("delta", "sdir", "parts"):
            a = got[f"{key}_{gb}"].astype(np.float64).ravel()
            for other, what in ((sim, "vs lockstep replay"), (ref, "vs the 1-rank run")):
                b = other[f"{key}_{gb}"].astype(np.float64).ravel()
                rel = np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)
                cos = a @ b / max(np.linalg.norm(a) * np.linalg.norm(b), 1e-30)
                assert rel <= 1e-2 and cos >= 0.9999, (gb, key, what, rel, cos)
