"""The sharded find_direction step with the pipelined three-stream schedule, world_size 2 on the GPU.

Two fresh rank processes (tests/dist_gpu_worker.py, gloo, both ranks on device 0: a one-GPU box cannot give
RCCL two ranks) run DirectionFinder with the default schedule -- the next iteration's batch index drawn one step
early, its original image prefetched on the third stream, empty-shard ranks skipping the prefetch -- at global
batch 4 (2 + 2), 3 (2 + 1, and a short last batch of 1 that empties rank 1) and 1 (rank 1 empty every step).
The result must equal this process's single-rank run of the same global batches within the CPU gloo test's
tolerance (tests/test_distributed_cpu.py): the all_reduce of the sum-form shard gradients reproduces the
single-process gradient up to fp32 reduction order and batch-size-dependent kernel plans (split-K factors).
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
    ref = W.run_cases(sdist.World(), dev, *W.problem(dev))
    for gb, _, steps in W.CASES:
        assert np.array_equal(got[f"picks_{gb}"], ref[f"picks_{gb}"]), gb
        assert np.isfinite(got[f"delta_{gb}"]).all()
        for key in ("delta", "sdir", "parts"):
            a, b = got[f"{key}_{gb}"], ref[f"{key}_{gb}"]
            err = float(np.abs(a - b).max())
            assert err <= 1e-4 * float(np.abs(b).max()) + 1e-7, (gb, key, err)
