"""The sharded find_direction step with the pipelined three-stream schedule, world_size 2 on the GPU.

Two fresh rank processes (tests/dist_gpu_worker.py, gloo, both ranks on device 0: a one-GPU box cannot give
RCCL two ranks) run DirectionFinder with the default schedule -- the next iteration's batch index drawn one step
early, its original image prefetched on the third stream, empty-shard ranks skipping the prefetch -- at global
batch 4 (2 + 2), 3 (2 + 1, and a short last batch of 1 that empties rank 1) and 1 (rank 1 empty every step).

Checks:
  * bit for bit against the same two rank views replayed in this process in lockstep (local_step on each view,
    the two buffers summed -- all_reduce(SUM) of two ranks is one fp32 add per element -- apply_step on each): the
    multi-process run, its prefetch pipeline and the exchange add nothing beyond that sum;
  * against the single-rank run of the same global batches: same batch picks; loss terms rtol 1e-3, update
    cosine >= 0.9999 and max-norm relative error <= 1e-2 -- shards of 2 images run other kernel plans (split-K
    factors chosen per grid) than the 4-image batch, and the directional CLIP term amplifies those fp32 rounding
    differences step over step (tests/test_gpu_find_direction.py's tolerances, same reason).
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
    init = initial_delta(0, 0.01).numpy().astype(np.float64).ravel()
    for gb, _, steps in W.CASES:
        assert np.isfinite(got[f"delta_{gb}"]).all()
        for key in ("picks", "delta", "sdir", "parts"):
            assert np.array_equal(got[f"{key}_{gb}"], sim[f"{key}_{gb}"]), (gb, key)
        assert np.array_equal(got[f"picks_{gb}"], ref[f"picks_{gb}"]), gb
        np.testing.assert_allclose(got[f"parts_{gb}"], ref[f"parts_{gb}"], rtol=1e-3, atol=1e-5)
        a = got[f"delta_{gb}"].astype(np.float64).ravel() - init
        b = ref[f"delta_{gb}"].astype(np.float64).ravel() - init
        cos = float(a @ b / np.linalg.norm(a) / np.linalg.norm(b))
        assert cos >= 0.9999, (gb, cos)
        err = float(np.abs(got[f"delta_{gb}"] - ref[f"delta_{gb}"]).max() / np.abs(ref[f"delta_{gb}"]).max())
        assert err <= 1e-2, (gb, err)
