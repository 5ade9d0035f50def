"""bench.py's own N-rank launcher (no GPU): `python bench.py --gpus N` without WORLD_SIZE starts N rank
processes with the torch.distributed.run environment; a launcher WORLD_SIZE that disagrees with --gpus is an
error; a failing rank makes the launcher fail."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=300)


def test_spawns_n_ranks():
    r = _run(["--gpus", "3", "--launch-probe"], SMC_SHARE_GPU="1")
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(int(l["RANK"]) for l in lines) == [0, 1, 2]
    assert {l["WORLD_SIZE"] for l in lines} == {"3"}
    assert {l["LOCAL_RANK"] for l in lines} == {"0", "1", "2"}
    assert len({l["MASTER_PORT"] for l in lines}) == 1
    assert {l["MASTER_ADDR"] for l in lines} == {"127.0.0.1"}
    assert {l["SMC_BENCH_LAUNCHER"] for l in lines} == {"bench.py"}


def test_failing_rank_fails_launcher():
    r = _run(["--gpus", "2", "--launch-probe"], SMC_SHARE_GPU="1", SMC_PROBE_FAIL_RANK="1")
    assert r.returncode == 3, (r.returncode, r.stderr)


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "4", "--launch-probe"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_too_few_gpus_without_sharing():
    r = _run(["--gpus", "2", "--launch-probe"], SMC_SHARE_GPU="0")
    assert r.returncode == 2
    assert "GPU(s) visible" in r.stderr
