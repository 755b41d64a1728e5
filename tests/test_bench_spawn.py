"""CPU: bench.py's own multi-rank launch (no torchrun). `--gpus N` without
WORLD_SIZE in the environment must start N fresh worker processes of itself
(RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1) before any
GPU call, relay rank 0's JSON line and return the workers' exit status. The
spawn_check workload runs the launch path over gloo and reports what each
rank saw; --gpus 1 stays a single process."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env, cwd=REPO)
    return p


def _line(p):
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, (p.stdout, p.stderr)
    return json.loads(lines[0])


def test_spawn_two_ranks_gloo():
    p = _run("--gpus", "2", "--workload", "spawn_check")
    assert p.returncode == 0, p.stderr
    res = _line(p)
    assert res["n_gpus"] == 2
    ranks = res["ranks"]
    assert [r[:3] for r in ranks] == [[0, 2, 0], [1, 2, 1]]  # rank, world, LOCAL_RANK (the GPU it binds)
    pids = {r[3] for r in ranks}
    assert len(pids) == 2  # two distinct worker processes


def test_single_gpu_is_not_spawned():
    p = _run("--gpus", "1", "--workload", "spawn_check")
    assert p.returncode == 0, p.stderr
    res = _line(p)
    assert res["n_gpus"] == 1 and [r[:3] for r in res["ranks"]] == [[0, 1, 0]]


def test_spawned_failure_propagates():
    """Workers that fail (here: the GPU workload in a container without a GPU,
    each worker's torch.cuda.set_device raises) make the launcher return
    non-zero, with no JSON line, instead of hanging."""
    p = _run("--gpus", "2", "--workload", "orswot", "--n-obj", "64")
    assert p.returncode != 0
    assert not [x for x in p.stdout.splitlines() if x.startswith("{")]
