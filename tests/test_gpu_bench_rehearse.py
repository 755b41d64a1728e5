"""GPU: bench.py's N > 1 accounting, rehearsed on the box's one MI355X
(--rehearse: every rank a process on cuda:0, the product's joins over the
gloo transport). The config-5 replica join must report exactly 3 host
synchronisations per step (crdt_ctx_host_syncs counted from the end of the
settle phase over warmup + timed steps) at N = 2 and 3, with identical bytes
on every rank and a sampled oracle check; config 4's all-reduce and its
owner-shard reduce-scatter both run through the product
(crdt_replica_*_max_transport) and pass their checks."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--rehearse", "--no-cpu-baseline",
                        "--settle-ms", "20", *args], capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 3])
def test_replica_join_three_syncs_per_step(world):
    r = _bench("--gpus", str(world), "--workload", "orswot_csr", "--n-obj", "12000", "--steps", "3", "--warmup", "2")
    assert r["n_gpus"] == world
    assert r["check"]["ok"], r["check"]
    assert r["comm"]["host_syncs_per_step"] == 3.0, r["comm"]
    assert r["settle"]["launches"] >= 1


def test_gcounter_ae_rehearsal_through_the_product():
    r = _bench("--gpus", "2", "--workload", "gcounter_ae", "--n-obj", "200000", "--steps", "2", "--warmup", "1")
    assert r["check"]["ok"], r["check"]
    assert r["comm"]["transport"] == "gloo (rehearsal)"
    assert r["comm"]["reduce_scatter"]["ms"] > 0
