"""bench.py's anti-entropy watchdog (N > 1): past --ae-deadline every rank
ends the process with exit code bench.AE_TIMEOUT_EXIT (3, non-zero: a hung
collective must not read as a clean run), and rank 0 first prints its one JSON line with
the unfinished part marked — a collective that never returns cannot cost the
measured headline. CPU only: the watchdog is exercised on a sleeping process."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = """
import argparse, sys, time
sys.path.insert(0, {repo!r})
import bench
res = {{"metric": "m", "value": 1.0, "anti_entropy": {{"config4_gcounter": {{"value": 2.0}}}}}}
bench._ae_watchdog(argparse.Namespace(ae_deadline=0.5), {rank}, res)
time.sleep(30)  # a collective that never returns
print("not reached")
"""


def _run(rank):
    return subprocess.run([sys.executable, "-c", PROG.format(repo=REPO, rank=rank)], capture_output=True, text=True,
                          timeout=60)


AE_TIMEOUT_EXIT = 3  # bench.AE_TIMEOUT_EXIT (checked below)


def test_rank0_prints_once_and_exits_nonzero():
    p = _run(0)
    assert p.returncode == AE_TIMEOUT_EXIT, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and d["anti_entropy"]["config4_gcounter"]["value"] == 2.0
    assert "unfinished" in d["anti_entropy"]


def test_other_ranks_exit_nonzero_silently():
    p = _run(1)
    assert p.returncode == AE_TIMEOUT_EXIT and p.stdout.strip() == ""


def test_exit_code_constant():
    sys.path.insert(0, REPO)
    import bench

    assert bench.AE_TIMEOUT_EXIT == AE_TIMEOUT_EXIT != 0


def test_emit_prints_at_most_once(capsys):
    sys.path.insert(0, REPO)
    import bench

    bench._emit.done = False
    assert bench._emit({"a": 1}) and not bench._emit({"a": 2})
    assert capsys.readouterr().out.strip() == json.dumps({"a": 1})
    bench._emit.done = False
