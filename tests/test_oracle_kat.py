"""CPU: pin the oracle to the reference's own tests (no GPU).

- every Orswot KAT script (tests/golden/kat_orswot.json) passes on the
  pure-Python restatement AND on the C++ oracle, and both produce the same
  canonical record after every merge;
- the VClock / GCounter / PNCounter KATs (tests/golden/kat_vclock_counters.json);
- prop_merge_converges (test/orswot.rs:37-76, test/pncounter.rs:22-53) with
  seeded op vectors;
- random differential: Python restatement vs C++ oracle, record-byte equal.
"""
import json
import os
import random

import numpy as np
import pytest

import crdts_ref
import kat_runner
import opgen
import records

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = kat_runner.load_cases()
QC = kat_runner.load_qc_scenarios()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_orswot_kat_python(case):
    kat_runner.run_case(case, kat_runner.PyBackend())


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_orswot_kat_oracle_matches_python(case, oracle):
    tp, to = [], []
    kat_runner.run_case(case, kat_runner.PyBackend(), trace=tp)
    kat_runner.run_case(case, kat_runner.OracleBackend(), trace=to)
    assert len(tp) == len(to)
    for (k1, n1, a), (k2, n2, b) in zip(tp, to):
        assert (k1, n1) == (k2, n2)
        assert records.from_py(a, 16) == b.encode(16), f"{case['name']} step {k1}"


def _kv():
    with open(os.path.join(GOLDEN, "kat_vclock_counters.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("kat", _kv()["vclock_binop"], ids=lambda k: k["name"])
def test_vclock_binop_kat(kat, oracle):
    exp = [tuple(x) for x in kat["expect"]]
    assert oracle.vclock_binop(kat["op"], kat["a"], kat["b"]) == exp
    a = crdts_ref.VClock(kat["a"])
    b = crdts_ref.VClock(kat["b"])
    getattr(a, kat["op"])(b)
    assert a.canonical() == tuple(exp)


def test_vclock_ordering_kat(oracle):
    kat = _kv()["vclock_ordering"]
    for st in kat["steps"]:
        assert oracle.vclock_partial_cmp(st["a"], st["b"]) == st["cmp"], st
        a, b = crdts_ref.VClock(st["a"]), crdts_ref.VClock(st["b"])
        got = {0: "Equal", 1: "Greater", -1: "Less", None: "None"}[a.partial_cmp(b)]
        assert got == st["cmp"], st


def test_gcounter_pncounter_basic_kat(oracle):
    kv = _kv()
    g = kv["gcounter_basic"]
    a, b = crdts_ref.GCounter(), crdts_ref.GCounter()
    a.apply(a.inc(g["a_ops"][0]))
    b.apply(b.inc(g["b_ops"][0]))
    assert [a.value(), b.value()] == g["values_after_first"]
    a.apply(a.inc(g["a_ops"][1]))
    assert a.value() == g["a_value_final"] and b.value() == g["b_value_final"]
    p = kv["pncounter_basic"]
    c = crdts_ref.PNCounter()
    vals = []
    for op in p["ops"]:
        c.apply(c.inc(0) if op == "inc" else c.dec(0))
        vals.append(c.value())
    assert vals == p["values"]


def _converge_orswot(ops, backend, n_actors=None):
    """test/orswot.rs:37-76 — witnesses by actor % i, merged in index order, + plunger."""
    result = None
    for i in range(2, 11):
        ws = [backend.new() for _ in range(i)]
        for actor, op in ops:
            opgen.apply_op(backend, ws[actor % i], op)
        merged = backend.new()
        for w in ws:
            backend.merge(merged, w)
        backend.merge(merged, backend.new())
        if result is None:
            result = merged
        else:
            yield result, merged


@pytest.mark.parametrize("seed", range(40))
def test_prop_orswot_merge_converges(seed, oracle):
    rng = random.Random(seed)
    ops = opgen.orswot_opvec(rng)
    py = kat_runner.PyBackend()
    for a, b in _converge_orswot(ops, py):
        assert a == b
    ob = kat_runner.OracleBackend()
    for a, b in _converge_orswot(ops, ob):
        assert a.encode(100) == b.encode(100)


@pytest.mark.parametrize("seed", range(20))
def test_prop_pncounter_merge_converges(seed, oracle):
    rng = random.Random(1000 + seed)
    ops = opgen.pncounter_opvec(rng)
    vals = set()
    for i in range(2, 11):
        ws = [crdts_ref.PNCounter() for _ in range(i)]
        for (actor, counter), pos in ops:
            ws[actor % i].apply(((actor, counter), pos))
        merged = crdts_ref.PNCounter()
        for w in ws:
            merged.merge(w)
        vals.add(merged.value())
        # oracle merge over the same rows
        rows = np.zeros((i, 2 * 11), dtype=np.uint64)
        for r, w in enumerate(ws):
            for a, c in w.p.inner.dots.items():
                rows[r, a] = c
            for a, c in w.n.inner.dots.items():
                rows[r, 11 + a] = c
        acc = np.zeros((1, 22), dtype=np.uint64)
        for r in range(i):
            acc = oracle.pncounter_merge(acc, rows[r:r + 1], 11)
        p = int(acc[0, :11].sum())
        n = int(acc[0, 11:].sum())
        assert p - n == merged.value()
    assert len(vals) == 1


def _random_pair(rng, n_actors=8, members=12, ops=24):
    """Two replicas diverging from a common ancestor via random ops."""
    anc = crdts_ref.Orswot()
    for _ in range(rng.randrange(0, 10)):
        a = rng.randrange(n_actors)
        anc.apply_add(anc.clock.inc(a), rng.randrange(members))
    sides = []
    for s in range(2):
        o = anc.clone()
        for _ in range(rng.randrange(0, ops)):
            r = rng.random()
            m = rng.randrange(members)
            a = rng.randrange(n_actors)
            if r < 0.5:
                o.apply_add(o.clock.inc(a), m)
            elif r < 0.8:
                o.apply_rm(o.contains_rm_clock(m), m)
            else:
                c = o.clock.clone()
                c.witness(a, c.get(a) + rng.randrange(1, 4))
                o.apply_rm(c, m)
        sides.append(o)
    return sides


def test_random_differential_python_vs_oracle(oracle):
    rng = random.Random(7)
    L, R = [], []
    for _ in range(300):
        a, b = _random_pair(rng)
        L.append(records.from_py(a, 8))
        R.append(records.from_py(b, 8))
    lb, lo = records.pack_batch(L)
    rb, ro = records.pack_batch(R)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 8, threads=4)
    got = records.unpack_batch(ob, oo)
    rng = random.Random(7)
    for k in range(300):
        a, b = _random_pair(rng)
        a.merge(b)
        assert records.from_py(a, 8) == got[k], k


def test_record_bytes_agree(oracle):
    rng = random.Random(3)
    for _ in range(200):
        args = [rng.randrange(0, 40) for _ in range(6)]
        assert oracle.record_bytes(*args) == records.record_bytes(*args)


# ------------------------------------------------------------ quickcheck_evolution.log
@pytest.mark.parametrize("scn", QC, ids=[s["name"] for s in QC])
def test_quickcheck_evolution_converges(scn, oracle):
    """The 8 op vectors of quickcheck_evolution.log (inputs only): replayed
    onto i = 2..10 witnesses, the reference's convergence property
    (test/orswot.rs:37-76) holds on the Python restatement and the C++ oracle,
    and the two agree record-for-record at every witness count."""
    py, ob = kat_runner.PyBackend(), kat_runner.OracleBackend()
    results = set()
    for i in range(2, 11):
        _, mp = kat_runner.qc_replay(scn, py, i)
        _, mo = kat_runner.qc_replay(scn, ob, i)
        assert records.from_py(mp, 16) == mo.encode(16), f"i={i}"
        results.add(mo.encode(16))
    assert len(results) == 1, f"{scn['name']}: {len(results)} distinct merged states"


@pytest.mark.parametrize("scn", QC, ids=[s["name"] for s in QC])
def test_quickcheck_evolution_witness_sets(scn, oracle):
    """Every witness list the log printed, folded in index order (+ plunger):
    Python restatement == C++ oracle after every merge."""
    for ws in scn["witness_sets"]:
        tp, to = [], []
        kat_runner.qc_fold(ws["witnesses"], kat_runner.PyBackend(), tp)
        kat_runner.qc_fold(ws["witnesses"], kat_runner.OracleBackend(), to)
        for k, (a, b) in enumerate(zip(tp, to)):
            assert records.from_py(a, 16) == b.encode(16), f"log lines {ws['log_lines']} step {k}"
