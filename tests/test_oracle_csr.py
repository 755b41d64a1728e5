"""CPU: the oracle's sparse (CSR) clock merge (oracle/ref_cpu.cpp
orc_vclock_csr_merge: runs -> std::map VClock, VClock::merge src/vclock.rs:131-137)
pinned by the reference's VClock merge KATs (test/vclock.rs:81-116, in
tests/golden/kat_vclock_counters.json) in CSR form, and against an
independent dict restatement of witness (src/vclock.rs:159-163) on random
runs, including empty runs and non-canonical rejection."""
import json
import os

import numpy as np
import pytest

import oracle_ffi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def csr(clocks):
    runs = [sorted(dict(c).items()) for c in clocks]
    ln = np.array([len(r) for r in runs], np.uint32)
    off = np.zeros(len(runs), np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    act = np.array([a for r in runs for a, _ in r] or [0], np.uint32)
    ctr = np.array([c for r in runs for _, c in r] or [1], np.uint64)
    return off, ln, act, ctr


def unpack(res):
    off, ln, act, ctr = res
    return [list(zip(act[o:o + n].tolist(), ctr[o:o + n].tolist())) for o, n in zip(off.tolist(), ln.tolist())]


def dict_merge(a, b):  # VClock::merge = witness every (actor, counter) of b
    r = dict(a)
    for x, c in b.items():
        if not r.get(x, 0) >= c:
            r[x] = c
    return sorted(r.items())


def witnessed(pairs):
    """The clock From<Vec<(A, u64)>> builds (src/vclock.rs:267-271): witness each pair."""
    c = {}
    for x, v in pairs:
        if not c.get(x, 0) >= v:
            c[x] = v
    return c


def test_reference_merge_kats_in_csr_form():
    kats = [k for k in json.load(open(os.path.join(GOLDEN, "kat_vclock_counters.json")))["vclock_binop"]
            if k["op"] == "merge"]
    assert len(kats) >= 3
    got = unpack(oracle_ffi.vclock_csr_merge(csr([witnessed(k["a"]) for k in kats]),
                                             csr([witnessed(k["b"]) for k in kats])))
    for k, g in zip(kats, got):
        assert g == [tuple(x) for x in k["expect"]], k["name"]


def test_random_runs_vs_dict_restatement():
    import crdts_hip

    s, o = crdts_hip.generate_clocks_csr(3000, seed=5)
    got = unpack(oracle_ffi.vclock_csr_merge(s, o))
    S = [dict(c) for c in unpack((s[0], s[1], s[2], s[3]))]
    O = [dict(c) for c in unpack((o[0], o[1], o[2], o[3]))]
    assert got == [dict_merge(a, b) for a, b in zip(S, O)]
    assert max(len(c) for c in S) <= 56 and np.mean([len(c) for c in S]) > 40


def test_empty_and_long_runs():
    rng = np.random.default_rng(3)
    A = [{}, {5: 1}, {}, {int(x): int(rng.integers(1, 9)) for x in rng.choice(5000, 700, replace=False)}]
    B = [{}, {}, {7: 2}, {int(x): int(rng.integers(1, 9)) for x in rng.choice(5000, 900, replace=False)}]
    got = unpack(oracle_ffi.vclock_csr_merge(csr(A), csr(B)))
    assert got == [dict_merge(a, b) for a, b in zip(A, B)]


@pytest.mark.parametrize("bad", ["zero", "unsorted"])
def test_noncanonical_runs_rejected(bad):
    off, ln, act, ctr = csr([{1: 1, 2: 2, 3: 3}])
    if bad == "zero":
        ctr[1] = 0
    else:
        act[[0, 1]] = act[[1, 0]]
    with pytest.raises(ValueError):
        oracle_ffi.vclock_csr_merge((off, ln, act, ctr), csr([{}]))
