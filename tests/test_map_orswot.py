"""Map<u64, Orswot<u64, A>, A>::merge and Orswot::truncate (SURVEY.md §8(f)
rank 3 as written; src/map.rs:192-269, src/orswot.rs:159-172) — CPU side.

- The reference's Map KATs (tests/golden/kat_map.json: test/orswot.rs:270-307
  test_reset_remove_semantics; test/map.rs:226-295, the Map<u8, MVReg> op-path
  KATs that pin the op semantics of the oracle's Map generators) pass on the
  pure-Python restatement and on the C++ oracle's own op path, which agree
  state-for-state.
- The two restatements agree on generated replica pairs (C++ generator: the
  reference's update / rm contexts, out-of-order delivery, removes carrying a
  third replica's clock at the map and at the nested set).
- Orswot::truncate never leaves an empty member clock on reachable states.
- The order question: Map::apply_deferred iterates a HashMap (src/map.rs:
  325-333); with Orswot values two deferred clocks naming one key truncate its
  set in sequence, and that order CAN change the result — settled by
  enumerating every order in the oracle on a reachable pair built by the op
  path. The product applies CLOCK ORDER, one of the orders the reference can
  take; generated pairs are enumerated too and the GPU tests check the
  product against the CLOCK ORDER oracle.
"""
import random

import numpy as np
import pytest

import map_kat_runner as mkr
import map_slab
import opgen
from map_slab import crdts_ref

CASES = mkr.load_cases()
A = 8


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_map_kat_python(case):
    mkr.run_case(case, mkr.PyMapBackend())


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_map_kat_oracle_matches_python(case, oracle):
    tp, to = [], []
    a = mkr.run_case(case, mkr.PyMapBackend(), tp)
    b = mkr.run_case(case, mkr.OracleMapBackend(), to)
    assert a.keys() == b.keys() and all(a[k] == b[k] for k in a)
    assert [(k, n) for k, n, _ in tp] == [(k, n) for k, n, _ in to]
    assert all(x == y for (_, _, x), (_, _, y) in zip(tp, to))


@pytest.mark.parametrize("pct_future", [10, 35])
def test_map_orswot_python_matches_oracle(oracle, pct_future):
    """Generated pairs, both orientations: Python restatement == C++ oracle, slab-row exact."""
    L, R = oracle.map_orswot_generate(0xA11CE + pct_future, 300, A, keys=4, members=6, ops=10,
                                      pct_future=pct_future)
    assert L.a["n_keys"].sum() > 300 and L.a["vn_def"].sum() > 20 and L.a["n_def"].sum() > 20
    for S, O in ((L, R), (R, L)):
        out = oracle.map_orswot_merge(S, O, A)
        import crdts_hip

        T = crdts_hip.MapOrswotSlab.alloc(S.n, A, **out.caps)
        for i in range(S.n):
            m = map_slab.orswot_map_from_row(S, i)
            m.merge(map_slab.orswot_map_from_row(O, i))
            map_slab.orswot_map_to_row(m, T, i, A)
            assert map_slab.rows_equal(T, i, out, i), i


def test_merged_maps_hold_no_empty_member_clock(oracle):
    """Orswot::truncate leaves a member whose clock it empties (src/orswot.rs:
    168-170 subtracts without a check), but on reachable states a member
    surviving the preceding merge with the empty set has an actor above the
    truncating clock, so none is ever emptied: checked over merged outputs."""
    L, R = oracle.map_orswot_generate(0xE3, 500, A, keys=4, members=6, ops=12, pct_future=30)
    out = oracle.map_orswot_merge(L, R, A)
    a = out.a
    for i in range(out.n):
        for k in range(int(a["n_keys"][i])):
            for j in range(int(a["vn_mem"][i, k])):
                assert a["vmclock"][i, k, j].any(), (i, k, j)


@pytest.mark.parametrize("seed", range(20))
def test_truncate_of_reachable_sets_keeps_member_clocks(seed):
    """Random reachable Orswots (op vectors of quickcheck's shape) truncated by
    random clocks: every surviving member keeps a non-empty clock."""
    rng = random.Random(seed)
    be = __import__("kat_runner").PyBackend()
    for _ in range(20):
        o = be.new()
        for actor, op in opgen.orswot_opvec(rng, max_len=30, size=8):
            opgen.apply_op(be, o, op)
        t = crdts_ref.VClock([(rng.randrange(8), rng.randrange(1, 6)) for _ in range(rng.randrange(0, 4))])
        o.truncate(t)
        assert all(not c.is_empty() for c in o.entries.values())


def _order_case():
    """A reachable pair where the final apply_deferred's order changes the
    result (actors x=0, y=1, w=2): replica a updates key 7 three times
    (nested adds by x: nested clock {x:3}), then removes member 2 inside it
    with the clock {x:2, y:1} (deferred in the nested set); replica b has only
    received two removes of key 7 carrying a third replica's clocks
    {x:3, w:5} and {y:1, w:6} (deferred in b's map)."""
    a = crdts_ref.Map(crdts_ref.Orswot)
    for _ in range(3):
        add, _, _ = a.get(7)
        dot = (0, add.get(0) + 1)
        a.apply_up(dot, 7, lambda s, d=dot: s.apply_add(d, 1))
    add, _, _ = a.get(7)
    dot = (0, add.get(0) + 1)
    a.apply_up(dot, 7, lambda s: s.apply_rm(crdts_ref.VClock([(0, 2), (1, 1)]), 2))
    b = crdts_ref.Map(crdts_ref.Orswot)
    b.apply_rm(7, crdts_ref.VClock([(0, 3), (2, 5)]))
    b.apply_rm(7, crdts_ref.VClock([(1, 1), (2, 6)]))
    return a, b


def test_deferred_order_can_change_the_result(oracle):
    import crdts_hip

    a, b = _order_case()
    results = []
    for order in (crdts_ref.clock_order, lambda cs: crdts_ref.clock_order(cs)[::-1]):
        m = a.clone()
        m.order = order
        m.merge(b)
        results.append(m)
    assert results[0] != results[1]
    # CLOCK ORDER keeps the nested deferred remove; the other order drops it
    assert len(results[0].entries[7][1].deferred) == 1 and len(results[1].entries[7][1].deferred) == 0
    # the oracle, enumerating every order of the final apply_deferred: two outcomes
    S = crdts_hip.MapOrswotSlab.alloc(1, A, **oracle.MAP_ORSWOT_CAPS)
    O = crdts_hip.MapOrswotSlab.alloc(1, A, **oracle.MAP_ORSWOT_CAPS)
    map_slab.orswot_map_to_row(a, S, 0, A)
    map_slab.orswot_map_to_row(b, O, 0, A)
    assert oracle.map_orswot_order_outcomes(S, O, A).tolist() == [2]
    out = oracle.map_orswot_merge(S, O, A)
    assert map_slab.orswot_map_from_row(out, 0) == results[0]


def test_deferred_order_on_generated_pairs(oracle):
    """Enumeration over generated pairs: every object's outcome count is
    recorded (most have one; the CLOCK ORDER result is always one of them)."""
    L, R = oracle.map_orswot_generate(0x0DE5, 400, A, keys=3, members=4, ops=12, pct_future=40)
    oc = oracle.map_orswot_order_outcomes(L, R, A, max_k=6)
    assert (oc != 0).all()
    assert (oc >= 1).mean() > 0.95
