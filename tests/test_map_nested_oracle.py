"""The nested Map of the reference's own Map tests — TestMap =
Map<u8, Map<u8, MVReg<u8, u8>, u8>, u8> (test/map.rs:4-8) — on the Python
restatement (oracle/crdts_ref.py Map, generic over its values as the
reference's Map<K, V: Val<A>, A> is): the merge KATs of test/map.rs:297-510
transcribed into tests/golden/kat_map.json (test_merge_deferred_remove and the
quickcheck regressions), and the quickcheck properties of test/map.rs:518-740
over op vectors built as build_opvec (test/map.rs:13-46) builds them.

This pins the restatement's Map::merge / apply_rm / truncate (src/map.rs:
131-158, 193-268, 325-350) — the code the GPU Map kernels are checked
against — with the reference's nested-map assertions. A GPU kernel for the
nested map itself is not built."""
import random

import pytest

import map_kat_runner as mkr

CASES = mkr.load_cases(nested=True)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_nested_map_kat(case):
    mkr.run_case(case, mkr.PyMapBackend())


def test_nested_cases_present():
    names = {c["name"] for c in CASES}
    assert {"test_merge_deferred_remove", "test_commute_quickcheck_bug", "test_idempotent_quickcheck_bug1",
            "test_idempotent_quickcheck_bug2", "test_op_exchange_same_as_merge_quickcheck1",
            "test_idempotent_quickcheck1", "test_nop_on_new_map_should_remain_a_new_map"} <= names


def build_opvec(actor, prims):
    """test/map.rs:13-46: op i's clock is Dot {actor, i}.into() (empty for
    i = 0: witness of counter 0), an Up's dot is clock.inc(actor)."""
    ops = []
    for i, (choice, inner_choice, key, inner_key, val) in enumerate(prims):
        clock = [[actor, i]] if i > 0 else []
        dot = [actor, i + 1]
        if choice % 3 == 0:
            if inner_choice % 3 == 0:
                inner = {"up": {"dot": dot, "key": inner_key, "op": {"put": {"clock": clock, "val": val}}}}
            elif inner_choice % 3 == 1:
                inner = {"rm": {"clock": clock, "key": inner_key}}
            else:
                inner = "nop"
            ops.append({"up": {"dot": dot, "key": key, "op": inner}})
        elif choice % 3 == 1:
            ops.append({"rm": {"clock": clock, "key": key}})
        else:
            ops.append("nop")
    return actor, ops


def rand_opvec(rng, actor=None):
    """An arbitrary (u8, Vec<(u8, u8, u8, u8, u8)>) with keys drawn from a
    small range (quickcheck's u8 keys rarely collide; a small range makes the
    removes and concurrent updates meet)."""
    n = rng.randrange(0, 12)
    prims = [(rng.randrange(256), rng.randrange(256), rng.randrange(4), rng.randrange(4), rng.randrange(256))
             for _ in range(n)]
    return build_opvec(rng.randrange(256) if actor is None else actor, prims)


def state(ops):
    m = mkr.nested_map()
    for op in ops:
        mkr.apply_raw(m, op)
    return m


def distinct(rng, k):
    acts = rng.sample(range(256), k)
    return [rand_opvec(rng, a) for a in acts]


N = 400


def test_prop_merge_commutative():  # test/map.rs:674-697
    rng = random.Random(1)
    for _ in range(N):
        (_, o1), (_, o2) = distinct(rng, 2)
        m1, m2 = state(o1), state(o2)
        s1 = m1.clone()
        m1.merge(m2)
        m2.merge(s1)
        assert m1 == m2


def test_prop_merge_associative():  # test/map.rs:646-672
    rng = random.Random(2)
    for _ in range(N):
        (_, o1), (_, o2), (_, o3) = distinct(rng, 3)
        m1, m2, m3 = state(o1), state(o2), state(o3)
        s1 = m1.clone()
        m1.merge(m2)
        m1.merge(m3)
        m2.merge(m3)
        s1.merge(m2)
        assert m1 == s1


def test_prop_merge_idempotent():  # test/map.rs:699-713
    rng = random.Random(3)
    for _ in range(N):
        _, o = rand_opvec(rng)
        m = state(o)
        s = m.clone()
        m.merge(s)
        assert m == s


def test_prop_op_exchange_same_as_merge():  # test/map.rs:520-545
    rng = random.Random(4)
    for _ in range(N):
        (_, o1), (_, o2) = distinct(rng, 2)
        m1, m2 = state(o1), state(o2)
        mm = m1.clone()
        mm.merge(m2)
        for op in o2:
            mkr.apply_raw(m1, op)
        for op in o1:
            mkr.apply_raw(m2, op)
        assert m1 == mm and m2 == mm


def test_prop_op_idempotent_and_exchange_converges():  # test/map.rs:547-569, 601-612
    rng = random.Random(5)
    for _ in range(N):
        (_, o1), (_, o2) = distinct(rng, 2)
        m = state(o1)
        s = m.clone()
        for op in o1:
            mkr.apply_raw(m, op)
        assert m == s
        m1, m2 = state(o1), state(o2)
        for op in o2:
            mkr.apply_raw(m1, op)
        for op in o1:
            mkr.apply_raw(m2, op)
        assert m1 == m2


def test_prop_truncate_with_empty_vclock_is_nop():  # test/map.rs:715-727
    from map_slab import crdts_ref

    rng = random.Random(6)
    for _ in range(N):
        _, o = rand_opvec(rng)
        m = state(o)
        s = m.clone()
        m.truncate(crdts_ref.VClock())
        assert m == s


@pytest.mark.parametrize("A,n", [(16, 250), (100, 60)])
def test_cpp_nested_map_merge_equals_restatement(A, n):
    """The C++ restatement's Map<u64, Map<u64, MVReg>>::merge (oracle/ref_cpu.cpp
    MapT<MapT<MVRegO>>, the CPU baseline of bench.py --workload map_map) equals
    the Python restatement's — the one these KATs pin — on op-simulated pairs,
    both orientations."""
    import random

    import crdts_hip
    import map_slab
    import nested_gen
    import oracle_ffi

    rng = random.Random(A + n)
    pool = list(range(A))
    pairs = [nested_gen.pair(rng, pool) for _ in range(n)]
    caps, inner = dict(kcap=4, dcap=8, scap=4), (4, 8, 8, 4)
    S = crdts_hip.MapMapSlab.alloc(n, A, inner_caps=inner, **caps)
    O = crdts_hip.MapMapSlab.alloc(n, A, inner_caps=inner, **caps)
    for i, (x, y) in enumerate(pairs):
        map_slab.nested_map_to_row(x, S, i, A)
        map_slab.nested_map_to_row(y, O, i, A)
    assert S.inner.a["n_def"].sum() > 0 and S.a["n_def"].sum() > 0
    for X, Y, flip in ((S, O, False), (O, S, True)):
        R = oracle_ffi.map_map_merge(X, Y, A)
        for i, (x, y) in enumerate(pairs):
            a, b = (y, x) if flip else (x, y)
            exp = a.clone()
            exp.merge(b)
            assert map_slab.nested_map_from_row(R, i) == exp, f"pair {i}"
