"""GPU parity of the batched op path (crdt_orswot_apply: CmRDT::apply for
Orswot, src/orswot.rs:61-85, with apply_remove :195-211 and apply_deferred
:235-243) against the C++ oracle's op path, byte-exact
on the canonical records: fresh and stale adds, removes with a read context,
removes with a future context (deferred), adds that later release deferred
removes, new members and actors, dense (config 3) and sparse (config 5)
records, malformed ops."""
import random

import numpy as np
import pytest

import records

pytestmark = pytest.mark.gpu


def _ops_for(st, A, rng, n_ops):
    clock = dict(st["clock"])
    keys = list(st["entries"])
    ops = []
    for _ in range(n_ops):
        r = rng.random()
        a = rng.randrange(A) if A <= 64 else rng.choice(list(clock) + [rng.randrange(A)])
        if r < 0.45:  # fresh add (existing or new member)
            c = clock.get(a, 0) + 1 + rng.randrange(2)
            m = rng.choice(keys) if keys and rng.random() < 0.6 else rng.getrandbits(64)
            ops.append(("add", a, c, m))
            clock[a] = max(clock.get(a, 0), c)
            keys.append(m)
        elif r < 0.55:  # stale add: already seen
            if clock:
                x = rng.choice(list(clock))
                ops.append(("add", x, rng.randrange(1, clock[x] + 1), rng.choice(keys) if keys else 7))
        elif r < 0.75 and keys:  # remove with a read context (the member's clock, or the top clock)
            m = rng.choice(keys)
            ctx = st["entries"].get(m) or sorted(clock.items())
            ops.append(("rm", m, sorted(ctx)))
        else:  # remove with a future context -> deferred (maybe released by later adds)
            m = rng.choice(keys) if keys and rng.random() < 0.7 else rng.getrandbits(64)
            fut = sorted(clock.items())
            if fut and rng.random() < 0.8:
                i = rng.randrange(len(fut))
                fut[i] = (fut[i][0], fut[i][1] + 1 + rng.randrange(2))
            else:
                fut = sorted(set(fut) | {(a, clock.get(a, 0) + 1)})
                fut = sorted(dict(fut).items())
            ops.append(("rm", m, fut))
    return ops


def _oracle_apply(oracle, rec, ops, A, flags):
    o = oracle.OracleOrswot.decode(rec)
    for op in ops:
        if op[0] == "add":
            o.apply_add(op[1], op[2], op[3])
        else:
            o.apply_rm(op[1], op[2])
    return o.encode(A, flags)


def _run(gpu, oracle, recs, A, flags, seed, max_ops=8):
    import crdts_hip

    rng = random.Random(seed)
    sts = [records.decode(r) for r in recs]
    per = [_ops_for(s, A, rng, rng.randrange(max_ops + 1)) for s in sts]
    B = crdts_hip.OrswotBatch.from_records(recs, A, flags=flags)
    ops = crdts_hip.OrswotOps.from_lists(per)
    out = gpu.orswot_apply(B, ops).records()
    exp = [_oracle_apply(oracle, r, o, A, flags) for r, o in zip(recs, per)]
    bad = [i for i, (g, e) in enumerate(zip(out, exp)) if g != e]
    assert not bad, (f"{len(bad)} / {len(exp)} differ; first {bad[0]} ops {per[bad[0]]}:\n"
                     f"gpu    {records.decode(out[bad[0]])}\noracle {records.decode(exp[bad[0]])}")
    return per, out


def test_apply_config3(gpu, oracle):
    import crdts_hip

    (b, o), _ = crdts_hip.generate_orswot(4_000, first_obj=17, threads=16)
    per, _ = _run(gpu, oracle, records.unpack_batch(b, o), 16, 0, seed=1)
    assert sum(len(p) for p in per) > 10_000


def test_apply_config3_deferred_heavy(gpu, oracle):
    """Objects that already hold deferred removes, long op lists."""
    import crdts_hip

    (b, o), _ = crdts_hip.generate_orswot(6_000, first_obj=3, threads=16)
    recs = [r for r in records.unpack_batch(b, o) if records.decode(r)["deferred"]]
    assert len(recs) > 100
    _, out = _run(gpu, oracle, recs, 16, 0, seed=2, max_ops=24)
    nd = [(len(records.decode(r)["deferred"]), len(records.decode(x)["deferred"])) for r, x in zip(recs, out)]
    assert sum(b < a for a, b in nd) > 5  # deferred removes released by later adds (apply_deferred)
    assert sum(b > a for a, b in nd) > 20  # new deferred removes


def test_apply_from_empty(gpu, oracle):
    empty = records.encode({}, {}, {}, 16)
    _run(gpu, oracle, [empty] * 500, 16, 0, seed=3, max_ops=12)


def test_apply_sparse_config5(gpu, oracle):
    import crdts_hip

    b, o = crdts_hip.generate_replicas(2_000, 2, first_obj=5, threads=16)[0]
    _run(gpu, oracle, records.unpack_batch(b, o), 1024, crdts_hip.SPARSE_CLOCK, seed=4)


def test_apply_no_ops_is_identity(gpu):
    import crdts_hip

    (b, o), _ = crdts_hip.generate_orswot(2_000, threads=16)
    recs = records.unpack_batch(b, o)
    B = crdts_hip.OrswotBatch.from_records(recs, 16)
    out = gpu.orswot_apply(B, crdts_hip.OrswotOps.from_lists([[] for _ in recs])).records()
    assert out == recs


def test_apply_malformed_ops(gpu):
    import crdts_hip
    from crdts_hip._lib import CrdtError

    rec = records.encode({1: 2}, {5: {1: 2}}, {}, 16)
    B = crdts_hip.OrswotBatch.from_records([rec], 16)
    for bad in ([("add", 99, 1, 5)],                      # actor >= n_actors
                [("rm", 5, [(2, 1), (1, 1)])],            # clock actors out of order
                [("rm", 5, [(1, 0)])]):                   # zero counter in a clock
        with pytest.raises(CrdtError):
            gpu.orswot_apply(B, crdts_hip.OrswotOps.from_lists([bad]))


def _record(rng, A, n_mem, n_def=0, sparse=False):
    """A canonical record with n_mem members (1-3 dots each, under the clock)
    and n_def deferred removes with future clocks."""
    acts = rng.sample(range(A), min(A, 24))
    clock = {a: rng.randrange(3, 40) for a in acts}
    entries = {}
    for _ in range(n_mem):
        dots = {a: rng.randrange(1, clock[a] + 1) for a in rng.sample(acts, rng.randrange(1, 4))}
        entries[rng.getrandbits(64)] = dots
    deferred = {}
    for _ in range(n_def):
        a = rng.choice(acts)
        deferred[((a, clock[a] + 1 + rng.randrange(3)),)] = {rng.getrandbits(64) for _ in range(rng.randrange(1, 4))}
    return records.encode(clock, entries, deferred, A, sparse=sparse)


def test_apply_workspace_tiers(gpu, oracle):
    """Objects that fit the small workspace, objects that start beyond it
    (65..128 members, > 256 dots, > 16 deferred clocks) and objects that outgrow
    it part way through their ops, mixed in one batch: the ones that do not fit
    are redone from their input in the large workspace."""
    rng = random.Random(11)
    recs = []
    for i in range(600):
        k = i % 4
        n_mem = [rng.randrange(0, 40), rng.randrange(65, 120), rng.randrange(58, 64), rng.randrange(20, 40)][k]
        n_def = [rng.randrange(0, 3), rng.randrange(0, 3), 0, rng.randrange(17, 24)][k]
        recs.append(_record(rng, 16, n_mem, n_def))
    _run(gpu, oracle, recs, 16, 0, seed=12, max_ops=16)


def test_apply_workspace_tiers_sparse(gpu, oracle):
    rng = random.Random(13)
    recs = [_record(rng, 1024, rng.choice([10, 62, 90]), rng.randrange(0, 3), sparse=True) for _ in range(400)]
    _run(gpu, oracle, recs, 1024, crdts_hip_sparse(), seed=14, max_ops=12)


def crdts_hip_sparse():
    import crdts_hip

    return crdts_hip.SPARSE_CLOCK


def test_apply_list_overflow(gpu, oracle):
    """More large-workspace objects than the context's object list holds:
    the large pass finds them by their out_off flag instead."""
    rng = random.Random(15)
    recs = [_record(rng, 16, rng.choice([20, 80]), 1) for _ in range(300)]
    gpu.set_list_cap(8)
    try:
        _run(gpu, oracle, recs, 16, 0, seed=16, max_ops=6)
    finally:
        gpu.set_list_cap(65536)


def test_apply_dense_wide_clock(gpu, oracle):
    """n_actors beyond the small workspace's dense clock: every object goes
    straight to the large one."""
    rng = random.Random(17)
    recs = [_record(rng, 100, rng.randrange(0, 50), rng.randrange(0, 3)) for _ in range(300)]
    _run(gpu, oracle, recs, 100, 0, seed=18, max_ops=8)


def test_apply_sparse_growth_fresh_actors(gpu, oracle):
    """Sparse records growing by the most an Add can add (a new top-clock
    actor, a new member and its dot: 36 B): 9..16 such Adds on empty sparse
    records, other objects after each in the batch. Every output must equal
    the oracle's, so none overwrote its neighbour (the per-op reservation of
    the CSR form, include/crdts_hip.h)."""
    import crdts_hip

    rng = random.Random(19)
    empty = records.encode({}, {}, {}, 1024, sparse=True)
    recs, per = [], []
    for i in range(300):
        if i % 2 == 0:
            n = 9 + rng.randrange(8)
            acts = rng.sample(range(1024), n)
            per.append([("add", a, 1 + rng.randrange(5), rng.getrandbits(64)) for a in acts])
            recs.append(empty)
        else:
            recs.append(_record(rng, 1024, rng.randrange(1, 20), rng.randrange(0, 2), sparse=True))
            per.append([])
    B = crdts_hip.OrswotBatch.from_records(recs, 1024, flags=crdts_hip.SPARSE_CLOCK)
    out = gpu.orswot_apply(B, crdts_hip.OrswotOps.from_lists(per)).records()
    exp = [_oracle_apply(oracle, r, o, 1024, crdts_hip.SPARSE_CLOCK) for r, o in zip(recs, per)]
    assert out == exp
