"""GPU: objects past the LDS tiers of every kernel on the path — 1 000+
members and 100+ deferred clocks per object — through ingest (from_binary,
src/lib.rs:78-83) -> merge (src/orswot.rs:87-157) -> apply (:61-85) -> egest
(to_binary, :62-64), byte-exact against the oracle at every step, mixed into
batches of ordinary config-3 objects (so the large-object kernels run beside
the fast paths, on the objects those list for them)."""
import random

import numpy as np
import pytest

import bincode_ref as BC
import records
from test_gpu_apply import _ops_for
from test_gpu_bincode import _blobs_of, _rec, _state, _upload_blobs

pytestmark = pytest.mark.gpu
A = 16


def big_state(oracle, rng, n_mem=1300, n_def=100, actors=range(8)):
    """An Orswot built by the reference's op path: n_mem members added by
    `actors`, some removed with read contexts, and n_def removes with FUTURE
    contexts (distinct clocks, each !(D <= clock)) that stay deferred."""
    o = oracle.OracleOrswot()
    clock = {}
    keys = rng.sample(range(1, 1 << 40), n_mem + 50)
    for m in keys[:n_mem]:
        a = rng.choice(list(actors))
        clock[a] = clock.get(a, 0) + 1
        o.apply_add(a, clock[a], m)
        if rng.random() < 0.3:  # a second dot on the member
            b = rng.choice(list(actors))
            clock[b] = clock.get(b, 0) + 1
            o.apply_add(b, clock[b], m)
    for m in rng.sample(keys[:n_mem], 20):  # read-context removes
        o.apply_rm(m, sorted(dict(o.entry(m)).items()) if hasattr(o, "entry") else [])
    for k in range(n_def):  # future-context removes: actor 15's counter ahead of the clock
        ctx = dict(clock)
        ctx[15] = 1000 + k
        for m in rng.sample(keys, rng.randrange(1, 4)):
            o.apply_rm(m, sorted(ctx.items()))
    return o


def _batch(oracle, seed, n_big=3):
    import crdts_hip

    rng = random.Random(seed)
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(2_000, threads=8, seed=seed)
    L, R = records.unpack_batch(lb, lo), records.unpack_batch(rb, ro)
    at = [17, 500, 1999][:n_big]
    for i in at:
        L[i] = big_state(oracle, rng).encode(A)
        R[i] = big_state(oracle, rng, n_mem=1500, n_def=110, actors=range(4, 12)).encode(A)
    return L, R, at


def test_big_objects_ingest_merge_apply_egest(gpu, oracle):
    import crdts_hip

    L, R, at = _batch(oracle, 3)
    for i in at:
        d = records.decode(L[i])
        assert len(d["entries"]) >= 1000 and len(d["deferred"]) >= 100
    # ingest: blobs in arbitrary HashMap order -> canonical records (packed and bound-placed)
    rng = random.Random(5)
    blobs = [BC.encode(_state(records.decode(r)), 1, 8, rng=rng) for r in L]
    t, bo, bl = _upload_blobs(blobs, rng)
    assert gpu.orswot_from_bincode(t, bo, bl, A, 1, 8).records() == L
    gapped = gpu.orswot_from_bincode(t, bo, bl, A, 1, 8, packed=False)
    assert gapped.records() == L
    # merge: the big pairs through the general kernel's HBM path
    LB = crdts_hip.OrswotBatch.from_records(L, A)
    RB = crdts_hip.OrswotBatch.from_records(R, A)
    merged = gpu.orswot_merge(LB, RB).records()
    lb, lo = records.pack_batch(L)
    rb, ro = records.pack_batch(R)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, A, threads=16)
    assert merged == records.unpack_batch(ob, oo)
    # apply: ops on the merged states (the big ones past both LDS workspaces)
    prng = random.Random(7)
    sts = [records.decode(r) for r in merged]
    per = [_ops_for(s, A, prng, 40 if i in at else prng.randrange(6)) for i, s in enumerate(sts)]
    applied = gpu.orswot_apply(crdts_hip.OrswotBatch.from_records(merged, A), crdts_hip.OrswotOps.from_lists(per))
    got = applied.records()
    for i, (r, ops) in enumerate(zip(merged, per)):
        o = oracle.OracleOrswot.decode(r)
        for op in ops:
            if op[0] == "add":
                o.apply_add(op[1], op[2], op[3])
            else:
                o.apply_rm(op[1], op[2])
        assert got[i] == o.encode(A), f"apply object {i}{' (big)' if i in at else ''}"
    # egest: records -> the reference's binary form
    out_blobs = _blobs_of(*gpu.orswot_to_bincode(crdts_hip.OrswotBatch.from_records(got, A), 1, 8))
    assert out_blobs == [BC.encode(_state(records.decode(r)), 1, 8) for r in got]


def test_apply_past_both_lds_workspaces(gpu, oracle):
    """Member clocks longer than 128 entries (a 300-actor dense clock) and
    300+ deferred clocks need the HBM workspace."""
    import crdts_hip

    AA = 300
    o = oracle.OracleOrswot()
    for a in range(AA):
        o.apply_add(a, 1, 42)  # one member whose clock has 300 entries
    for m in range(1, 200):
        o.apply_add(m % AA, 2, m)
    for k in range(120):
        o.apply_rm(7 + k, [(AA - 1, 10 + k)])  # future contexts: 120 deferred clocks
    rec = o.encode(AA)
    ops = [[("rm", 42, [(a, 1) for a in range(0, AA, 2)]), ("add", 5, 3, 42), ("add", 299, 200, 9)]]
    got = gpu.orswot_apply(crdts_hip.OrswotBatch.from_records([rec], AA), crdts_hip.OrswotOps.from_lists(ops))
    exp = oracle.OracleOrswot.decode(rec)
    exp.apply_rm(42, [(a, 1) for a in range(0, AA, 2)])
    exp.apply_add(5, 3, 42)
    exp.apply_add(299, 200, 9)
    assert got.records() == [exp.encode(AA)]
