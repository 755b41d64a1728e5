"""CPU: the CSR (sparse) top-clock record form — SURVEY.md §8(a) A2, config 5.

The sparse form changes only how the top clock is laid out (include/crdts_hip.h,
header flags bit 0), so it is pinned to the dense form, which the reference's
KATs pin (tests/test_oracle_kat.py):
- three independent codecs (product host C++, oracle C++, tests/records.py)
  produce byte-identical sparse records and decode them to the same state;
- the oracle's merge over sparse records gives, for every object, the same
  state as its merge over the dense records of the same states;
- the config-5 replica generator is deterministic, shard-invariant and
  canonical, with the SURVEY.md §8(d) shape (1024-actor universe).
"""
import random

import numpy as np
import pytest

import crdts_hip
import opgen
import records

SPARSE = 1


def _state(rec):
    d = records.decode(rec)
    return d["clock"], d["entries"], d["deferred"]


def _apply_both(ops):
    import oracle_ffi

    h, o = crdts_hip.HostOrswot(), oracle_ffi.OracleOrswot()
    for _, op in ops:
        if op[0] == "add":
            h.apply_add(op[1], op[2], op[3])
            o.apply_add(op[1], op[2], op[3])
        else:
            h.apply_rm(op[1], op[2])
            o.apply_rm(op[1], op[2])
    return h, o


@pytest.mark.parametrize("seed", range(40))
def test_sparse_codecs_agree(seed, oracle):
    rng = random.Random(1000 + seed)
    ops = opgen.orswot_opvec(rng, max_len=60, size=100, actor_range=48, member_range=16)
    h, o = _apply_both(ops)
    sp = h.encode(48, SPARSE)
    assert sp == o.encode(48, SPARSE)
    d = records.decode(sp)
    assert d["flags"] == SPARSE
    # same state as the dense form, and the test codec re-encodes it byte-exactly
    assert _state(sp) == _state(h.encode(48))
    ents = {m: dict(r) for m, r in d["entries"].items()}
    defs = {tuple(k): set(v) for k, v in d["deferred"]}
    assert records.encode(d["clock"], ents, defs, 48, sparse=True) == sp
    # the product's Python codec reads it too
    pd = crdts_hip.decode_record(sp)
    assert pd["clock"] == d["clock"] and pd["entries"] == d["entries"]
    # host decode -> encode round trip in both forms
    h2 = crdts_hip.HostOrswot.decode(sp)
    assert h2.encode(48, SPARSE) == sp and h2.encode(48) == h.encode(48)


def test_sparse_record_bytes():
    assert records.record_bytes(3, 1, 1, 0, 0, 0, sparse=True) == 32 + 40 + 24 == 96
    assert crdts_hip.lib.crdt_orswot_record_bytes_ex(3, 1, 1, 0, 0, 0, SPARSE) == 96
    assert crdts_hip.lib.crdt_orswot_record_bytes_ex(0, 0, 0, 0, 0, 0, SPARSE) == 32
    assert crdts_hip.lib.crdt_orswot_record_bytes_ex(5, 2, 3, 1, 2, 2, 0) == \
        crdts_hip.lib.crdt_orswot_record_bytes(5, 2, 3, 1, 2, 2)


def test_oracle_sparse_merge_matches_dense(oracle):
    """Same states, both forms: merged states agree object by object."""
    rng = random.Random(5)
    A = 40
    Ls, Rs = [], []
    for _ in range(400):
        for side in (Ls, Rs):
            h, _ = _apply_both(opgen.orswot_opvec(rng, max_len=40, size=100, actor_range=A, member_range=12))
            side.append(h)
    for (la, ra) in ((Ls, Rs), (Rs, Ls)):  # both orientations
        dl, do = records.pack_batch([x.encode(A) for x in la])
        dr, dro = records.pack_batch([x.encode(A) for x in ra])
        sl, so = records.pack_batch([x.encode(A, SPARSE) for x in la])
        sr, sro = records.pack_batch([x.encode(A, SPARSE) for x in ra])
        ob, oo = oracle.orswot_merge_batch(dl, do, dr, dro, A)
        sb, soo = oracle.orswot_merge_batch(sl, so, sr, sro, A, flags=SPARSE)
        dense = records.unpack_batch(ob, oo)
        sparse = records.unpack_batch(sb, soo)
        for d, s in zip(dense, sparse):
            assert records.decode(s)["flags"] == SPARSE
            assert _state(d) == _state(s)


def test_replica_generator_config5_shape():
    reps = crdts_hip.generate_replicas(3000, 8, threads=4)
    assert len(reps) == 8
    a = crdts_hip.generate_replicas(200, 8, first_obj=1000, threads=3)
    for r in range(8):  # sharding-invariant: object i depends on i only
        b, o = reps[r]
        x = records.unpack_batch(b, o)[1000:1200]
        assert x == records.unpack_batch(*a[r])
    nnz, sizes = [], []
    for b, o in reps:
        for rec in records.unpack_batch(b, o)[:300]:
            d = records.decode(rec)
            assert d["flags"] == SPARSE
            assert all(0 <= x < 1024 for x in d["clock"])
            nnz.append(len(d["clock"]))
            sizes.append(d["size"])
    assert 20 <= np.mean(nnz) <= 48
    assert 1000 <= np.mean(sizes) <= 2500


def test_replica_fold_oracle_converges(oracle):
    """Anti-entropy: every rank folds the replicas in rank order; the result
    is the same bytes whichever fold is used as long as the order is fixed,
    and every replica ⊔ fold(all) == fold(all) in value."""
    reps = crdts_hip.generate_replicas(500, 4, threads=4)
    acc = reps[0]
    for r in range(1, 4):
        acc = oracle.orswot_merge_batch(acc[0], acc[1], reps[r][0], reps[r][1], 1024, flags=SPARSE)
    fold = records.unpack_batch(*acc)
    assert all(records.decode(x)["flags"] == SPARSE for x in fold)
    # idempotence: fold ⊔ fold == fold
    again = oracle.orswot_merge_batch(acc[0], acc[1], acc[0], acc[1], 1024, flags=SPARSE)
    assert records.unpack_batch(*again) == fold
