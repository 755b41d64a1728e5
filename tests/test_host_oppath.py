"""CPU: the product's host op path and generators against the oracle.

- crdt_host_orswot_* (Orswot::apply, src/orswot.rs:61-85) builds states that
  are record-identical to the oracle's apply on the same op streams;
- the config-3 generator is deterministic, sharding-invariant, produces
  canonical records, and has the SURVEY.md §8(d) shape;
- the record codecs (product Python, tests, oracle) agree.
"""
import random

import numpy as np
import pytest

import crdts_hip
import opgen
import records


def _apply_both(ops, n_actors):
    h = crdts_hip.HostOrswot()
    import oracle_ffi

    o = oracle_ffi.OracleOrswot()
    for _, op in ops:
        if op[0] == "add":
            h.apply_add(op[1], op[2], op[3])
            o.apply_add(op[1], op[2], op[3])
        else:
            h.apply_rm(op[1], op[2])
            o.apply_rm(op[1], op[2])
    return h, o


@pytest.mark.parametrize("seed", range(60))
def test_host_oppath_matches_oracle(seed, oracle):
    rng = random.Random(seed)
    ops = opgen.orswot_opvec(rng, max_len=60, size=100, actor_range=24, member_range=16)
    h, o = _apply_both(ops, 24)
    assert h.encode(24) == o.encode(24)


def test_host_decode_encode_roundtrip(oracle):
    rng = random.Random(5)
    for _ in range(50):
        ops = opgen.orswot_opvec(rng, max_len=50, actor_range=10, member_range=10)
        h, _ = _apply_both(ops, 10)
        rec = h.encode(10)
        assert crdts_hip.HostOrswot.decode(rec).encode(10) == rec
        assert oracle.OracleOrswot.decode(rec).encode(10) == rec
        d = crdts_hip.decode_record(rec)
        assert crdts_hip.encode_record(d["clock"], {m: dict(r) for m, r in d["entries"].items()},
                                       {tuple(k): v for k, v in d["deferred"]}, 10) == rec
        assert records.decode(rec)["entries"] == d["entries"]


def test_encode_rejects_actor_out_of_range():
    h = crdts_hip.HostOrswot()
    h.apply_add(20, 1, 7)
    with pytest.raises(crdts_hip.CrdtError):
        h.encode(16)


def _check_canonical(rec, n_actors):
    d = records.decode(rec)
    assert d["size"] == len(rec) and d["flags"] == 0
    keys = list(d["entries"])
    assert keys == sorted(set(keys))
    for m, run in d["entries"].items():
        assert run and all(c > 0 and a < n_actors for a, c in run)
        assert [a for a, _ in run] == sorted({a for a, _ in run})
    clocks = [tuple(c) for c, _ in d["deferred"]]
    assert clocks == sorted(set(clocks))
    for c, ms in d["deferred"]:
        assert c and ms and ms == sorted(set(ms))


def test_generator_deterministic_and_shard_invariant():
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(200, first_obj=0, threads=4)
    (lb2, lo2), (rb2, ro2) = crdts_hip.generate_orswot(200, first_obj=0, threads=1)
    assert records.unpack_batch(lb, lo) == records.unpack_batch(lb2, lo2)
    (lb3, lo3), (rb3, ro3) = crdts_hip.generate_orswot(80, first_obj=120, threads=3)
    assert records.unpack_batch(lb, lo)[120:] == records.unpack_batch(lb3, lo3)
    assert records.unpack_batch(rb, ro)[120:] == records.unpack_batch(rb3, ro3)


def test_generator_canonical_and_config3_shape():
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(3000, threads=8)
    recs = records.unpack_batch(lb, lo) + records.unpack_batch(rb, ro)
    for r in recs[:400]:
        _check_canonical(r, 16)
    dec = [records.decode(r) for r in recs]
    mem = np.array([len(d["entries"]) for d in dec])
    dots = np.array([sum(len(v) for v in d["entries"].values()) for d in dec])
    has_def = np.array([len(d["deferred"]) > 0 for d in dec])
    assert 24 <= mem.mean() <= 36, mem.mean()  # "~32 members" per side
    assert 1.0 <= dots.mean() / mem.mean() <= 2.5
    assert 0.01 <= has_def.mean() <= 0.10, has_def.mean()  # deferred in a few % of records
    sizes = np.array([len(r) for r in recs])
    assert 800 <= sizes.mean() <= 1600 and sizes.max() <= 2048


def test_generator_oracle_merge_runs(oracle):
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(500, threads=4)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 16, threads=4)
    outs = records.unpack_batch(ob, oo)
    for r in outs[:200]:
        _check_canonical(r, 16)


def test_dense_generator():
    a = crdts_hip.generate_dense(1000, 64, seed=0xC0FFEE02)
    b = crdts_hip.generate_dense(1000, 64, seed=0xC0FFEE02)
    assert (a == b).all()
    z = (a == 0).mean()
    assert 0.2 < z < 0.3
    assert a.max() < (1 << 40)
    c = crdts_hip.generate_dense(500, 64, seed=0xC0FFEE02, first_obj=500)
    assert (a[500:] == c).all()
