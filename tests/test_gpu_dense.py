"""GPU parity: dense VClock / GCounter / PNCounter join vs the oracle (bit-exact)."""
import json
import os
import random

import numpy as np
import pytest

import opgen

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to("cuda:0")


def _host(t):
    return t.cpu().numpy().view(np.uint64)


def test_vclock_merge_kats_on_gpu(gpu):
    import crdts_hip

    kats = json.load(open(os.path.join(GOLDEN, "kat_vclock_counters.json")))["vclock_binop"]
    for k in [k for k in kats if k["op"] == "merge"]:
        a = crdts_hip.VClock(k["a"], n_actors=8)
        b = crdts_hip.VClock(k["b"], n_actors=8)
        a.merge(b, engine=gpu)
        assert sorted(a.dots.items()) == [tuple(x) for x in k["expect"]], k["name"]


@pytest.mark.parametrize("n_actors", [1, 3, 16, 64, 100])
@pytest.mark.parametrize("kind", ["vclock", "gcounter", "pncounter"])
def test_dense_random_vs_oracle(kind, n_actors, gpu, oracle):
    import crdts_hip

    n = 20_011  # odd: exercises the scalar tail
    slots = n_actors * (2 if kind == "pncounter" else 1)
    a = crdts_hip.generate_dense(n, slots, seed=1 + n_actors, bits=64, pct_zero=30)
    b = crdts_hip.generate_dense(n, slots, seed=2 + n_actors, bits=64, pct_zero=30)
    da, db = _dev(a), _dev(b)
    gpu.dense_merge(da, db, n_actors, kind)
    gpu.status()
    exp = oracle.pncounter_merge(a, b, n_actors) if kind == "pncounter" else oracle.dense_merge(a, b, n_actors)
    assert (_host(da) == exp).all()
    assert (_host(db) == b).all()  # other is read-only


def test_dense_unaligned_pointers(gpu, oracle):
    import torch

    a = np.random.default_rng(0).integers(0, 2**63, size=(1001, 16), dtype=np.uint64)
    b = np.random.default_rng(1).integers(0, 2**63, size=(1001, 16), dtype=np.uint64)
    ta = torch.zeros(1001 * 16 + 1, dtype=torch.int64, device="cuda:0")
    tb = torch.zeros(1001 * 16 + 1, dtype=torch.int64, device="cuda:0")
    ta[1:].copy_(_dev(a.ravel()))
    tb[1:].copy_(_dev(b.ravel()))
    gpu.dense_merge(ta[1:], tb[1:], 16, "gcounter")
    gpu.status()
    assert (_host(ta[1:]) == oracle.dense_merge(a, b, 16).ravel()).all()


def test_pncounter_prop_converges_on_gpu(gpu):
    """test/pncounter.rs:22-53 with seeded op vectors; merges on the GPU."""
    import crdts_hip

    for seed in range(20):
        rng = random.Random(seed)
        ops = opgen.pncounter_opvec(rng)
        vals = set()
        for i in range(2, 11):
            ws = [crdts_hip.PNCounter(n_actors=11) for _ in range(i)]
            for (actor, counter), pos in ops:
                ws[actor % i].apply(((actor, counter), pos))
            merged = crdts_hip.PNCounter(n_actors=11)
            for w in ws:
                merged.merge(w, engine=gpu)
            vals.add(merged.value())
        assert len(vals) == 1


def test_gcounter_config2_chunk_properties(gpu):
    """BASELINE configs[1] shape (64 dense actors, U[0,2^40) with 25% zeros) on a
    2M-counter chunk: result == numpy maximum, idempotent, commutative."""
    import crdts_hip

    n = 2_000_000
    a = crdts_hip.generate_dense(n, 64, seed=0xC0FFEE02, threads=16)
    b = crdts_hip.generate_dense(n, 64, seed=0xC0FFEE02 ^ 0x5555, threads=16)
    da, db = _dev(a), _dev(b)
    gpu.dense_merge(da, db, 64, "gcounter")
    gpu.status()
    r = _host(da)
    assert (r == np.maximum(a, b)).all()
    db2 = _dev(b)
    gpu.dense_merge(db2, _dev(a), 64, "gcounter")  # commutative
    gpu.dense_merge(da, da.clone(), 64, "gcounter")  # idempotent
    gpu.status()
    assert (_host(db2) == r).all() and (_host(da) == r).all()


@pytest.mark.parametrize("slots", [16, 128])
def test_dense_merge_host_entry_point(gpu, oracle, slots):
    """crdt_dense_merge_host (host rows: H2D, dense_max_kernel, D2H) — the
    entry point INTEGRATION.md's MergeBatch for VClock / GCounter / PNCounter
    calls — equals the oracle's VClock::merge per row (src/vclock.rs:131-137)."""
    import ctypes as C

    import crdts_hip
    from crdts_hip._lib import check, lib

    a = crdts_hip.generate_dense(3001, slots, seed=91)
    b = crdts_hip.generate_dense(3001, slots, seed=92)
    a[:5] = np.uint64((1 << 64) - 1)  # u64 values above 2^63 stay exact
    exp = oracle.dense_merge(a, b, slots)
    got = np.ascontiguousarray(a.copy())
    check(lib.crdt_dense_merge_host(gpu.ctx, got.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p),
                                    got.shape[0], slots), "dense_merge_host")
    assert (got == exp).all()
