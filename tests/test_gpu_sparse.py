"""GPU parity for CSR (sparse) top clocks — config 5 (BASELINE.json configs[4]).

The HIP join over sparse records (crdt_orswot_merge_ex, flags =
CRDT_ORSWOT_SPARSE_CLOCK) against the oracle's sparse merge, byte-exact:
the reference's KATs with every state crossing the ABI in sparse form, the
config-5 replica fold (((r0 ⊔ r1) ⊔ r2) ... ⊔ r7) step by step, both
orientations, random states with deferred removes over a 1024-actor universe,
and validation / rejection of records in the wrong form.
"""
import random

import numpy as np
import pytest

import kat_runner
import records
from gpu_backend import GpuBackend

pytestmark = pytest.mark.gpu
CASES = kat_runner.load_cases()
SPARSE = 1
U = 1024


def _compare(got, ob, oo, what=""):
    exp = records.unpack_batch(ob, oo)
    assert len(got) == len(exp)
    bad = [i for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    if bad:
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} / {len(exp)} objects differ; first {i}:\n"
                             f"gpu    {records.decode(got[i])}\noracle {records.decode(exp[i])}")


def _merge(gpu, lb, lo, rb, ro, A=U):
    import crdts_hip

    L = crdts_hip.OrswotBatch.from_host(lb, lo, A, flags=SPARSE)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, A, flags=SPARSE)
    return gpu.orswot_merge(L, R)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_orswot_kat_sparse_on_gpu(case, gpu, oracle):
    be = GpuBackend(gpu, n_actors=U, sparse=True)
    tg, to = [], []
    kat_runner.run_case(case, be, trace=tg)
    kat_runner.run_case(case, kat_runner.OracleBackend(), trace=to)
    for (k1, _, a), (k2, _, b) in zip(tg, to):
        assert a.record() == b.encode(U, SPARSE), f"{case['name']} step {k1}"


def test_config5_replica_fold(gpu, oracle):
    import crdts_hip

    n = 60_000
    reps = crdts_hip.generate_replicas(n, 8, threads=16)
    acc_g = crdts_hip.OrswotBatch.from_host(*reps[0], U, flags=SPARSE)
    acc_o = reps[0]
    for r in range(1, 8):
        R = crdts_hip.OrswotBatch.from_host(*reps[r], U, flags=SPARSE)
        acc_g = gpu.orswot_merge(acc_g, R)
        acc_o = oracle.orswot_merge_batch(acc_o[0], acc_o[1], reps[r][0], reps[r][1], U, threads=16, flags=SPARSE)
        _compare(acc_g.records(), acc_o[0], acc_o[1], f"fold step {r}")
    gpu.orswot_validate(gpu.orswot_compact(acc_g))
    nnz = [records.decode(x)["size"] for x in acc_g.records()[:100]]
    assert np.mean(nnz) > 0


def test_config5_reverse_orientation(gpu, oracle):
    import crdts_hip

    reps = crdts_hip.generate_replicas(20_000, 2, first_obj=11, threads=16,
                                       params=dict(pct_deferred_obj=50, pct_future_rm=30))
    (ab, ao), (bb, bo) = reps
    out = _merge(gpu, bb, bo, ab, ao)
    ob, oo = oracle.orswot_merge_batch(bb, bo, ab, ao, U, threads=16, flags=SPARSE)
    _compare(out.records(), ob, oo, "reverse")


def _random_state(rng, members, ops):
    import crdts_hip

    h = crdts_hip.HostOrswot()
    actors = [rng.randrange(U) for _ in range(10)]
    for _ in range(ops):
        r = rng.random()
        m = rng.randrange(members)
        a = rng.choice(actors)
        st = crdts_hip.decode_record(h.encode(U, SPARSE))
        if r < 0.55:
            h.apply_add(a, st["clock"].get(a, 0) + 1 + rng.randrange(2), m)
        elif r < 0.8:
            h.apply_rm(m, st["entries"].get(m, []))
        else:
            clk = dict(st["clock"])
            clk[a] = clk.get(a, 0) + rng.randrange(1, 5)
            h.apply_rm(m, sorted(clk.items()))
    return h


def test_random_sparse_states_with_deferred(gpu, oracle):
    rng = random.Random(31)
    L = [_random_state(rng, 12, rng.randrange(0, 40)).encode(U, SPARSE) for _ in range(1200)]
    R = [_random_state(rng, 12, rng.randrange(0, 40)).encode(U, SPARSE) for _ in range(1200)]
    lb, lo = records.pack_batch(L)
    rb, ro = records.pack_batch(R)
    out = _merge(gpu, lb, lo, rb, ro)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, U, threads=16, flags=SPARSE)
    _compare(out.records(), ob, oo, "random sparse")
    assert sum(len(records.decode(r)["deferred"]) > 0 for r in L) > 200


def test_sparse_large_records_hbm_path(gpu, oracle):
    """Records larger than the 4 KB LDS stage are joined straight from HBM."""
    import crdts_hip

    reps = crdts_hip.generate_replicas(300, 2, threads=16, seed=3,
                                       params=dict(pool_actors=400, ancestor_adds=900, member_universe=900,
                                                   max_div_ops=60))
    (ab, ao), (bb, bo) = reps
    assert max(records.decode(r)["size"] for r in records.unpack_batch(ab, ao)) > 4096
    out = _merge(gpu, ab, ao, bb, bo)
    ob, oo = oracle.orswot_merge_batch(ab, ao, bb, bo, U, threads=16, flags=SPARSE)
    _compare(out.records(), ob, oo, "large sparse")


def test_sparse_validate_and_form_mismatch(gpu):
    import crdts_hip

    reps = crdts_hip.generate_replicas(2000, 2, threads=16)
    B = crdts_hip.OrswotBatch.from_host(*reps[0], U, flags=SPARSE)
    gpu.orswot_validate(B)
    # dense records through the sparse path (and the reverse) are rejected
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(500, threads=8)
    with pytest.raises(crdts_hip.CrdtError):
        _merge(gpu, lb, lo, rb, ro, 16)
    with pytest.raises(crdts_hip.CrdtError):
        gpu.orswot_merge(crdts_hip.OrswotBatch.from_host(*reps[0], U), crdts_hip.OrswotBatch.from_host(*reps[1], U))
    # an unsorted sparse clock fails deep validation
    b, o = reps[0]
    b = b.copy()
    rec = records.decode(b[int(o[3]):int(o[3]) + 4096].tobytes())
    n = len(rec["clock"])
    assert n >= 2
    acts = b[int(o[3]) + 32 + 8 * n: int(o[3]) + 32 + 12 * n].view(np.uint32)
    acts[0], acts[1] = acts[1], acts[0]
    with pytest.raises(crdts_hip.CrdtError):
        gpu.orswot_validate(crdts_hip.OrswotBatch.from_host(b, o, U, flags=SPARSE))


def test_dense_and_sparse_launches_alternate_on_one_context(gpu, oracle):
    """The dense and the sparse join share the context's alternating
    control-word sets (no memset before a launch: each launch's general
    kernel zeroes the set the next launch uses). Dense and sparse launches,
    with objects past the 2 KB / 6 KB stages in both, interleaved on one
    context in runs of 1, 2 and 3 — every output equals the oracle's."""
    import crdts_hip

    (db, do), (eb, eo) = crdts_hip.generate_orswot(6_000, threads=16, seed=71)
    big = dict(member_universe=200, ancestor_adds=150, max_div_ops=40)
    (fb, fo), (gb, go) = crdts_hip.generate_orswot(200, threads=16, seed=72, params=big)
    dl, dr = records.unpack_batch(db, do) + records.unpack_batch(fb, fo), \
        records.unpack_batch(eb, eo) + records.unpack_batch(gb, go)
    lb, lo = records.pack_batch(dl)
    rb, ro = records.pack_batch(dr)
    dexp = oracle.orswot_merge_batch(lb, lo, rb, ro, 16, threads=16)
    (sa, sao), (sb, sbo) = crdts_hip.generate_replicas(6_000, 2, threads=16, seed=73)
    sexp = oracle.orswot_merge_batch(sa, sao, sb, sbo, U, threads=16, flags=SPARSE)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    for k, kind in enumerate("dsddssdddsss"):
        if kind == "d":
            _compare(gpu.orswot_merge(L, R).records(), *dexp, f"dense launch {k}")
        else:
            _compare(_merge(gpu, sa, sao, sb, sbo).records(), *sexp, f"sparse launch {k}")


# ------------------------------------------------------------------ heavy CSR objects
def test_csr_heavy_tail_100k(gpu, oracle):
    """Config 5's record form with a heavy tail (bench.py --workload
    orswot_csr_tail): every 20th object at ~100 / 300 / 1000 members per side
    (the reference's entries map and clock are unbounded, src/orswot.rs:26-30,
    src/vclock.rs:54-57). Objects past 128 union positions or the general
    stage take orswot_big_kernel<true> (one workgroup per object, CSR top
    clock); byte-exact against the oracle, both orientations."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot_csr_tail(100_000, threads=16)
    recs = records.unpack_batch(lb, lo)
    heavy = list(range(0, 100_000, 20))
    sizes = [len(records.decode(recs[i])["entries"]) for i in heavy]
    assert sum(s > 128 for s in sizes) > len(heavy) // 2 and max(len(recs[i]) for i in heavy) > 16_384
    for a, b in (((lb, lo), (rb, ro)), ((rb, ro), (lb, lo))):
        got = _merge(gpu, *a, *b).records()
        ob, oo = oracle.orswot_merge_batch(*a, *b, U, threads=16, flags=SPARSE)
        _compare(got, ob, oo, "CSR heavy tail")


def test_csr_big_kernel_hbm_path(gpu, oracle):
    """CSR objects of ~3 000 members per side (records past the big kernel's
    32 KB LDS stage: its HBM-table path) mixed 1:1 with config-5 objects,
    byte-exact against the oracle, both orientations."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot_csr_tail(400, frac=0.5, sizes=(3000,), threads=16)
    recs = records.unpack_batch(lb, lo)
    assert max(len(recs[i]) for i in range(0, 400, 2)) > 32_768
    for a, b in (((lb, lo), (rb, ro)), ((rb, ro), (lb, lo))):
        got = _merge(gpu, *a, *b).records()
        ob, oo = oracle.orswot_merge_batch(*a, *b, U, threads=16, flags=SPARSE)
        _compare(got, ob, oo, "CSR big HBM path")


def test_csr_heavy_tail_list_caps(gpu, oracle):
    """CSR heavy tail with list caps that overflow the big half, both halves,
    or leave no list at all: the big objects still reach
    orswot_big_kernel<true> (by the pending flags), byte-exact."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot_csr_tail(20_000, threads=16)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, U, threads=16, flags=SPARSE)
    try:
        for cap in (65536, 1500, 8, 0, 65536):
            gpu.set_list_cap(cap)
            _compare(_merge(gpu, lb, lo, rb, ro).records(), ob, oo, f"CSR tail, cap {cap}")
    finally:
        gpu.set_list_cap(65536)
