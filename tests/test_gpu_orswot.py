"""GPU parity: the HIP Orswot join (through the C ABI) vs the oracle.

Bar: bit-exact canonical records for every object.
"""
import random

import numpy as np
import pytest

import kat_runner
import opgen
import records
from gpu_backend import GpuBackend

pytestmark = pytest.mark.gpu
CASES = kat_runner.load_cases()
QC = kat_runner.load_qc_scenarios()


def _dev_batch(crdts_hip, base, off, n_actors):
    return crdts_hip.OrswotBatch.from_host(base, off, n_actors)


def _gpu_merge(gpu, lb, lo, rb, ro, n_actors):
    import crdts_hip

    L = _dev_batch(crdts_hip, lb, lo, n_actors)
    R = _dev_batch(crdts_hip, rb, ro, n_actors)
    out = gpu.orswot_merge(L, R)
    return out


def _compare(gpu_out, ob, oo, what=""):
    got = gpu_out.records()
    exp = records.unpack_batch(ob, oo)
    assert len(got) == len(exp)
    bad = [i for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    if bad:
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} / {len(exp)} objects differ; first {i}:\n"
                             f"gpu    {records.decode(got[i])}\noracle {records.decode(exp[i])}")


# ------------------------------------------------------------------ KATs
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_orswot_kat_on_gpu(case, gpu, oracle):
    be = GpuBackend(gpu, n_actors=16)
    tg, to = [], []
    kat_runner.run_case(case, be, trace=tg)
    kat_runner.run_case(case, kat_runner.OracleBackend(), trace=to)
    assert be.merges == sum(st[0] == "merge" for st in case["steps"])
    for (k1, n1, a), (k2, n2, b) in zip(tg, to):
        assert a.record() == b.encode(16), f"{case['name']} step {k1}"


# ------------------------------------------------------------------ quickcheck_evolution.log
@pytest.mark.parametrize("scn", QC, ids=[s["name"] for s in QC])
def test_quickcheck_evolution_on_gpu(scn, gpu, oracle):
    """quickcheck_evolution.log's 8 op vectors (inputs only, tests/golden/
    quickcheck_evolution.json): every merge of the convergence property
    (i = 2..10 witnesses + plunger) and of every logged witness-list fold runs
    on the kernel; the merged record equals the oracle's at every witness
    count and every fold step, and the witness counts converge."""
    be, ob = GpuBackend(gpu, n_actors=16), kat_runner.OracleBackend()
    results = set()
    for i in range(2, 11):
        _, mg = kat_runner.qc_replay(scn, be, i)
        _, mo = kat_runner.qc_replay(scn, ob, i)
        assert mg.record() == mo.encode(16), f"i={i}"
        results.add(mg.record())
    assert len(results) == 1
    for ws in scn["witness_sets"]:
        tg, to = [], []
        kat_runner.qc_fold(ws["witnesses"], be, tg)
        kat_runner.qc_fold(ws["witnesses"], ob, to)
        for k, (a, b) in enumerate(zip(tg, to)):
            assert a.record() == b.encode(16), f"log lines {ws['log_lines']} step {k}"
    assert be.merges > 0


# ------------------------------------------------------------------ prop_merge_converges
def test_prop_merge_converges_on_gpu(gpu, oracle):
    """test/orswot.rs:37-76: for every op vector, folding i = 2..10 witnesses
    (witness = actor % i) into an empty set in index order, then merging an
    empty 'defer plunger', converges; every fold step runs as one batched
    kernel launch over all (opvec, i) folds, and every step is compared with
    the oracle's fold."""
    import crdts_hip

    A = 100
    rng = random.Random(2024)
    opvecs = [opgen.orswot_opvec(rng) for _ in range(60)]
    folds = []  # (opvec index, i, witnesses as host states, oracle witnesses)
    for v, ops in enumerate(opvecs):
        for i in range(2, 11):
            hw = [crdts_hip.HostOrswot() for _ in range(i)]
            ow = [oracle.OracleOrswot() for _ in range(i)]
            for actor, op in ops:
                for be, w in ((hw, hw[actor % i]), (ow, ow[actor % i])):
                    if op[0] == "add":
                        w.apply_add(op[1], op[2], op[3])
                    else:
                        w.apply_rm(op[1], op[2])
            folds.append((v, i, hw, ow))
    merged = [crdts_hip.HostOrswot().encode(A) for _ in folds]
    omerged = [oracle.OracleOrswot() for _ in folds]
    for step in range(11):
        others = []
        for f, (v, i, hw, ow) in enumerate(folds):
            if step < i:
                others.append(hw[step].encode(A))
                omerged[f].merge(ow[step])
            else:  # the defer plunger, then idempotent re-plunges
                others.append(crdts_hip.HostOrswot().encode(A))
                omerged[f].merge(oracle.OracleOrswot())
        L = crdts_hip.OrswotBatch.from_records(merged, A)
        R = crdts_hip.OrswotBatch.from_records(others, A)
        merged = gpu.orswot_merge(L, R).records()
        for f in range(len(folds)):
            assert merged[f] == omerged[f].encode(A), f"fold {folds[f][:2]} step {step}"
    by_vec = {}
    for f, (v, i, _, _) in enumerate(folds):
        by_vec.setdefault(v, set()).add(merged[f])
    assert all(len(s) == 1 for s in by_vec.values())


# ------------------------------------------------------------------ config 3 differential
def test_config3_differential_200k(gpu, oracle):
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(200_000, threads=16)
    out = _gpu_merge(gpu, lb, lo, rb, ro, 16)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 16, threads=16)
    _compare(out, ob, oo, "config3 200k")
    # output offsets are self.off + other.off
    assert (out.off.cpu().numpy().view(np.uint64) == lo + ro).all()


def test_config3_reverse_orientation(gpu, oracle):
    """Orswot merge is structurally non-commutative (src/orswot.rs:98-103 vs
    :132-137): R ⊔ L must match the oracle's R.merge(&L), not L ⊔ R."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(20_000, first_obj=7, threads=16,
                                                    params=dict(pct_shared_actor=50))
    out = _gpu_merge(gpu, rb, ro, lb, lo, 16)
    ob, oo = oracle.orswot_merge_batch(rb, ro, lb, lo, 16, threads=16)
    _compare(out, ob, oo, "reverse")


@pytest.mark.parametrize("params", [
    dict(pct_deferred_obj=100, pct_future_rm=40),                    # deferred-heavy
    dict(pct_shared_actor=100),                                     # same-actor adds
    dict(n_actors=3, member_universe=8, ancestor_adds=4),          # tiny
    dict(n_actors=64, member_universe=200, ancestor_adds=150, max_div_ops=40),  # > 2 KB stage -> big kernel (LDS)
    dict(n_actors=32, member_universe=2000, ancestor_adds=1500, max_div_ops=60),  # > 16 KB -> big kernel (HBM)
    dict(n_actors=1, member_universe=16, ancestor_adds=8),
    dict(ancestor_adds=0, min_div_ops=0, max_div_ops=3),           # empty / near-empty objects
], ids=["deferred_heavy", "shared_actor", "tiny", "big_lds", "big_hbm", "one_actor", "empty"])
def test_generated_variants(params, gpu, oracle):
    import crdts_hip

    n = 300 if params.get("member_universe", 0) >= 2000 else 5_000
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(n, threads=16, seed=99, params=params)
    A = params.get("n_actors", 16)
    out = _gpu_merge(gpu, lb, lo, rb, ro, A)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, A, threads=16)
    _compare(out, ob, oo, str(params))


def _random_state(rng, A, members, ops):
    import crdts_hip

    h = crdts_hip.HostOrswot()
    for _ in range(ops):
        r = rng.random()
        m = rng.randrange(members)
        a = rng.randrange(A)
        st = crdts_hip.decode_record(h.encode(A))
        if r < 0.55:
            h.apply_add(a, st["clock"].get(a, 0) + 1 + rng.randrange(2), m)
        elif r < 0.8:
            h.apply_rm(m, st["entries"].get(m, []))
        else:
            clk = dict(st["clock"])
            clk[a] = clk.get(a, 0) + rng.randrange(1, 5)
            h.apply_rm(m, sorted(clk.items()))
    return h


def test_random_states_with_deferred(gpu, oracle):
    """Independent random states (no shared ancestor) with many future-context removes."""
    rng = random.Random(77)
    A = 8
    L = [_random_state(rng, A, 12, rng.randrange(0, 40)).encode(A) for _ in range(1500)]
    R = [_random_state(rng, A, 12, rng.randrange(0, 40)).encode(A) for _ in range(1500)]
    lb, lo = records.pack_batch(L)
    rb, ro = records.pack_batch(R)
    out = _gpu_merge(gpu, lb, lo, rb, ro, A)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, A, threads=16)
    _compare(out, ob, oo, "random deferred")
    assert sum(len(records.decode(r)["deferred"]) > 0 for r in L) > 300


def test_self_merge_and_chained_fold(gpu, oracle):
    """x ⊔ x, and a 3-way fold whose intermediate batch (with gaps) is fed back."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(8_000, threads=16, seed=5)
    (cb, co), _ = crdts_hip.generate_orswot(8_000, threads=16, seed=6)
    out = _gpu_merge(gpu, lb, lo, lb, lo, 16)
    ob, oo = oracle.orswot_merge_batch(lb, lo, lb, lo, 16, threads=16)
    _compare(out, ob, oo, "self")
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    C = crdts_hip.OrswotBatch.from_host(cb, co, 16)
    lr = gpu.orswot_merge(L, R)
    lrc = gpu.orswot_merge(lr, C)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 16, threads=16)
    ob2, oo2 = oracle.orswot_merge_batch(ob, oo, cb, co, 16, threads=16)
    _compare(lrc, ob2, oo2, "fold")
    # compaction keeps every record, and outputs validate as canonical
    comp = gpu.orswot_compact(lrc)
    assert comp.records() == lrc.records()
    assert comp.bytes <= lrc.bytes
    gpu.orswot_validate(comp)


def test_validate_and_noncanonical_inputs(gpu):
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(100, threads=4)
    gpu.orswot_validate(crdts_hip.OrswotBatch.from_host(lb, lo, 16))
    bad = lb.copy()
    o = int(lo[10])
    d = records.decode(bad[o:o + int(bad[o:o + 4].view(np.uint32)[0])].tobytes())
    # swap the first two member keys -> not strictly increasing
    key_off = o + 32 + 8 * 16
    k0 = bad[key_off:key_off + 8].copy()
    bad[key_off:key_off + 8] = bad[key_off + 8:key_off + 16]
    bad[key_off + 8:key_off + 16] = k0
    with pytest.raises(crdts_hip.CrdtError):
        gpu.orswot_validate(crdts_hip.OrswotBatch.from_host(bad, lo, 16))
    # a wrong header (n_clk != n_actors) is rejected by the merge kernel itself
    bad2 = lb.copy()
    bad2[int(lo[3]) + 4:int(lo[3]) + 8] = np.frombuffer(np.uint32(17).tobytes(), np.uint8)
    with pytest.raises(crdts_hip.CrdtError):
        _gpu_merge(gpu, bad2, lo, rb, ro, 16)
    assert len(d["entries"]) > 1


def test_misordered_offsets_rejected(gpu):
    """The output placement out.off[i] = self.off[i] + other.off[i] needs each
    side's records in increasing, non-overlapping offset order
    (include/crdts_hip.h); a permuted batch must fail with CRDT_EINVAL
    instead of two objects writing the same output bytes."""
    import crdts_hip
    from crdts_hip._lib import CRDT_EINVAL

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(100, threads=4)
    perm = lo.copy()
    perm[[10, 11]] = perm[[11, 10]]  # records 10 and 11 swapped on the self side only
    with pytest.raises(crdts_hip.CrdtError) as e:
        _gpu_merge(gpu, lb, perm, rb, ro, 16)
    assert e.value.code == CRDT_EINVAL
    shared = lo.copy()
    shared[20] = shared[19]  # two objects sharing one record: overlapping
    with pytest.raises(crdts_hip.CrdtError) as e:
        _gpu_merge(gpu, lb, shared, rb, ro, 16)
    assert e.value.code == CRDT_EINVAL
    _gpu_merge(gpu, lb, lo, rb, ro, 16)  # the context is clean again


def test_capacity_and_empty_batch(gpu):
    import torch

    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(64, threads=2)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    small = crdts_hip.OrswotBatch(torch.empty(L.bytes, dtype=torch.uint8, device="cuda:0"),
                                  torch.empty(64, dtype=torch.int64, device="cuda:0"), 16, L.bytes)
    with pytest.raises(crdts_hip.CrdtError):
        gpu.orswot_merge(L, R, out=small)
    E = crdts_hip.OrswotBatch.from_records([], 16)
    out = gpu.orswot_merge(E, E)
    assert out.n_obj == 0


def test_merge_host_path_matches_device_path(gpu):
    import ctypes as C

    import crdts_hip
    from crdts_hip._lib import lib

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(3_000, threads=8, seed=31)
    dev = _gpu_merge(gpu, lb, lo, rb, ro, 16).records()
    out = np.zeros(lb.nbytes + rb.nbytes, np.uint8)
    ooff = np.zeros(3000, np.uint64)
    used = C.c_size_t()
    rc = lib.crdt_orswot_merge_host(gpu.ctx, lb.ctypes.data, lo.ctypes.data, lb.nbytes, rb.ctypes.data,
                                    ro.ctypes.data, rb.nbytes, 3000, 16, out.ctypes.data, ooff.ctypes.data,
                                    out.nbytes, C.byref(used))
    assert rc == 0
    assert records.unpack_batch(out, ooff) == dev
    assert used.value == sum(len(r) for r in dev)


def test_config3_full_size_bitexact(gpu, oracle):
    """BASELINE.json configs[2] at full size (1M objects): every record equals the oracle's."""
    import crdts_hip

    n = 1_000_000
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(n, threads=16)
    out = _gpu_merge(gpu, lb, lo, rb, ro, 16)
    gb, go = out.to_host()
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 16, threads=16)
    # compare record by record with numpy views (sizes first, then bytes)
    gs = gb.view(np.uint32)[(go // 4).astype(np.int64)]
    os_ = ob.view(np.uint32)[(oo // 4).astype(np.int64)]
    assert (gs == os_).all()
    gi = np.concatenate([np.arange(o, o + s, dtype=np.int64) for o, s in zip(go[:50_000], gs[:50_000])])
    oi = np.concatenate([np.arange(o, o + s, dtype=np.int64) for o, s in zip(oo[:50_000], os_[:50_000])])
    assert (gb[gi] == ob[oi]).all()
    # the rest via a checksum of per-record checksums
    def digest(base, offs, sizes):
        h = np.zeros(len(offs), dtype=np.uint64)
        w = base.view(np.uint64)
        for k in range(int(sizes.max()) // 8):
            m = sizes > 8 * k
            h[m] = (h[m] * np.uint64(0x100000001B3)) ^ w[(offs[m] // 8 + k).astype(np.int64)]
        return h
    assert (digest(gb, go, gs) == digest(ob, oo, os_)).all()


def test_general_path_list_overflow_and_reset(gpu, oracle):
    """Objects the fast kernel cannot take go through the general kernel's
    list; with a tiny list it falls back to scanning every output offset.
    Launches alternate so the list counter reset between launches is exercised."""
    import crdts_hip

    params = dict(n_actors=64, member_universe=200, ancestor_adds=150, max_div_ops=40)
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(700, threads=16, seed=4, params=params)
    (cb, co), (db, do) = crdts_hip.generate_orswot(3000, threads=16, seed=8)  # fast path only
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 64, threads=16)
    ob2, oo2 = oracle.orswot_merge_batch(cb, co, db, do, 16, threads=16)
    try:
        for cap in (8, 0, 65536, 8):
            gpu.set_list_cap(cap)
            _compare(_gpu_merge(gpu, lb, lo, rb, ro, 64), ob, oo, f"cap {cap}")
            _compare(_gpu_merge(gpu, cb, co, db, do, 16), ob2, oo2, f"fast after cap {cap}")
    finally:
        gpu.set_list_cap(65536)


def test_empty_side_key_equal_to_clock_word(gpu, oracle):
    """A side without members next to a member whose key equals the word in
    front of the empty side's key section (its last top-clock counter): the
    member is self-only / other-only, never matched (regression: the clamped
    equal-key probe of the join read that word)."""
    A = 4
    full = records.encode({0: 1, 3: 2}, {3: {0: 1}, 7: {3: 2}}, {}, A)
    empty = records.encode({3: 3}, {}, {}, A)  # top clock word [A-1] == 3 == a key of `full`
    for L, R in ((full, empty), (empty, full)):
        lb, lo = records.pack_batch([L] * 65 + [R])
        rb, ro = records.pack_batch([R] * 65 + [L])
        out = _gpu_merge(gpu, lb, lo, rb, ro, A)
        ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, A, threads=4)
        _compare(out, ob, oo, "empty side")


@pytest.mark.parametrize("n", [1, 2, 7, 63, 64, 65, 1000, 4097, 24_583])
def test_guided_split_batch_sizes(n, gpu, oracle):
    """The guided chunk schedule (static chunks for the first 5/8 of the
    objects, ticket chunks of 20 for the rest; csrc/sched.h) covers every
    object exactly once at sizes around its chunk boundaries: all-ticket
    batches (n = 1), partial tickets, a partial last static round, and
    repeated launches on one context (the ticket counter is re-zeroed)."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(n, threads=16, seed=1234 + n)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 16, threads=16)
    for _ in range(2):
        out = _gpu_merge(gpu, lb, lo, rb, ro, 16)
        _compare(out, ob, oo, f"n={n}")


def _mixed_batch(n_small=20_000, seed=21):
    """Config-3 pairs with two kinds of objects past the join's limits mixed
    in at random positions, all over 16 actors: records past the 2 KB stage
    (listed at the chunk step) and pairs of near-disjoint ~45-member sides
    whose union passes 64 members (found inside the join)."""
    import crdts_hip

    (sb, so), (tb, to) = crdts_hip.generate_orswot(n_small, threads=16, seed=seed)
    big = dict(member_universe=200, ancestor_adds=150, max_div_ops=40)
    (bb, bo), (cb, co) = crdts_hip.generate_orswot(300, threads=16, seed=seed + 1, params=big)
    wide = dict(member_universe=100_000, ancestor_adds=45, min_div_ops=0, max_div_ops=2)
    (wb, wo), _ = crdts_hip.generate_orswot(300, threads=16, seed=seed + 2, params=wide)
    (xb, xo), _ = crdts_hip.generate_orswot(300, threads=16, seed=seed + 3, params=wide)
    L = records.unpack_batch(sb, so) + records.unpack_batch(bb, bo) + records.unpack_batch(wb, wo)
    R = records.unpack_batch(tb, to) + records.unpack_batch(cb, co) + records.unpack_batch(xb, xo)
    perm = np.random.default_rng(seed).permutation(len(L))
    lb, lo = records.pack_batch([L[i] for i in perm])
    rb, ro = records.pack_batch([R[i] for i in perm])
    return lb, lo, rb, ro


def test_mixed_batch_general_path_list_caps(gpu, oracle):
    """Objects past the join kernel's limits at random positions of a
    config-3 batch — records past the 2 KB stage (listed at the chunk step)
    and unions past 64 members (found inside the join) — go to the general
    kernel; with a small or empty list it scans the flags instead. Launches
    repeat on one context and alternate with the 64-actor path (every object
    general)."""
    lb, lo, rb, ro = _mixed_batch()
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 16, threads=16)
    # how many objects leave the fast path: some of each kind
    hl = lb.view(np.uint32)[(lo // 4).astype(np.int64)]
    hr = rb.view(np.uint32)[(ro // 4).astype(np.int64)]
    assert ((hl > 2048) | (hr > 2048)).sum() > 100
    gl = np.stack([lb[int(o) + 8:int(o) + 12].view(np.uint32)[0] for o in lo])
    assert (gl >= 40).sum() > 100
    import crdts_hip

    params = dict(n_actors=64, member_universe=200, ancestor_adds=150, max_div_ops=40)
    (pb, po), (qb, qo) = crdts_hip.generate_orswot(200, threads=16, seed=4, params=params)
    pob, poo = oracle.orswot_merge_batch(pb, po, qb, qo, 64, threads=16)
    try:
        for cap in (65536, 8, 0, 65536, 65536):
            gpu.set_list_cap(cap)
            _compare(_gpu_merge(gpu, lb, lo, rb, ro, 16), ob, oo, f"mixed, cap {cap}")
            _compare(_gpu_merge(gpu, pb, po, qb, qo, 64), pob, poo, f"64 actors after cap {cap}")
        for k in range(3):  # back to back on one stream
            _compare(_gpu_merge(gpu, lb, lo, rb, ro, 16), ob, oo, f"repeat {k}")
    finally:
        gpu.set_list_cap(65536)


def test_header_without_deferred_clocks_but_deferred_counts_rejected(gpu):
    """A record whose header says n_def = 0 but counts deferred dots or
    members (sized to match, so the size check alone passes) is not
    canonical: the merge kernel rejects it (header_ok) rather than copy
    those counts into an output header."""
    import crdts_hip
    from crdts_hip._lib import CRDT_ENONCANON

    A = 16
    good = records.encode({0: 2, 3: 1}, {5: {0: 2}, 9: {3: 1}}, {}, A)
    for dot, mem in ((1, 0), (0, 1)):
        n = records.record_bytes(A, 2, 2, 0, dot, mem)
        bad = bytearray(good) + bytes(n - len(good))
        h = np.frombuffer(bad, np.uint32)
        h[0], h[5], h[6] = n, dot, mem
        lb, lo = records.pack_batch([bytes(bad)] * 70)
        rb, ro = records.pack_batch([good] * 70)
        with pytest.raises(crdts_hip.CrdtError) as e:
            _gpu_merge(gpu, lb, lo, rb, ro, A)
        assert e.value.code == CRDT_ENONCANON
    lb, lo = records.pack_batch([good] * 70)
    _gpu_merge(gpu, lb, lo, lb, lo, A)  # the context is clean again


# ------------------------------------------------------------------ 33-64 dense actors
@pytest.mark.parametrize("A,n", [(64, 100_000), (33, 30_000), (48, 30_000)])
def test_dense_33_to_64_actors(gpu, oracle, A, n):
    """Dense top clocks of 33-64 actors take the join kernel's 64-bit actor
    mask form (mask3_object<AW 64>; the reference clock has no actor bound,
    src/vclock.rs:54-57): config-3-shaped pairs over A actors, deferred-remove
    objects included, byte-exact against the oracle (bench.py --n-actors 64
    times the same form)."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(n, threads=16, seed=0xC0FFEE03 + A, params={"n_actors": A})
    recs = records.unpack_batch(lb, lo)
    assert sum(1 for r in recs[:2000] if records.decode(r)["deferred"]) > 20  # deferred removes present
    assert max(a for r in recs[:2000] for a in records.decode(r)["clock"]) >= 32  # actors past the 32-bit masks
    out = _gpu_merge(gpu, lb, lo, rb, ro, A)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, A, threads=16)
    _compare(out, ob, oo, f"A={A}")


# ------------------------------------------------------------------ 65-1024 dense actors
@pytest.mark.parametrize("A,n,anc", [(100, 100_000, 32), (128, 100_000, 32), (200, 20_000, 100), (700, 5_000, 32)])
def test_dense_wide_actors(gpu, oracle, A, n, anc):
    """Dense top clocks wider than the 64-bit actor masks (65-1024 actors; the
    reference clock has no actor bound, src/vclock.rs:54-57) take the sparse
    mask join over each object's union of PRESENT actors (a dense clock stores
    0 for an absent actor) in its dense form, and objects whose union passes
    64 actors (A = 200 with 100 ancestor adds) or whose pair passes the 6 KB
    stage (A = 700: 5.6 KB of clocks alone) the general kernel; config-3-shaped
    pairs with deferred removes, byte-exact against the oracle (bench.py
    --n-actors 128 times the same form)."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(n, threads=16, seed=0xC0FFEE03 + A,
                                                   params={"n_actors": A, "ancestor_adds": anc})
    recs = records.unpack_batch(lb, lo)
    assert sum(1 for r in recs[:2000] if records.decode(r)["deferred"]) > 20  # deferred removes present
    assert max(a for r in recs[:2000] for a in records.decode(r)["clock"]) >= 64  # actors past the 64-bit masks
    out = _gpu_merge(gpu, lb, lo, rb, ro, A)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, A, threads=16)
    _compare(out, ob, oo, f"A={A}")


WIDE_UNION = {"n_actors": 128, "ancestor_adds": 96, "member_universe": 32, "pct_add": 45, "max_div_ops": 20}


def test_dense_wide_union(gpu, oracle):
    """The wide-union distribution (bench.py --n-actors 128 --gen-params of
    DESIGN.md §11): 128 dense actors with ~72 present per object pair — the
    union of present actors passes 64 for ~98 % of the objects, with <= 64
    members and ~80 dots per side — so nearly every object leaves the DN
    mask join; byte-exact against the oracle, both orientations."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(30_000, threads=16, seed=0xC0FFEE80, params=WIDE_UNION)
    A = WIDE_UNION["n_actors"]
    q = lb.view(np.uint64)
    idx = (lo // 8 + 4).astype(np.int64)[:, None] + np.arange(A)[None, :]
    qr = rb.view(np.uint64)
    idr = (ro // 8 + 4).astype(np.int64)[:, None] + np.arange(A)[None, :]
    union = ((q[idx] != 0) | (qr[idr] != 0)).sum(1)
    assert (union > 64).mean() > 0.9
    for a, b in (((lb, lo), (rb, ro)), ((rb, ro), (lb, lo))):
        out = _gpu_merge(gpu, *a, *b, A)
        ob, oo = oracle.orswot_merge_batch(*a, *b, A, threads=16)
        _compare(out, ob, oo, "wide union")
    # orswot_dense_wide_kernel (pairs past the DN kernel's 6 KB stage, ~5 %)
    # from the DN kernel's list, and from the flags when the list overflows
    # (cap 8: halves of 4) or is absent (0)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, A, threads=16)
    try:
        for cap in (8, 0):
            gpu.set_list_cap(cap)
            _compare(_gpu_merge(gpu, lb, lo, rb, ro, A), ob, oo, f"wide union, cap {cap}")
    finally:
        gpu.set_list_cap(65536)


@pytest.mark.parametrize("U", [63, 64, 65, 127, 128, 129])
def test_dense_wide_union_boundaries(gpu, oracle, U):
    """Object pairs whose top clocks hold exactly U present actors between
    them, at 160 dense actors: the dense-wide join's 64-bit masks up to 64,
    its 128-bit masks up to 128, the general kernel past 128 — in the DN
    kernel for pairs within its 6 KB stage (10-55 % of them here) and in
    orswot_dense_wide_kernel for the larger ones. Shared and one-sided
    actors, removes through the whole clock (read context) and
    future-context removes left deferred; byte-exact against the oracle in
    both orientations (src/orswot.rs:87-157, src/vclock.rs:54-57)."""
    import crdts_hip

    rng = random.Random(0xB0 + U)
    A, n = 160, 160
    L, R = [], []
    for _ in range(n):
        acts = rng.sample(range(A), U)
        ns = rng.randrange(U // 4, U // 2 + 1)
        shared, rest = acts[:ns], acts[ns:]
        cut = rng.randrange(len(rest) + 1)
        for side, dst in ((shared + rest[:cut], L), (shared + rest[cut:], R)):
            h, clk = crdts_hip.HostOrswot(), {}
            for a in side:  # every actor of the side in its top clock
                clk[a] = clk.get(a, 0) + 1
                h.apply_add(a, clk[a], rng.randrange(24))
            for _ in range(rng.randrange(0, 30)):
                a, m, r = rng.choice(side), rng.randrange(24), rng.random()
                if r < 0.6:
                    clk[a] += 1
                    h.apply_add(a, clk[a], m)
                elif r < 0.85:
                    h.apply_rm(m, sorted(clk.items()))
                else:  # a context past the clock: left deferred
                    h.apply_rm(m, sorted({**clk, a: clk[a] + rng.randrange(1, 4)}.items()))
            dst.append(h.encode(A))
    union = [len(set(records.decode(x)["clock"]) | set(records.decode(y)["clock"])) for x, y in zip(L, R)]
    assert set(union) == {U}
    assert sum(1 for r in L if records.decode(r)["deferred"]) > n // 10
    lb, lo = records.pack_batch(L)
    rb, ro = records.pack_batch(R)
    for a, b in (((lb, lo), (rb, ro)), ((rb, ro), (lb, lo))):
        out = _gpu_merge(gpu, *a, *b, A)
        ob, oo = oracle.orswot_merge_batch(*a, *b, A, threads=16)
        _compare(out, ob, oo, f"union of {U}")


# ------------------------------------------------------------------ heavy-tailed batches
def test_heavy_tail_100k(gpu, oracle):
    """Config 3 with a heavy tail (bench.py --workload orswot_tail): every 20th
    object op-simulated at 100 / 300 / 1000 members per side (the reference's
    entries map is unbounded, src/orswot.rs:26-30) — records up to ~28 KB,
    past the join kernel's 2 KB stage and 64-member masks — byte-exact against
    the oracle, both orientations."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot_tail(100_000, threads=16)
    recs = records.unpack_batch(lb, lo)
    big = [i for i in range(0, 100_000, 20)]
    assert max(len(recs[i]) for i in big) > 16_384 and min(len(records.decode(recs[i])["entries"]) for i in big) > 64
    for a, b in (((lb, lo), (rb, ro)), ((rb, ro), (lb, lo))):
        out = _gpu_merge(gpu, *a, *b, 16)
        ob, oo = oracle.orswot_merge_batch(*a, *b, 16, threads=16)
        _compare(out, ob, oo, "heavy tail")


def _synth_heavy_pair(rng, n, n_actors=16, n_def=4):
    """One op-shaped pair of n-member Orswots from a common ancestor (one dot
    per member, top clock = per-actor max): self adds / removes as actors
    0-7, other as 8-15, and each side defers n_def removes whose context
    runs ahead of it on the other side's actors — the reference's
    remove-before-add case (src/orswot.rs:197-203). Built directly as records
    (the op simulator takes minutes at 100k+ members)."""
    pool = rng.choice(1 << 40, size=int(n * 1.25), replace=False).astype(np.uint64).tolist()
    anc, fresh = pool[:n], pool[n:]
    ctr = [0] * n_actors
    ent = {}
    for m, a in zip(anc, rng.integers(0, n_actors, size=n).tolist()):
        ctr[a] += 1
        ent[m] = {a: ctr[a]}
    sides = []
    for lo_a, hi_a in ((0, n_actors // 2), (n_actors // 2, n_actors)):
        c = list(ctr)
        e = {m: dict(d) for m, d in ent.items()}
        n_add = n // 6
        for m in rng.choice(anc, size=n_add, replace=False).tolist() + fresh[lo_a * 1000:lo_a * 1000 + n // 20]:
            a = int(rng.integers(lo_a, hi_a))
            c[a] += 1
            e.setdefault(m, {})[a] = c[a]
        for m in rng.choice(anc, size=n // 10, replace=False).tolist():
            e.pop(m, None)
        deferred = {}
        for _ in range(n_def):
            a = int(rng.integers(n_actors // 2 - lo_a, n_actors - lo_a)) % n_actors  # an actor of the other side
            ctx = tuple(sorted({a: ctr[a] + int(rng.integers(1, n // 8 + 2))}.items()))
            deferred[ctx] = set(rng.choice(anc, size=3, replace=False).tolist())
        clock = {a: v for a, v in enumerate(c) if v}
        sides.append(records.encode(clock, e, deferred, n_actors))
    return sides


def test_big_kernel_paths(gpu, oracle):
    """orswot_big_kernel's three paths, byte-exact against the oracle, both
    orientations: records staged in LDS (<= 32 KB a side), records joined
    from HBM with the tables in the stage (P <= 262 144 union positions), and
    past those tables one wave (merge_object), next to config-3 pairs."""
    import crdts_hip

    rng = np.random.default_rng(0xB16)
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(40, threads=4)
    Ls, Rs = records.unpack_batch(lb, lo), records.unpack_batch(rb, ro)
    for k, n in enumerate((150, 700, 1200, 3000, 20000, 150000)):
        a, b = _synth_heavy_pair(rng, n, n_def=4 + 8 * (k % 2))
        Ls[5 * k + 1], Rs[5 * k + 1] = a, b
    sizes = sorted(len(r) for r in Ls)
    assert sizes[-1] > 3_000_000 and sizes[-3] > 32768
    lb, lo = records.pack_batch(Ls)
    rb, ro = records.pack_batch(Rs)
    for x, y in (((lb, lo), (rb, ro)), ((rb, ro), (lb, lo))):
        out = _gpu_merge(gpu, *x, *y, 16)
        ob, oo = oracle.orswot_merge_batch(*x, *y, 16, threads=8)
        _compare(out, ob, oo, "big kernel paths")


def test_heavy_tail_list_caps(gpu, oracle):
    """The heavy tail's objects reach orswot_big_kernel by the join's big list
    (headers already big), the general list, or — when a half of the
    context's list is full — the pending flags: caps that overflow neither
    half, only the big half (1 500: halves of 750 < 1 000 heavy objects),
    both (8), and none at all (0); byte-exact every time, alternating with the
    unlimited cap on one context."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot_tail(20_000, threads=16)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 16, threads=16)
    try:
        for cap in (65536, 1500, 8, 0, 65536):
            gpu.set_list_cap(cap)
            _compare(_gpu_merge(gpu, lb, lo, rb, ro, 16), ob, oo, f"tail, cap {cap}")
    finally:
        gpu.set_list_cap(65536)
