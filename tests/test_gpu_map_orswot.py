"""GPU parity: Map<u64, Orswot<u64, A>, A>::merge (crdt_map_orswot_merge,
rust-crdt_amd/csrc/map_orswot.hip) against the oracle — slab-row exact — and
the reference's Map KATs with every merge on the kernel.

Map Val semantics: src/map.rs:192-269 (merge), :325-350 (apply_deferred,
apply_rm), src/orswot.rs:87-172 (nested merge, truncate). The final
apply_deferred runs in CLOCK ORDER (tests/test_map_orswot.py settles that the
reference's HashMap order can matter; CLOCK ORDER is one of its orders)."""
import numpy as np
import pytest

import map_kat_runner as mkr
import map_slab
import test_map_orswot as tmo
from map_slab import crdts_ref

pytestmark = pytest.mark.gpu
A = 8
CASES = mkr.load_cases()


class GpuMapBackend(mkr.PyMapBackend):
    """States built by the Python op path; every merge runs on the kernel: both
    maps are interned to dense actor ids (order-preserving), written to slabs,
    merged by crdt_map_orswot_merge (Orswot values) or crdt_map_mvreg_merge
    (MVReg values), and read back."""

    def __init__(self, eng):
        self.eng = eng
        self.merges = 0

    def merge(self, dst, src):
        import crdts_hip

        acts = sorted(map_slab.actors_of(dst) | map_slab.actors_of(src)) or [0]
        fwd = {a: i for i, a in enumerate(acts)}
        back = {i: a for a, i in fwd.items()}
        n = len(acts)
        d, s = map_slab.relabel(dst, fwd), map_slab.relabel(src, fwd)
        if dst.factory is crdts_ref.Orswot:
            S = crdts_hip.MapOrswotSlab.alloc(1, n, **mkr.CAPS)
            O = crdts_hip.MapOrswotSlab.alloc(1, n, **mkr.CAPS)
            map_slab.orswot_map_to_row(d, S, 0, n)
            map_slab.orswot_map_to_row(s, O, 0, n)
            R = self.eng.map_orswot_merge(S.to("cuda"), O.to("cuda"), n).host()
            out = map_slab.orswot_map_from_row(R, 0)
        else:
            S = crdts_hip.MapSlab.alloc(1, n, 4, 4, 4, 4)
            O = crdts_hip.MapSlab.alloc(1, n, 4, 4, 4, 4)
            map_slab.mvreg_map_to_row(d, S, 0, n)
            map_slab.mvreg_map_to_row(s, O, 0, n)
            R = self.eng.map_mvreg_merge(S.to("cuda"), O.to("cuda"), n).host()
            out = map_slab.mvreg_map_from_row(R, 0)
        out = map_slab.relabel(out, back)
        dst.clock, dst.entries, dst.deferred = out.clock, out.entries, out.deferred
        self.merges += 1


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_map_kat_on_gpu(case, gpu, oracle):
    """Every KAT script with each merge on the kernel; the reference's asserts
    hold and every merged state equals the oracle's."""
    be = GpuMapBackend(gpu)
    tg, to = [], []
    a = mkr.run_case(case, be, tg)
    b = mkr.run_case(case, mkr.OracleMapBackend(), to)
    assert be.merges == sum(st[0] == "merge" for st in case["steps"])
    assert all(x == y for (_, _, x), (_, _, y) in zip(tg, to))
    assert all(a[k] == b[k] for k in a)


def test_map_mvreg_kat_final_states_merge_on_gpu(gpu):
    """The Map<u8, MVReg> op-path KATs end in equal maps; merging every pair of
    their final states on the kernel gives the Python restatement's merge."""
    be = GpuMapBackend(gpu)
    for case in CASES:
        fin = mkr.run_case(case, mkr.PyMapBackend())
        names = sorted(fin)
        for x in names:
            for y in names:
                g, p = fin[x].clone(), fin[x].clone()
                be.merge(g, fin[y])
                p.merge(fin[y])
                assert g == p, (case["name"], x, y)


@pytest.mark.parametrize("pct_future", [10, 35])
def test_map_orswot_random_parity(gpu, oracle, pct_future):
    """20k generated pairs, both orientations: kernel == oracle, slab-row exact."""
    L, R = oracle.map_orswot_generate(0xB0B + pct_future, 20000, A, keys=4, members=6, ops=10,
                                      pct_future=pct_future)
    import crdts_hip

    for S, O in ((L, R), (R, L)):
        exp = oracle.map_orswot_merge(S, O, A).canonical()
        # the kernel writes only the used slots: the rest of a reused output
        # keeps whatever it held (here a pattern), so canonical forms are compared
        caps = {k: S.caps[k] + O.caps[k] for k in S.caps}
        out = crdts_hip.MapOrswotSlab.alloc(S.n, A, device="cuda", **caps)
        for v in out.a.values():
            v.fill_(0x5A5A5A5A)
        got = gpu.map_orswot_merge(S.to("cuda"), O.to("cuda"), A, out=out).canonical()
        for f in exp.a:
            bad = np.nonzero((np.asarray(got.a[f]) != np.asarray(exp.a[f])).reshape(S.n, -1).any(axis=1))[0]
            assert bad.size == 0, f"{f}: {bad.size} objects differ, first {bad[:5].tolist()}"


def test_map_orswot_order_case_on_gpu(gpu, oracle):
    """The reachable pair whose result depends on the deferred order: the
    kernel gives the CLOCK ORDER outcome."""
    import crdts_hip

    a, b = tmo._order_case()
    S = crdts_hip.MapOrswotSlab.alloc(1, A, **oracle.MAP_ORSWOT_CAPS)
    O = crdts_hip.MapOrswotSlab.alloc(1, A, **oracle.MAP_ORSWOT_CAPS)
    map_slab.orswot_map_to_row(a, S, 0, A)
    map_slab.orswot_map_to_row(b, O, 0, A)
    got = map_slab.orswot_map_from_row(gpu.map_orswot_merge(S.to("cuda"), O.to("cuda"), A).host(), 0)
    exp = a.clone()
    exp.merge(b)
    assert got == exp and len(got.entries[7][1].deferred) == 1


def test_map_orswot_errors(gpu, oracle):
    import crdts_hip

    L, R = oracle.map_orswot_generate(0xC4, 64, A, keys=4, members=6, ops=10, pct_future=20)
    # output capacity: one key slot per map
    caps = dict(oracle.MAP_ORSWOT_CAPS, kcap=1)
    with pytest.raises(crdts_hip.CrdtError) as e:
        gpu.map_orswot_merge(L.to("cuda"), R.to("cuda"), A, out_caps=caps)
    assert e.value.code == crdts_hip.CRDT_ECAPACITY
    # malformed counts: a nested member count above its capacity
    bad = crdts_hip.MapOrswotSlab({f: v.copy() for f, v in L.a.items()}, L.caps)
    k = int(np.nonzero(bad.a["n_keys"])[0][0])
    bad.a["vn_mem"][k, 0] = bad.caps["mcap"] + 1
    with pytest.raises(crdts_hip.CrdtError) as e:
        gpu.map_orswot_merge(bad.to("cuda"), R.to("cuda"), A)
    assert e.value.code == crdts_hip.CRDT_ENONCANON
    gpu.status()  # the context is usable again after the latched error


def test_map_orswot_200_keys_100_actors(gpu, oracle):
    """Maps past the round-3 slab limits (32 keys, 64 actors): ~200 keys per
    map over 100 actors (the kernel's two-slots-per-lane rows: lane l holds
    actors l and l + 64), nested and map-level deferred removes whose clocks
    name actor 99, both orientations, slab-row exact against the oracle
    (src/map.rs:192-269)."""
    import crdts_hip

    A100 = 100
    caps = dict(kcap=512, mcap=8, vdcap=8, vscap=8, dcap=32, scap=64)
    L, R = oracle.map_orswot_generate(0x200A, 48, A100, keys=400, members=6, ops=450, pct_future=20, caps=caps)
    assert (L.a["n_keys"] >= 200).sum() > 10 and L.a["clock"][:, 64:].any()
    assert L.a["vn_def"].sum() > 20 and L.a["n_def"].sum() > 10
    for S, O in ((L, R), (R, L)):
        exp = oracle.map_orswot_merge(S, O, A100).canonical()
        got = gpu.map_orswot_merge(S.to("cuda"), O.to("cuda"), A100).canonical()
        for f in exp.a:
            bad = np.nonzero((np.asarray(got.a[f]) != np.asarray(exp.a[f])).reshape(S.n, -1).any(axis=1))[0]
            assert bad.size == 0, f"{f}: {bad.size} objects differ, first {bad[:5].tolist()}"


@pytest.mark.parametrize("scap", [16, 64])
def test_map_orswot_many_keys_16_actors(gpu, oracle, scap):
    """Past 64 keys per map at 16 actors (one slot per lane): the key walk
    reads keys and counts past the first 64 from the slab, and the map
    deferred sets are staged in LDS per object (scap 16: 4 KB, the staging
    limit) or read from HBM (scap 64); both orientations, slab-row exact."""
    A = 16
    caps = dict(kcap=256, mcap=16, vdcap=8, vscap=16, dcap=16, scap=scap)
    L, R = oracle.map_orswot_generate(0x3A1, 64, A, keys=120, members=6, ops=160, pct_future=20, caps=caps)
    assert (L.a["n_keys"] > 64).sum() > 10 and L.a["n_def"].sum() > 10
    for S, O in ((L, R), (R, L)):
        exp = oracle.map_orswot_merge(S, O, A).canonical()
        got = gpu.map_orswot_merge(S.to("cuda"), O.to("cuda"), A).canonical()
        for f in exp.a:
            bad = np.nonzero((np.asarray(got.a[f]) != np.asarray(exp.a[f])).reshape(S.n, -1).any(axis=1))[0]
            assert bad.size == 0, f"{f}: {bad.size} objects differ, first {bad[:5].tolist()}"


def test_map_orswot_100_map_deferred_clocks(gpu, oracle):
    """Past the round-4 map deferred cap (32 per side): maps holding 57-157
    map-level deferred removes per side (dcap 160; the combined list up to
    ~300 entries, key sets up to 40 keys, read from HBM past the staging
    area), both orientations, slab-row exact against the oracle
    (src/map.rs:255-260 deferral, :325-350 apply_deferred / apply_rm)."""
    caps = dict(kcap=256, mcap=8, vdcap=8, vscap=8, dcap=160, scap=64)
    L, R = oracle.map_orswot_generate(0x100D, 16, 16, keys=300, members=4, ops=800, pct_future=70, caps=caps)
    assert L.a["n_def"].max() >= 100 and R.a["n_def"].max() >= 100 and (L.a["n_def"] >= 100).sum() >= 4
    for S, O in ((L, R), (R, L)):
        exp = oracle.map_orswot_merge(S, O, 16).canonical()
        assert exp.a["n_def"].max() > 128
        got = gpu.map_orswot_merge(S.to("cuda"), O.to("cuda"), 16).canonical()
        for f in exp.a:
            bad = np.nonzero((np.asarray(got.a[f]) != np.asarray(exp.a[f])).reshape(S.n, -1).any(axis=1))[0]
            assert bad.size == 0, f"{f}: {bad.size} objects differ, first {bad[:5].tolist()}"


def _nested_deferred_map(seed, keys, n_mem, n_rm, me, other):
    """Map<u64, Orswot> through the op path: per key, n_mem members added by
    actor `me`, then n_rm member removes whose clocks run ahead on actor
    `other` (a context from a replica this one has not heard from) — each
    deferred inside the nested set (src/orswot.rs:190-203), n_rm distinct
    clocks per key."""
    import random

    rng = random.Random(seed)
    m = crdts_ref.Map(crdts_ref.Orswot)
    for k in range(keys):
        for j in range(n_mem):
            add, _, _ = m.get(k)
            dot = (me, add.get(me) + 1)
            m.apply_up(dot, k, lambda s, d=dot, x=j: s.apply_add(d, x))
        for j in range(n_rm):
            add, _, _ = m.get(k)
            dot = (me, add.get(me) + 1)
            ctx = crdts_ref.VClock([(me, rng.randint(1, n_mem)), (other, 40 + 3 * j + rng.randint(0, 2))])
            m.apply_up(dot, k, lambda s, c=ctx, x=rng.randrange(n_mem): s.apply_rm(c, x))
    return m


def test_map_orswot_nested_deferred_past_32(gpu, oracle):
    """Past the round-4 nested deferred cap (32 per key per side): nested sets
    holding 45-60 deferred removes per side (vdcap 64), both orientations,
    GPU == oracle slab-row exact and == the Python restatement's merge."""
    import crdts_hip

    A8 = 4
    a = _nested_deferred_map(1, 3, 24, 60, 0, 1)
    b = _nested_deferred_map(2, 3, 24, 45, 1, 0)
    assert max(len(v[1].deferred) for v in a.entries.values()) > 32
    caps = dict(kcap=4, mcap=32, vdcap=64, vscap=4, dcap=4, scap=4)
    for x, y in ((a, b), (b, a)):
        S = crdts_hip.MapOrswotSlab.alloc(1, A8, **caps)
        O = crdts_hip.MapOrswotSlab.alloc(1, A8, **caps)
        map_slab.orswot_map_to_row(x, S, 0, A8)
        map_slab.orswot_map_to_row(y, O, 0, A8)
        exp = oracle.map_orswot_merge(S, O, A8)
        got = gpu.map_orswot_merge(S.to("cuda"), O.to("cuda"), A8).host()
        ce, cg = exp.canonical(), got.canonical()
        for f in ce.a:
            assert np.array_equal(np.asarray(cg.a[f]), np.asarray(ce.a[f])), f
        py = x.clone()
        py.merge(y)
        assert map_slab.orswot_map_from_row(got, 0) == py
        assert max(int(v) for v in np.asarray(ce.a["vn_def"]).reshape(-1)) > 32
