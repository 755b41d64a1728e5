"""GPU parity of the nested map merge, crdt_map_map_merge: Map<u64,
Map<u64, MVReg<u64>>> — the reference's own Map test type (TestMap,
test/map.rs:4-8) — against the Python restatement (oracle/crdts_ref.py Map,
generic over its values as src/map.rs is), slab-exact after canonicalisation:

- the reference's nested-map KATs (tests/golden/kat_map.json, test/map.rs:
  297-510) with every merge executed by the kernel, the reference's asserts
  holding and every merged state equal to the restatement's;
- replica pairs built by the op path (nested puts, outer removes and inner
  removes through their read contexts, a third replica's removes arriving
  early and staying deferred, partial out-of-order exchange), at 16 actors
  and at 100 (two slots per lane), both orientations.
The CPU-side pin of the restatement itself is tests/test_map_nested_oracle.py."""
import random

import numpy as np
import pytest

import map_kat_runner as mkr
import map_slab
import nested_gen
from map_slab import crdts_ref

pytestmark = pytest.mark.gpu

CAPS = dict(kcap=4, dcap=8, scap=4)
INNER = (4, 8, 8, 4)  # kcap, mcap, dcap, scap of the nested maps
CASES = mkr.load_cases(nested=True)


def gpu_merge(eng, dst, src):
    """dst ⊔ src on the kernel (actors interned order-preserving to 0..n-1)."""
    import crdts_hip

    acts = sorted(map_slab.actors_of(dst) | map_slab.actors_of(src)) or [0]
    fwd = {a: i for i, a in enumerate(acts)}
    back = {i: a for a, i in fwd.items()}
    n = len(acts)
    S = crdts_hip.MapMapSlab.alloc(1, n, inner_caps=INNER, **CAPS)
    O = crdts_hip.MapMapSlab.alloc(1, n, inner_caps=INNER, **CAPS)
    map_slab.nested_map_to_row(map_slab.relabel(dst, fwd), S, 0, n)
    map_slab.nested_map_to_row(map_slab.relabel(src, fwd), O, 0, n)
    R = eng.map_map_merge(S.to("cuda"), O.to("cuda"), n).host()
    return map_slab.relabel(map_slab.nested_map_from_row(R, 0), back)


class GpuNestedBackend(mkr.PyMapBackend):
    def __init__(self, eng):
        self.eng = eng
        self.merges = 0

    def merge(self, dst, src):
        out = gpu_merge(self.eng, dst, src)
        dst.clock, dst.entries, dst.deferred = out.clock, out.entries, out.deferred
        self.merges += 1


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_nested_map_kat_on_gpu(case, gpu):
    be = GpuNestedBackend(gpu)
    tg, tp = [], []
    a = mkr.run_case(case, be, tg)
    b = mkr.run_case(case, mkr.PyMapBackend(), tp)
    assert be.merges == sum(st[0] == "merge" for st in case["steps"])
    assert all(x == y for (_, _, x), (_, _, y) in zip(tg, tp))
    assert all(a[k] == b[k] for k in a)


@pytest.mark.parametrize("A,n", [(16, 300), (100, 120)])
def test_nested_map_pairs_on_gpu(gpu, A, n):
    import crdts_hip

    rng = random.Random(A)
    pool = list(range(A))
    pairs = [nested_gen.pair(rng, pool) for _ in range(n)]
    S = crdts_hip.MapMapSlab.alloc(n, A, inner_caps=INNER, **CAPS)
    O = crdts_hip.MapMapSlab.alloc(n, A, inner_caps=INNER, **CAPS)
    for i, (x, y) in enumerate(pairs):
        map_slab.nested_map_to_row(x, S, i, A)
        map_slab.nested_map_to_row(y, O, i, A)
    # outer and inner deferred removes, concurrent values and entries occur
    assert S.a["n_def"].sum() > n // 10 and S.inner.a["n_def"].sum() > n // 100 and S.a["n_keys"].sum() > n
    assert (S.inner.a["mv_n"] > 1).sum() > n // 20
    if A > 64:
        assert S.a["clock"][:, 64:].any()
    for X, Y, flip in ((S, O, False), (O, S, True)):
        R = gpu.map_map_merge(X.to("cuda"), Y.to("cuda"), A).host()
        for i, (x, y) in enumerate(pairs):
            a, b = (y, x) if flip else (x, y)
            exp = a.clone()
            exp.merge(b)
            got = map_slab.nested_map_from_row(R, i)
            assert got == exp, f"pair {i}: {got.canonical()} != {exp.canonical()}"


def test_nested_map_limits(gpu):
    """Outer limits kcap 4096, dcap 64, scap 4096 and n_actors 128 accepted;
    one past each CRDT_EINVAL; an output smaller than the sums CRDT_EINVAL."""
    import crdts_hip
    from crdts_hip._lib import CRDT_EINVAL

    def run(A, inner=INNER, **kw):
        caps = dict(CAPS, **kw)
        S = crdts_hip.MapMapSlab.alloc(2, A, inner_caps=inner, device="cuda:0", **caps)
        return gpu.map_map_merge(S, S, A)

    run(128)
    for kw in ({"kcap": 4096}, {"dcap": 64}, {"scap": 4096}):
        run(8, inner=(1, 1, 1, 1), **kw)
    for A, kw in ((129, {}), (8, {"kcap": 4097}), (8, {"dcap": 65}), (8, {"scap": 4097})):
        with pytest.raises(crdts_hip.CrdtError) as e:
            run(A, inner=(1, 1, 1, 1), **kw)
        assert e.value.code == CRDT_EINVAL, (A, kw)
    S = crdts_hip.MapMapSlab.alloc(2, 8, inner_caps=INNER, device="cuda:0", **CAPS)
    small = crdts_hip.MapMapSlab.alloc(2, 8, inner_caps=INNER, device="cuda:0", **CAPS)  # not the sums
    with pytest.raises(crdts_hip.CrdtError) as e:
        gpu.map_map_merge(S, S, 8, out=small)
    assert e.value.code == CRDT_EINVAL


def test_nested_map_malformed_inner_under_truncation(gpu):
    """A malformed nested map (n_keys past its kcap) in the tasks of the fused
    merge-and-truncate kernel (map_mvreg_merge_kernel<G>: each task merges one
    output key's nested maps and applies Map::truncate as it writes,
    src/map.rs:131-158). The scratch now holds only the tasks and their
    truncating clocks (map_map_scratch_bytes); it is filled with garbage
    first. A task whose nested map is malformed latches CRDT_ENONCANON and
    writes no row from the bad counts; the well-formed objects of the same
    batch still merge and truncate exactly (against the Python restatement)."""
    import crdts_hip
    from crdts_hip._lib import CRDT_ENONCANON

    A, n = 16, 200
    rng = random.Random(5)
    pool = list(range(A))
    pairs = [nested_gen.pair(rng, pool) for _ in range(n)]
    S = crdts_hip.MapMapSlab.alloc(n, A, inner_caps=INNER, **CAPS)
    O = crdts_hip.MapMapSlab.alloc(n, A, inner_caps=INNER, **CAPS)
    for i, (x, y) in enumerate(pairs):
        map_slab.nested_map_to_row(x, S, i, A)
        map_slab.nested_map_to_row(y, O, i, A)
    gpu.map_map_merge(S.to("cuda"), O.to("cuda"), A)  # (allocates the engine's scratch)
    bad_objs = [i for i in range(0, n, 3) if S.a["n_keys"][i] > 0]
    kc = S.inner.kcap
    for i in bad_objs:  # every used key slot's nested map claims kcap + 1 keys
        for k in range(int(S.a["n_keys"][i])):
            S.inner.a["n_keys"][i * S.kcap + k] = kc + 1
    gpu._map_map_scratch.fill_(0x7F)  # garbage counts in the task scratch
    R = gpu.map_map_merge(S.to("cuda"), O.to("cuda"), A, check_status=False)
    with pytest.raises(crdts_hip.CrdtError) as e:
        gpu.status()
    assert e.value.code == CRDT_ENONCANON
    R = R.host()
    bad = set(bad_objs)
    for i, (x, y) in enumerate(pairs):
        if i in bad:
            continue
        exp = x.clone()
        exp.merge(y)
        assert map_slab.nested_map_from_row(R, i) == exp, f"pair {i}"
