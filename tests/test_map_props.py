"""The reference's Map properties, outright, on its own generator shape
(test/map.rs:13-46 build_opvec, :654-730 prop_merge_associative /
prop_merge_commutative / prop_merge_idempotent), for both value kinds built
here: Map<u64, MVReg<u64>> and Map<u64, Orswot<u64>>.

build_opvec: one actor per op vector; op i carries clock = Dot{actor, i}.into()
and dot = clock.inc(actor) = (actor, i + 1); choice % 3 picks Up / Rm / Nop
(Up's nested op: Put{clock, val} for MVReg; for Orswot an Add with the same
dot, or a nested Rm with the same clock). Maps built from different actors'
vectors (the reference discards equal actors). Checked on the Python
restatement and the C++ oracle's op path (which agree map for map), and on
the GPU kernels (tests marked gpu).
"""
import random

import numpy as np
import pytest

import map_kat_runner as mkr
import map_slab
from map_slab import crdts_ref

SIZE = 100  # quickcheck's default size: u8 draws in [0, 100)


def opvec(rng, actor, n_max=24, keys=SIZE, kind="mvreg"):
    ops = []
    for i in range(rng.randrange(0, n_max + 1)):
        choice, inner, key, val = (rng.randrange(SIZE), rng.randrange(SIZE), rng.randrange(keys),
                                   rng.randrange(SIZE))
        clock = [(actor, i)] if i > 0 else []  # Dot{actor, 0}.into() is the empty clock
        dot = (actor, i + 1)
        if choice % 3 == 0:
            ops.append(("up", dot, key, inner % 2 if kind == "orswot" else 0, val, clock))
        elif choice % 3 == 1:
            ops.append(("rm", None, key, None, None, clock))
    return ops


def apply_ops(be, m, ops, kind):
    for op, dot, key, sub, val, clock in ops:
        if op == "rm":
            be.apply_rm(m, key, clock)
        elif kind == "mvreg":
            be.apply_up_put(m, dot, key, clock, val)
        elif sub == 0:
            be.apply_up_add(m, dot, key, val)
        else:
            _apply_up_orswot_rm(be, m, dot, key, val, clock)


def _apply_up_orswot_rm(be, m, dot, key, member, clock):
    if isinstance(be, mkr.OracleMapBackend):
        m.apply_up_orswot(dot, key, 1, member, clock)
    else:
        m.apply_up(dot, key, lambda s: s.apply_rm(crdts_ref.VClock(clock), member))


def build(rng, kind, keys, be):
    a1, a2, a3 = rng.sample(range(SIZE), 3)
    out = []
    for a in (a1, a2, a3):
        m = be.new(kind)
        apply_ops(be, m, opvec(rng, a, keys=keys, kind=kind), kind)
        out.append(m)
    return out


@pytest.mark.parametrize("kind", ["mvreg", "orswot"])
@pytest.mark.parametrize("keys", [4, SIZE])
def test_map_merge_properties_outright(kind, keys, oracle):
    rng = random.Random(hash((kind, keys)) & 0xFFFF)
    py = mkr.PyMapBackend()
    ob = mkr.OracleMapBackend(SIZE, dict(kcap=32, mcap=32, vdcap=16, vscap=16, dcap=32, scap=32))
    for t in range(150):
        st = rng.getstate()
        m1, m2, m3 = build(rng, kind, keys, py)
        rng.setstate(st)
        o1, o2, o3 = build(rng, kind, keys, ob)
        for x, y in ((m1, o1), (m2, o2), (m3, o3)):
            assert x == ob.view(y)
        # commutative (test/map.rs:688-714)
        a, b = m1.clone(), m2.clone()
        a.merge(m2)
        b.merge(m1)
        assert a == b, t
        oa, obb = o1.clone(), o2.clone()
        oa.merge(o2)
        obb.merge(o1)
        assert ob.view(oa) == a and ob.view(obb) == b
        # idempotent (:716-730)
        c = m1.clone()
        c.merge(m1)
        assert c == m1
        # associative (:654-686)
        x, y = m1.clone(), m2.clone()
        x.merge(m2)
        x.merge(m3)
        y.merge(m3)
        z = m1.clone()
        z.merge(y)
        assert x == z, t


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["mvreg", "orswot"])
def test_map_merge_properties_on_gpu(kind, gpu):
    """The same generator, 2000 pairs per launch: kernel(m1, m2) ==
    kernel(m2, m1) == the restatement's merge, and kernel(m1, m1) == m1."""
    import crdts_hip

    rng = random.Random(77)
    py = mkr.PyMapBackend()
    pairs = [build(rng, kind, 4, py)[:2] for _ in range(2000)]
    # actors interned per pair, order-preserving (every comparison is kept)
    fwds = [{a: i for i, a in enumerate(sorted(map_slab.actors_of(m1) | map_slab.actors_of(m2)))}
            for m1, m2 in pairs]
    A = 8
    assert max(len(f) for f in fwds) <= A
    n = len(pairs)

    def slabs(ms):
        if kind == "orswot":
            S = crdts_hip.MapOrswotSlab.alloc(n, A, kcap=8, mcap=8, vdcap=8, vscap=8, dcap=16, scap=8)
            for i, m in enumerate(ms):
                map_slab.orswot_map_to_row(map_slab.relabel(m, fwds[i]), S, i, A)
        else:
            S = crdts_hip.MapSlab.alloc(n, A, 8, 8, 16, 8)
            for i, m in enumerate(ms):
                map_slab.mvreg_map_to_row(map_slab.relabel(m, fwds[i]), S, i, A)
        return S.to("cuda")

    S1, S2 = slabs([p[0] for p in pairs]), slabs([p[1] for p in pairs])
    f = gpu.map_orswot_merge if kind == "orswot" else gpu.map_mvreg_merge
    rd = map_slab.orswot_map_from_row if kind == "orswot" else map_slab.mvreg_map_from_row
    r12, r21, r11 = f(S1, S2, A).host(), f(S2, S1, A).host(), f(S1, S1, A).host()
    for i, (m1, m2) in enumerate(pairs):
        back = {v: a for a, v in fwds[i].items()}
        exp = m1.clone()
        exp.merge(m2)
        assert map_slab.relabel(rd(r12, i), back) == exp, i
        assert map_slab.relabel(rd(r21, i), back) == exp, i
        assert map_slab.relabel(rd(r11, i), back) == m1, i
