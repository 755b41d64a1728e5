"""Host slab rows <-> the pure-Python Map restatement (oracle/crdts_ref.py) —
test infrastructure for the Map KATs and the Map<u64, Orswot> parity tests.

Layouts: crdt_map_orswot_slab / crdt_map_mvreg_slab (include/crdts_hip.h);
slabs are crdts_hip.MapOrswotSlab / MapSlab with numpy arrays.
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import crdts_ref  # noqa: E402


def _row(clock, A):
    r = np.zeros(A, dtype=np.uint64)
    for a, c in clock.dots.items():
        r[a] = c
    return r


def _clock(row):
    return crdts_ref.VClock([(a, int(c)) for a, c in enumerate(row) if c])


def orswot_map_to_row(m, S, i, A):
    """Write a crdts_ref.Map of Orswot values as row i of a host MapOrswotSlab."""
    a, cp = S.a, S.caps
    for f in a:
        a[f][i] = 0
    a["clock"][i] = _row(m.clock, A)
    keys = sorted(m.entries)
    assert len(keys) <= cp["kcap"] and len(m.deferred) <= cp["dcap"]
    a["n_keys"][i] = len(keys)
    for k, key in enumerate(keys):
        ec, o = m.entries[key]
        a["keys"][i, k] = key
        a["eclock"][i, k] = _row(ec, A)
        a["vclock"][i, k] = _row(o.clock, A)
        mem = sorted(o.entries)
        assert len(mem) <= cp["mcap"] and len(o.deferred) <= cp["vdcap"]
        a["vn_mem"][i, k] = len(mem)
        for j, x in enumerate(mem):
            a["vmem"][i, k, j] = x
            a["vmclock"][i, k, j] = _row(o.entries[x], A)
        defs = crdts_ref.clock_order(list(o.deferred))
        a["vn_def"][i, k] = len(defs)
        for d, c in enumerate(defs):
            s = sorted(o.deferred[c])
            assert len(s) <= cp["vscap"]
            a["vdclock"][i, k, d] = _row(c, A)
            a["vdset_n"][i, k, d] = len(s)
            a["vdset"][i, k, d, :len(s)] = s
    defs = crdts_ref.clock_order(list(m.deferred))
    a["n_def"][i] = len(defs)
    for d, c in enumerate(defs):
        s = sorted(m.deferred[c])
        assert len(s) <= cp["scap"]
        a["dclock"][i, d] = _row(c, A)
        a["dset_n"][i, d] = len(s)
        a["dset"][i, d, :len(s)] = s


def orswot_map_from_row(S, i):
    """Row i of a host MapOrswotSlab -> crdts_ref.Map of Orswot values."""
    a = S.a
    m = crdts_ref.Map(crdts_ref.Orswot)
    m.clock = _clock(a["clock"][i])
    for k in range(int(a["n_keys"][i])):
        o = crdts_ref.Orswot()
        o.clock = _clock(a["vclock"][i, k])
        for j in range(int(a["vn_mem"][i, k])):
            o.entries[int(a["vmem"][i, k, j])] = _clock(a["vmclock"][i, k, j])
        for d in range(int(a["vn_def"][i, k])):
            n = int(a["vdset_n"][i, k, d])
            o.deferred[_clock(a["vdclock"][i, k, d])] = set(int(x) for x in a["vdset"][i, k, d, :n])
        m.entries[int(a["keys"][i, k])] = [_clock(a["eclock"][i, k]), o]
    for d in range(int(a["n_def"][i])):
        n = int(a["dset_n"][i, d])
        m.deferred[_clock(a["dclock"][i, d])] = set(int(x) for x in a["dset"][i, d, :n])
    return m


def mvreg_map_to_row(m, S, i, A):
    """Write a crdts_ref.Map of MVReg values as row i of a host MapSlab (values in Vec order)."""
    a = S.a
    for f in a:
        a[f][i] = 0
    a["clock"][i] = _row(m.clock, A)
    keys = sorted(m.entries)
    assert len(keys) <= S.kcap and len(m.deferred) <= S.dcap
    a["n_keys"][i] = len(keys)
    for k, key in enumerate(keys):
        ec, r = m.entries[key]
        a["keys"][i, k] = key
        a["eclock"][i, k] = _row(ec, A)
        assert len(r.vals) <= S.mcap
        a["mv_n"][i, k] = len(r.vals)
        for v, (c, val) in enumerate(r.vals):
            a["mv_clock"][i, k, v] = _row(c, A)
            a["mv_val"][i, k, v] = val
    defs = crdts_ref.clock_order(list(m.deferred))
    a["n_def"][i] = len(defs)
    for d, c in enumerate(defs):
        s = sorted(m.deferred[c])
        a["dclock"][i, d] = _row(c, A)
        a["dset_n"][i, d] = len(s)
        a["dset"][i, d, :len(s)] = s


def mvreg_map_from_row(S, i):
    a = S.a
    m = crdts_ref.Map(crdts_ref.MVReg)
    m.clock = _clock(a["clock"][i])
    for k in range(int(a["n_keys"][i])):
        r = crdts_ref.MVReg()
        r.vals = [(_clock(a["mv_clock"][i, k, v]), int(a["mv_val"][i, k, v])) for v in range(int(a["mv_n"][i, k]))]
        m.entries[int(a["keys"][i, k])] = [_clock(a["eclock"][i, k]), r]
    for d in range(int(a["n_def"][i])):
        n = int(a["dset_n"][i, d])
        m.deferred[_clock(a["dclock"][i, d])] = set(int(x) for x in a["dset"][i, d, :n])
    return m


def nested_map_to_row(m, S, i, A):
    """Write a crdts_ref.Map of Map<u64, MVReg> values (the reference's
    TestMap) as row i of a host MapMapSlab: the outer map's arrays, and key
    slot k's nested map as inner object i * kcap + k."""
    a = S.a
    for f in a:
        a[f][i] = 0
    a["clock"][i] = _row(m.clock, A)
    keys = sorted(m.entries)
    assert len(keys) <= S.kcap and len(m.deferred) <= S.dcap
    a["n_keys"][i] = len(keys)
    for k in range(S.kcap):
        for f in S.inner.a:
            S.inner.a[f][i * S.kcap + k] = 0
    for k, key in enumerate(keys):
        ec, v = m.entries[key]
        a["keys"][i, k] = key
        a["eclock"][i, k] = _row(ec, A)
        mvreg_map_to_row(v, S.inner, i * S.kcap + k, A)
    defs = crdts_ref.clock_order(list(m.deferred))
    a["n_def"][i] = len(defs)
    for d, c in enumerate(defs):
        ks = sorted(m.deferred[c])
        assert len(ks) <= S.scap
        a["dclock"][i, d] = _row(c, A)
        a["dset_n"][i, d] = len(ks)
        a["dset"][i, d, :len(ks)] = ks


def nested_map_from_row(S, i):
    a = S.a
    m = crdts_ref.Map(lambda: crdts_ref.Map(crdts_ref.MVReg))
    m.clock = _clock(a["clock"][i])
    for k in range(int(a["n_keys"][i])):
        m.entries[int(a["keys"][i, k])] = [_clock(a["eclock"][i, k]), mvreg_map_from_row(S.inner, i * S.kcap + k)]
    for d in range(int(a["n_def"][i])):
        n = int(a["dset_n"][i, d])
        m.deferred[_clock(a["dclock"][i, d])] = set(int(x) for x in a["dset"][i, d, :n])
    return m


def rows_equal(S, i, T, j):
    return all(np.array_equal(S.a[f][i], T.a[f][j]) for f in S.a)


def _relabel_clock(c, f):
    return crdts_ref.VClock([(f[a], n) for a, n in c.dots.items()])


def relabel(m, f):
    """A copy of map `m` (any value kind: MVReg, Orswot, a nested map) with
    every actor id a renamed to f[a] (an order-preserving interning keeps
    CLOCK ORDER and every comparison)."""
    r = crdts_ref.Map(m.factory, m.order)
    r.clock = _relabel_clock(m.clock, f)
    for k, (c, v) in m.entries.items():
        if isinstance(v, crdts_ref.Map):
            o = relabel(v, f)
        elif isinstance(v, crdts_ref.Orswot):
            o = crdts_ref.Orswot()
            o.clock = _relabel_clock(v.clock, f)
            o.entries = {x: _relabel_clock(e, f) for x, e in v.entries.items()}
            o.deferred = {_relabel_clock(d, f): set(s) for d, s in v.deferred.items()}
        else:
            o = crdts_ref.MVReg()
            o.vals = [(_relabel_clock(cc, f), val) for cc, val in v.vals]
        r.entries[k] = [_relabel_clock(c, f), o]
    r.deferred = {_relabel_clock(d, f): set(s) for d, s in m.deferred.items()}
    return r


def actors_of(m):
    s = set(m.clock.dots)
    for c, v in m.entries.values():
        s |= set(c.dots)
        if isinstance(v, crdts_ref.Map):
            s |= actors_of(v)
        elif isinstance(v, crdts_ref.Orswot):
            s |= set(v.clock.dots)
            for e in v.entries.values():
                s |= set(e.dots)
            for d in v.deferred:
                s |= set(d.dots)
        else:
            for cc, _ in v.vals:
                s |= set(cc.dots)
    for d in m.deferred:
        s |= set(d.dots)
    return s
