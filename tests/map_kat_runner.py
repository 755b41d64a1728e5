"""Interpreter for the reference's Map known-answer tests (tests/golden/kat_map.json).

Backends:
  - PyMapBackend: the pure-Python restatement (oracle/crdts_ref.py Map);
  - OracleMapBackend: the C++ oracle's Map handles (oracle/ref_cpu.cpp MapO /
    MapOrswotO, the op path of its generators);
  - GpuMapBackend (tests/test_gpu_map_orswot.py): states built by the Python
    op path, every `merge` executed by the HIP kernel through the C ABI.
Assertions are the reference's, so a backend that passes is pinned to the
reference's behaviour on these cases.
"""
from __future__ import annotations

import json
import os

import map_slab
from map_slab import crdts_ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CAPS = dict(kcap=4, mcap=4, vdcap=4, vscap=4, dcap=4, scap=4)


def load_cases(nested=False):
    """The flat Map KATs (Orswot / MVReg values: every backend), or with
    nested=True the TestMap ones (Map<u8, Map<u8, MVReg>>: the Python
    restatement only)."""
    with open(os.path.join(GOLDEN, "kat_map.json")) as f:
        cases = json.load(f)["cases"]
    return [c for c in cases if (c.get("kind") == "nested") == nested]


def nested_map():
    """TestMap (test/map.rs:8): Map<u8, Map<u8, MVReg<u8, u8>, u8>, u8>."""
    return crdts_ref.Map(lambda: crdts_ref.Map(crdts_ref.MVReg))


def apply_raw(m, op):
    """A literal nested Op (the JSON form of kat_map.json's `raw` steps):
    Op::Nop, Op::Rm {clock, key}, Op::Up {dot, key, op} with the inner
    Map<u8, MVReg> op Nop | Rm | Up {dot, key, Put {clock, val}} (src/map.rs:160-190)."""
    if op == "nop":
        return
    if "rm" in op:
        m.apply_rm(op["rm"]["key"], crdts_ref.VClock([tuple(p) for p in op["rm"]["clock"]]))
        return
    up = op["up"]
    m.apply_up(tuple(up["dot"]), up["key"], lambda v: apply_raw_inner(v, up["op"]))


def apply_raw_inner(v, op):
    if op == "nop":
        return
    if "rm" in op:
        v.apply_rm(op["rm"]["key"], crdts_ref.VClock([tuple(p) for p in op["rm"]["clock"]]))
        return
    up = op["up"]
    put = up["op"]["put"]
    v.apply_up(tuple(up["dot"]), up["key"],
               lambda r: r.apply_put(crdts_ref.VClock([tuple(p) for p in put["clock"]]), put["val"]))


def _pairs(clock):
    return sorted(clock.dots.items())


class PyMapBackend:
    def new(self, kind):
        if kind == "nested":
            return nested_map()
        return crdts_ref.Map(crdts_ref.Orswot if kind == "orswot" else crdts_ref.MVReg)

    def clone(self, m):
        return m.clone()

    def view(self, m):
        return m

    def apply_up_add(self, m, dot, key, member):
        m.apply_up(dot, key, lambda s: s.apply_add(dot, member))

    def apply_up_put(self, m, dot, key, put_pairs, val):
        m.apply_up(dot, key, lambda r: r.apply_put(crdts_ref.VClock(put_pairs), val))

    def apply_rm(self, m, key, pairs):
        m.apply_rm(key, crdts_ref.VClock(pairs))

    def apply_nested_put(self, m, dot, key1, key2, clock, val):
        # map.update(key1, ctx, |map, ctx| map.update(key2, ctx, |reg, ctx| reg.set(val, ctx))):
        # Op::Up {ctx.dot, key1, Op::Up {ctx.dot, key2, Put {ctx.clock, val}}}
        apply_raw(m, {"up": {"dot": list(dot), "key": key1,
                             "op": {"up": {"dot": list(dot), "key": key2, "op": {"put": {"clock": clock, "val": val}}}}}})

    def apply_raw(self, m, op):
        apply_raw(m, op)

    def merge(self, dst, src):
        dst.merge(src)


class OracleMapBackend:
    """C++ oracle handles; reads go through a slab row and the Python decoder."""

    def __init__(self, n_actors=100, caps=None):
        import oracle_ffi

        self.f = oracle_ffi
        self.A = n_actors
        self.caps = caps or CAPS

    def new(self, kind):
        return self.f.OracleMap(kind)

    def clone(self, m):
        return m.clone()

    def view(self, m):
        S = m.slab(self.A, self.caps)
        return map_slab.orswot_map_from_row(S, 0) if m.kind == "orswot" else map_slab.mvreg_map_from_row(S, 0)

    def apply_up_add(self, m, dot, key, member):
        m.apply_up_orswot(dot, key, 0, member)

    def apply_up_put(self, m, dot, key, put_pairs, val):
        m.apply_up_mvreg(dot, key, put_pairs, val)

    def apply_rm(self, m, key, pairs):
        m.apply_rm(key, pairs)

    def merge(self, dst, src):
        dst.merge(src)


def run_case(case, backend, trace=None):
    """Run one Map KAT script; AssertionError on the first failing assert.
    `trace` (optional list) receives (step, name, view of the map) after every merge."""
    maps, ctxs, ops = {}, {}, {}
    name = case["name"]
    for k, st in enumerate(case["steps"]):
        op = st[0]
        where = f"{name} step {k} {st}"
        if op == "new":
            maps[st[1]] = backend.new(st[2])
        elif op == "clone":
            maps[st[1]] = backend.clone(maps[st[2]])
        elif op == "get":  # Map::get ReadCtx: add_clock = map clock, rm_clock = entry clock
            v = backend.view(maps[st[2]])
            add, rm, _ = v.get(st[3])
            ctxs[st[1]] = (_pairs(add), _pairs(rm))
        elif op in ("up_add", "up_put", "nup_put"):  # derive_add_ctx(actor): dot = add_clock.inc(actor), clock = add_clock + dot
            add, _ = ctxs[st[2]]
            actor = st[3]
            dot = (actor, dict(add).get(actor, 0) + 1)
            clock = sorted({**dict(add), actor: dot[1]}.items())
            ops[st[1]] = (op, dot, st[4], st[5:] if op == "nup_put" else st[5], clock)
        elif op == "raw":
            ops[st[1]] = ("raw", None, None, st[2], None)
        elif op == "rm":  # derive_rm_ctx: the entry clock
            ops[st[1]] = ("rm", None, st[3], None, ctxs[st[2]][1])
        elif op == "apply":
            kind, dot, key, arg, clock = ops[st[2]]
            m = maps[st[1]]
            if kind == "up_add":
                backend.apply_up_add(m, dot, key, arg)
            elif kind == "up_put":
                backend.apply_up_put(m, dot, key, clock, arg)
            elif kind == "nup_put":
                backend.apply_nested_put(m, dot, key, arg[0], clock, arg[1])
            elif kind == "raw":
                backend.apply_raw(m, arg)
            else:
                backend.apply_rm(m, key, clock)
        elif op == "merge":
            backend.merge(maps[st[1]], maps[st[2]])
            if trace is not None:
                trace.append((k, st[1], backend.view(maps[st[1]]).clone()))
        elif op == "assert_none":
            assert backend.view(maps[st[1]]).get(st[2])[2] is None, where
        elif op == "assert_set":
            v = backend.view(maps[st[1]]).get(st[2])[2]
            assert v is not None and sorted(v.entries) == sorted(st[3]), f"{where}: {v and sorted(v.entries)}"
        elif op == "assert_read":
            v = backend.view(maps[st[1]]).get(st[2])[2]
            assert v is not None and sorted(v.read()) == sorted(st[3]), f"{where}"
        elif op == "assert_nested_read":  # get(k1).val.and_then(|m| m.get(k2).val).map(|r| r.read().val)
            v = backend.view(maps[st[1]]).get(st[2])[2]
            r = v.get(st[3])[2] if v is not None else None
            assert r is not None and sorted(r.read()) == sorted(st[4]), f"{where}"
        elif op == "assert_eq":
            a, b = backend.view(maps[st[1]]), backend.view(maps[st[2]])
            assert a == b, f"{where}: {a.canonical()} != {b.canonical()}"
        else:
            raise ValueError(f"unknown step {op}")
    return {n: backend.view(m) for n, m in maps.items()}
