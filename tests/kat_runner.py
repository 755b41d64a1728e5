"""Interpreter for the reference's Orswot known-answer tests (tests/golden/kat_orswot.json).

A case is a script of the reference's own test steps; a *backend* supplies the
replica objects. The same script runs on
  - the pure-Python restatement (oracle/crdts_ref.py),
  - the C++ oracle (tests/oracle_ffi.py),
  - the product: states built by the product's host op path, every `merge`
    executed by the HIP kernel through the C ABI (tests/gpu_backend.py).
Assertions are the reference's assertions, so a backend that passes is pinned
to the reference's behaviour on these cases.
"""
from __future__ import annotations

import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_cases():
    with open(os.path.join(GOLDEN, "kat_orswot.json")) as f:
        return json.load(f)["cases"]


def load_qc_scenarios():
    """tests/golden/quickcheck_evolution.json (tools/make_golden_qc.py)."""
    with open(os.path.join(GOLDEN, "quickcheck_evolution.json")) as f:
        return json.load(f)["scenarios"]


def _state_record(state, n_actors=16):
    import records

    return records.encode(dict((a, c) for a, c in state["clock"]),
                          {m: dict((a, c) for a, c in clk) for m, clk in state["entries"]},
                          {tuple((a, c) for a, c in d): set(ms) for d, ms in state["deferred"]}, n_actors)


class PyBackend:
    """Backend over oracle/crdts_ref.py."""

    def __init__(self):
        import sys

        sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN), "..", "oracle"))
        import crdts_ref  # noqa: E402

        self.m = crdts_ref

    def new(self):
        return self.m.Orswot()

    def load(self, state):
        o = self.m.Orswot()
        o.clock = self.m.VClock([tuple(x) for x in state["clock"]])
        o.entries = {m: self.m.VClock([tuple(x) for x in c]) for m, c in state["entries"]}
        o.deferred = {self.m.VClock([tuple(x) for x in d]): set(ms) for d, ms in state["deferred"]}
        return o

    def clone(self, o):
        return o.clone()

    def apply_add(self, o, actor, counter, member):
        o.apply_add((actor, counter), member)

    def apply_rm(self, o, member, pairs):
        o.apply_rm(self.m.VClock(pairs), member)

    def merge(self, dst, src):
        dst.merge(src)

    def clock(self, o):
        return sorted(o.clock.dots.items())

    def entry(self, o, member):
        c = o.entries.get(member)
        return None if c is None else sorted(c.dots.items())

    def value(self, o):
        return sorted(o.entries)

    def deferred_len(self, o):
        return len(o.deferred)


class OracleBackend:
    """Backend over the C++ oracle handles."""

    def __init__(self):
        import oracle_ffi

        self.f = oracle_ffi

    def new(self):
        return self.f.OracleOrswot()

    def load(self, state):
        return self.f.OracleOrswot.decode(_state_record(state))

    def clone(self, o):
        return o.clone()

    def apply_add(self, o, actor, counter, member):
        o.apply_add(actor, counter, member)

    def apply_rm(self, o, member, pairs):
        o.apply_rm(member, pairs)

    def merge(self, dst, src):
        dst.merge(src)

    def clock(self, o):
        return o.clock()

    def entry(self, o, member):
        return o.entry(member)

    def value(self, o):
        return o.value()

    def deferred_len(self, o):
        return o.deferred_len()


def run_case(case, backend, trace=None):
    """Run one KAT script; raises AssertionError on the first failing assert.

    `trace` (optional list) receives (step_index, name, replica) after every
    merge so callers can compare replicas across backends.
    """
    im = case.get("intern", {})
    actors = im.get("actors", {})
    members = im.get("members", {})

    def A(x):
        return actors[x] if isinstance(x, str) else int(x)

    def M(x):
        return members[x] if isinstance(x, str) else int(x)

    reps, ctxs = {}, {}
    name = case["name"]
    for k, st in enumerate(case["steps"]):
        op = st[0]
        where = f"{name} step {k} {st}"
        if op == "new":
            reps[st[1]] = backend.new()
        elif op == "clone":
            reps[st[1]] = backend.clone(reps[st[2]])
        elif op == "read":  # Orswot::value() ReadCtx, src/orswot.rs:227-233
            c = backend.clock(reps[st[2]])
            ctxs[st[1]] = {"add": c, "rm": c, "val": None}
        elif op == "contains":  # Orswot::contains, src/orswot.rs:214-224
            e = backend.entry(reps[st[2]], M(st[3]))
            ctxs[st[1]] = {"add": backend.clock(reps[st[2]]), "rm": e or [], "val": e is not None}
        elif op == "add":  # derive_add_ctx src/ctx.rs:599-607 then apply Add
            ctx = ctxs[st[3]]
            a = A(st[4])
            ctr = dict(ctx["add"]).get(a, 0) + 1
            backend.apply_add(reps[st[1]], a, ctr, M(st[2]))
        elif op == "rm":  # derive_rm_ctx src/ctx.rs:610-614 then apply Rm
            backend.apply_rm(reps[st[1]], M(st[2]), list(ctxs[st[3]]["rm"]))
        elif op == "rm_clock":
            backend.apply_rm(reps[st[1]], M(st[2]), [(A(a), int(c)) for a, c in st[3]])
        elif op == "merge":
            backend.merge(reps[st[1]], reps[st[2]])
            if trace is not None:  # a snapshot: the replica may change in later steps
                trace.append((k, st[1], backend.clone(reps[st[1]])))
        elif op == "assert_value":
            got = backend.value(reps[st[1]])
            exp = sorted(M(x) for x in st[2])
            assert got == exp, f"{where}: value {got} != {exp}"
        elif op == "assert_deferred_len":
            got = backend.deferred_len(reps[st[1]])
            assert got == st[2], f"{where}: deferred len {got} != {st[2]}"
        elif op == "assert_ctx_rm_clock":
            exp = sorted((A(a), int(c)) for a, c in st[2])
            got = sorted(ctxs[st[1]]["rm"])
            assert got == exp, f"{where}: rm_clock {got} != {exp}"
        elif op == "assert_ctx_add_clock":
            exp = sorted((A(a), int(c)) for a, c in st[2])
            got = sorted(ctxs[st[1]]["add"])
            assert got == exp, f"{where}: add_clock {got} != {exp}"
        elif op == "assert_ctx_val":
            assert ctxs[st[1]]["val"] == st[2], f"{where}"
        elif op == "assert_next_dot":
            a = A(st[2])
            dot = (a, dict(ctxs[st[1]]["add"]).get(a, 0) + 1)
            exp = (A(st[3][0]), int(st[3][1]))
            assert dot == exp, f"{where}: next dot {dot} != {exp}"
        else:
            raise ValueError(f"unknown step {op}")
    return reps


def qc_replay(scn, backend, i):
    """One witness count of a quickcheck_evolution scenario: the op vector
    replayed onto i witnesses (rule in the fixture's _doc), folded in index
    order into a new set, then the empty 'defer plunger' (test/orswot.rs:44-62).
    Returns (witnesses, merged)."""
    ws = [backend.new() for _ in range(i)]
    adds = {}
    for op in scn["ops"]:
        w = ws[op["actor"] % i]
        if op["kind"] == "add":
            adds[op["actor"]] = adds.get(op["actor"], 0) + 1
            backend.apply_add(w, op["actor"], adds[op["actor"]], op["member"])
        elif op["ctx"] is None:  # contains(member).derive_rm_ctx() on that witness
            backend.apply_rm(w, op["member"], list(backend.entry(w, op["member"]) or []))
        else:
            backend.apply_rm(w, op["member"], [tuple(x) for x in op["ctx"]])
    merged = backend.new()
    for w in ws:
        backend.merge(merged, w)
    backend.merge(merged, backend.new())
    return ws, merged


def qc_fold(states, backend, trace=None):
    """Fold a logged witness list in index order into a new set, then the plunger."""
    merged = backend.new()
    for k, st in enumerate(states):
        backend.merge(merged, backend.load(st))
        if trace is not None:
            trace.append(backend.clone(merged))
    backend.merge(merged, backend.new())
    if trace is not None:
        trace.append(backend.clone(merged))
    return merged
