"""ORACLE — TEST INFRASTRUCTURE ONLY.

Independent pure-Python restatement of the etsangsplk/rust-crdt (crate
`crdts` 1.3.0) types on the merge hot path. Used by tests/ to (a) run the
reference's own known-answer tests (transcribed into tests/golden/*.json) and
(b) cross-check the C++ oracle (oracle/ref_cpu.cpp) on small random cases.
Never imported by the product package.

Python dicts stand in for BTreeMap/HashMap; iteration order is irrelevant to
the results because every operation below is order-independent, and
structural equality is compared through `canonical()`.
"""
from __future__ import annotations


class VClock:
    """src/vclock.rs:54-57 — `dots: BTreeMap<A, u64>`."""

    __slots__ = ("dots",)

    def __init__(self, dots=None):
        self.dots = {}
        for a, c in (dots.items() if isinstance(dots, dict) else (dots or [])):
            self.witness(a, c)  # From<Vec<(A,u64)>> / FromIterator, :255-271

    def clone(self):
        v = VClock()
        v.dots = dict(self.dots)
        return v

    def get(self, a):  # :206-210
        return self.dots.get(a, 0)

    def witness(self, a, c):  # :159-163
        if not (self.get(a) >= c):
            self.dots[a] = c

    def inc(self, a):  # :182-185 -> Dot (actor, counter)
        return (a, self.get(a) + 1)

    def apply(self, dot):  # CmRDT for VClock :123-129
        self.witness(dot[0], dot[1])

    def merge(self, other):  # CvRDT :131-137
        for a, c in other.dots.items():
            self.witness(a, c)

    def __eq__(self, other):  # derive(PartialEq) :53
        return isinstance(other, VClock) and self.dots == other.dots

    def __hash__(self):
        return hash(tuple(sorted(self.dots.items())))

    def partial_cmp(self, other):  # :59-71 ; 0 Eq, 1 Greater, -1 Less, None
        if self == other:
            return 0
        if all(self.get(w) >= c for w, c in other.dots.items()):
            return 1
        if all(other.get(w) >= c for w, c in self.dots.items()):
            return -1
        return None

    def __le__(self, other):
        return self.partial_cmp(other) in (0, -1)

    def __lt__(self, other):
        return self.partial_cmp(other) == -1

    def __ge__(self, other):
        return self.partial_cmp(other) in (0, 1)

    def __gt__(self, other):
        return self.partial_cmp(other) == 1

    def is_empty(self):  # :213-215
        return not self.dots

    def intersection(self, other):  # :219-228
        v = VClock()
        v.dots = {a: c for a, c in self.dots.items() if other.get(a) == c}
        return v

    def subtract(self, other):  # :236-242
        for a, c in other.dots.items():
            if c >= self.get(a):
                self.dots.pop(a, None)

    def truncate(self, other):  # Causal for VClock :103-120
        for a in list(self.dots):
            m = min(self.dots[a], other.get(a))
            if m > 0:
                self.dots[a] = m
            else:
                del self.dots[a]

    def canonical(self):
        return tuple(sorted(self.dots.items()))


class GCounter:
    """src/gcounter.rs:26-28; merge :58-62; PartialEq is value-only :43-48."""

    def __init__(self):
        self.inner = VClock()

    def inc(self, actor):
        return self.inner.inc(actor)

    def apply(self, dot):
        self.inner.apply(dot)

    def merge(self, other):
        self.inner.merge(other.inner)

    def value(self):  # :76-78 (u64 sum)
        return sum(self.inner.dots.values()) & 0xFFFFFFFFFFFFFFFF


class PNCounter:
    """src/pncounter.rs:33-36; merge :90-95."""

    def __init__(self):
        self.p = GCounter()
        self.n = GCounter()

    def inc(self, actor):  # :103-105 -> (dot, Pos)
        return (self.p.inc(actor), True)

    def dec(self, actor):
        return (self.n.inc(actor), False)

    def apply(self, op):  # :80-87
        dot, pos = op
        (self.p if pos else self.n).apply(dot)

    def merge(self, other):
        self.p.merge(other.p)
        self.n.merge(other.n)

    def value(self):  # :117-119  (p as i64 - n as i64)
        def i64(x):
            x &= 0xFFFFFFFFFFFFFFFF
            return x - (1 << 64) if x >= (1 << 63) else x

        return i64(i64(self.p.value()) - i64(self.n.value()))


class Orswot:
    """src/orswot.rs:26-30."""

    def __init__(self):
        self.clock = VClock()
        self.entries = {}   # member -> VClock
        self.deferred = {}  # VClock -> set(member)

    def clone(self):
        o = Orswot()
        o.clock = self.clock.clone()
        o.entries = {m: c.clone() for m, c in self.entries.items()}
        o.deferred = {c.clone(): set(s) for c, s in self.deferred.items()}
        return o

    # --- op path (used to BUILD states; src/orswot.rs:61-85)
    def apply_add(self, dot, member):
        actor, counter = dot
        if self.clock.get(actor) >= counter:
            return
        self.entries.setdefault(member, VClock()).apply(dot)
        self.clock.apply(dot)
        self.apply_deferred()

    def apply_rm(self, clock, member):
        self.apply_remove(member, clock)

    def apply_remove(self, member, clock):  # :195-211
        if not (clock <= self.clock):
            drops = self.deferred.pop(clock, set())
            drops.add(member)
            self.deferred[clock.clone()] = drops
        existing = self.entries.pop(member, None)
        if existing is not None:
            existing.subtract(clock)
            if not existing.is_empty():
                self.entries[member] = existing

    def apply_deferred(self):  # :235-243
        deferred = {c.clone(): set(s) for c, s in self.deferred.items()}
        self.deferred = {}
        for clock, members in deferred.items():
            for m in members:
                self.apply_remove(m, clock)

    # --- read path (src/orswot.rs:213-233; contexts src/ctx.rs)
    def value(self):
        return set(self.entries)

    def read_add_clock(self):
        return self.clock.clone()

    def contains_rm_clock(self, member):
        c = self.entries.get(member)
        return c.clone() if c is not None else VClock()

    # --- the hot path: CvRDT::merge, src/orswot.rs:87-157
    def merge(self, other):
        other_remaining = {m: c.clone() for m, c in other.entries.items()}
        keep = {}
        for entry, clock in [(m, c.clone()) for m, c in self.entries.items()]:
            oc = other.entries.get(entry)
            if oc is None:
                if clock <= other.clock:
                    pass
                else:
                    keep[entry] = clock
            else:
                oc = oc.clone()
                common = clock.intersection(oc)
                clock.subtract(common)
                oc.subtract(common)
                clock.subtract(other.clock)
                oc.subtract(self.clock)
                common.merge(clock)
                common.merge(oc)
                if not common.is_empty():
                    keep[entry] = common
                del other_remaining[entry]
        for entry, clock in other_remaining.items():
            clock.subtract(self.clock)
            if not clock.is_empty():
                keep[entry] = clock
        for clock, members in other.deferred.items():
            ours = self.deferred.pop(clock, set())
            ours |= members
            self.deferred[clock.clone()] = ours
        self.entries = keep
        self.clock.merge(other.clock)
        self.apply_deferred()

    def truncate(self, clock):  # Causal for Orswot :159-172
        empty = Orswot()
        empty.clock = clock.clone()
        self.merge(empty)
        self.clock.subtract(clock)
        for c in self.entries.values():
            c.subtract(clock)

    def canonical(self):
        """Structural identity: (clock, sorted entries, deferred in CLOCK ORDER)."""
        return (
            self.clock.canonical(),
            tuple((m, self.entries[m].canonical()) for m in sorted(self.entries)),
            tuple(sorted((c.canonical(), tuple(sorted(s))) for c, s in self.deferred.items())),
        )

    def __eq__(self, other):
        return self.canonical() == other.canonical()
