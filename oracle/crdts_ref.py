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


class MVReg:
    """src/mvreg.rs:14-18 — `vals: Vec<(VClock, V)>`; equality is set-like (:74-96)."""

    def __init__(self):
        self.vals = []

    def clone(self):
        r = MVReg()
        r.vals = [(c.clone(), v) for c, v in self.vals]
        return r

    def truncate(self, clock):  # Causal :100-113
        out = []
        for c, v in self.vals:
            c = c.clone()
            c.subtract(clock)
            if not c.is_empty():
                out.append((c, v))
        self.vals = out

    def merge(self, other):  # CvRDT :121-153
        vals = [(c.clone(), v) for c, v in self.vals if not any(c < oc for oc, _ in other.vals)]
        for c, v in other.vals:
            if any(c < sc for sc, _ in self.vals):
                continue
            if all(ec != c for ec, _ in vals):
                vals.append((c.clone(), v))
        self.vals = vals

    def apply_put(self, clock, val):  # CmRDT Op::Put :158-186
        if clock.is_empty():
            return
        self.vals = [(c, v) for c, v in self.vals if not (c <= clock)]
        if not any(c > clock for c, _ in self.vals):
            self.vals.append((clock.clone(), val))

    def read(self):
        return [v for _, v in self.vals]

    def canonical(self):
        return ("mvreg", tuple(sorted((c.canonical(), v) for c, v in self.vals)))


def clock_order(clocks):
    """CLOCK ORDER: lexicographic over the sorted (actor, counter) pairs."""
    return sorted(clocks, key=lambda c: c.canonical())


class Map:
    """src/map.rs:82-98 — Map<K, V, A> with V = MVReg or Orswot (`factory`).

    `order` is the iteration order apply_deferred (:325-333) takes over the
    deferred clocks — a HashMap in the reference, so unspecified; default
    CLOCK ORDER. With Orswot values the order can matter (see
    tests/test_map_orswot.py)."""

    def __init__(self, factory, order=clock_order):
        self.factory = factory
        self.order = order
        self.clock = VClock()
        self.entries = {}   # key -> [entry clock, val]   (BTreeMap)
        self.deferred = {}  # VClock -> set(key)          (HashMap<VClock, BTreeSet<K>>)

    def clone(self):
        m = Map(self.factory, self.order)
        m.clock = self.clock.clone()
        m.entries = {k: [c.clone(), v.clone()] for k, (c, v) in self.entries.items()}
        m.deferred = {c.clone(): set(s) for c, s in self.deferred.items()}
        return m

    def truncate(self, clock):  # Causal :131-158
        for k in list(self.entries):
            c, v = self.entries[k]
            c.subtract(clock)
            if c.is_empty():
                del self.entries[k]
            else:
                v.truncate(clock)
        d = {}
        for c, s in self.deferred.items():
            c = c.clone()
            c.subtract(clock)
            if not c.is_empty():
                d[c] = set(s)
        self.deferred = d
        self.clock.subtract(clock)

    # --- op path (src/map.rs:160-190, 304-323; ctx src/ctx.rs:45-60)
    def get(self, key):
        """ReadCtx: (add_clock, rm_clock, val or None), :291-302."""
        e = self.entries.get(key)
        return self.clock.clone(), (e[0].clone() if e else VClock()), (e[1] if e else None)

    def apply_up(self, dot, key, inner):
        """Op::Up {dot, key, op}: `inner(val)` applies the nested op (:169-187)."""
        actor, counter = dot
        if self.clock.get(actor) >= counter:
            return
        c, v = self.entries.pop(key, [VClock(), self.factory()])
        c.witness(actor, counter)
        inner(v)
        self.entries[key] = [c, v]
        self.clock.witness(actor, counter)
        self.apply_deferred()

    def apply_rm(self, key, clock):  # :336-350
        if not (clock <= self.clock):
            self.deferred.setdefault(clock.clone(), set()).add(key)
        e = self.entries.pop(key, None)
        if e is not None:
            c, v = e
            c.subtract(clock)
            if not c.is_empty():
                v.truncate(clock)
                self.entries[key] = [c, v]

    def apply_deferred(self):  # :325-333, in `order`
        d = {c.clone(): set(s) for c, s in self.deferred.items()}
        self.deferred = {}
        for c in self.order(list(d)):
            for k in sorted(d[c]):
                self.apply_rm(k, c)

    # --- CvRDT::merge :193-268
    def merge(self, other):
        other_remaining = {k: [c.clone(), v.clone()] for k, (c, v) in other.entries.items()}
        keep = {}
        for key, (c, v) in [(k, (c.clone(), v.clone())) for k, (c, v) in self.entries.items()]:
            oe = other.entries.get(key)
            if oe is None:
                c.subtract(other.clock)
                if not c.is_empty():
                    deleted = other.clock.clone()
                    deleted.subtract(c)
                    v.truncate(deleted)
                    keep[key] = [c, v]
            else:
                oc, ov = oe[0].clone(), oe[1].clone()
                common = c.intersection(oc)
                c.subtract(common)
                oc.subtract(common)
                c.subtract(other.clock)
                oc.subtract(self.clock)
                common.merge(c)
                common.merge(oc)
                if not common.is_empty():
                    v.merge(ov)
                    deleted = c.clone()
                    deleted.merge(oc)
                    deleted.subtract(common)
                    v.truncate(deleted)
                    keep[key] = [common, v]
                del other_remaining[key]
        for key, (c, v) in other_remaining.items():
            c.subtract(self.clock)
            if not c.is_empty():
                deleted = self.clock.clone()
                deleted.subtract(c)
                v.truncate(deleted)
                keep[key] = [c, v]
        for clock, keys in other.deferred.items():  # apply_rm on the old entries: only the deferral lasts
            for k in sorted(keys):
                self.apply_rm(k, clock)
        self.entries = keep
        self.clock.merge(other.clock)
        self.apply_deferred()

    def canonical(self):
        return (self.clock.canonical(),
                tuple((k, c.canonical(), v.canonical()) for k, (c, v) in sorted(self.entries.items())),
                tuple(sorted((c.canonical(), tuple(sorted(s))) for c, s in self.deferred.items())))

    def __eq__(self, other):
        return self.canonical() == other.canonical()
