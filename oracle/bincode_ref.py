"""CPU restatement of the reference's binary form of an Orswot — TEST
INFRASTRUCTURE ONLY (tests/, bench.py's cpu_baseline leg). The product codec
is the HIP one behind crdt_orswot_{from,to}_bincode.

The reference serialises with `to_binary` / `from_binary` (src/lib.rs:62-83):
`bincode::serialize(s, Infinite)` / `bincode::deserialize` of the serde
derives on

    Orswot<M, A> { clock: VClock<A>,                           (src/orswot.rs:26-30)
                   entries: HashMap<M, VClock<A>>,
                   deferred: HashMap<VClock<A>, HashSet<M>> }
    VClock<A>    { dots: BTreeMap<A, u64> }                    (src/vclock.rs:54-57)

bincode 0.9 and serde 1.0 (Cargo.toml:17-20) are not vendored in
/root/reference and no Rust toolchain exists here, so their published data
format is restated: a struct is its fields in declaration order with no
framing; a map is its length as u64 followed by (key, value) pairs in the
map's iteration order (BTreeMap: ascending key; HashMap: arbitrary); a set is
its length as u64 followed by its elements; integers are fixed-width
little-endian. Actors and members here are unsigned integers of a fixed byte
width (u8/u16/u32/u64 in the reference's generic parameters).

Parity of exact bytes is unpinned by reference output (the reference's own
tests only assert to_binary -> from_binary round trips, src/lib.rs:53-60);
it is pinned to this restatement of the published format, and the round-trip
property is tested on every state the KAT suite and the generators produce.
"""
from __future__ import annotations

import random
import struct

_FMT = {1: "B", 2: "H", 4: "I", 8: "Q"}


def _int(w):
    return "<" + _FMT[w]


def encode(state, actor_bytes, member_bytes, rng: random.Random | None = None):
    """state: dict(clock={a: c}, entries={m: [(a, c), ...]}, deferred=[([(a, c)], [m])]).
    HashMap / HashSet iteration order is ascending unless rng is given (then
    shuffled, as a reference HashMap with a random SipHash key would be)."""
    fa, fm = _int(actor_bytes), _int(member_bytes)
    out = bytearray()

    def vclock(pairs):
        pairs = sorted(pairs)  # BTreeMap order
        out.extend(struct.pack("<Q", len(pairs)))
        for a, c in pairs:
            out.extend(struct.pack(fa, a))
            out.extend(struct.pack("<Q", c))

    vclock(list(state["clock"].items()))
    ents = sorted(state["entries"].items())
    if rng is not None:
        rng.shuffle(ents)
    out.extend(struct.pack("<Q", len(ents)))
    for m, dots in ents:
        out.extend(struct.pack(fm, m))
        vclock(list(dots))
    defs = [(sorted(c), sorted(ms)) for c, ms in state["deferred"]]
    defs.sort()
    if rng is not None:
        rng.shuffle(defs)
    out.extend(struct.pack("<Q", len(defs)))
    for c, ms in defs:
        vclock(c)
        ms = list(ms)
        if rng is not None:
            rng.shuffle(ms)
        out.extend(struct.pack("<Q", len(ms)))
        for m in ms:
            out.extend(struct.pack(fm, m))
    return bytes(out)


class FormatError(ValueError):
    pass


def decode(blob, actor_bytes, member_bytes):
    """bytes -> the same dict form (entries: member -> sorted [(a, c)])."""
    blob = bytes(blob)
    pos = 0
    fa, fm = _int(actor_bytes), _int(member_bytes)

    def take(fmt, n):
        nonlocal pos
        if pos + n > len(blob):
            raise FormatError("truncated")
        v = struct.unpack_from(fmt, blob, pos)[0]
        pos += n
        return v

    def vclock():
        n = take("<Q", 8)
        pairs, last = [], None
        for _ in range(n):
            a = take(fa, actor_bytes)
            c = take("<Q", 8)
            if last is not None and a <= last:
                raise FormatError("BTreeMap keys not increasing")
            last = a
            pairs.append((a, c))
        return pairs

    clock = dict(vclock())
    entries = {}
    for _ in range(take("<Q", 8)):
        m = take(fm, member_bytes)
        if m in entries:
            raise FormatError("duplicate member")
        entries[m] = vclock()
    deferred = []
    seen = set()
    for _ in range(take("<Q", 8)):
        c = vclock()
        if tuple(c) in seen:
            raise FormatError("duplicate deferred clock")
        seen.add(tuple(c))
        ms = [take(fm, member_bytes) for _ in range(take("<Q", 8))]
        if len(set(ms)) != len(ms):
            raise FormatError("duplicate set element")
        deferred.append((c, sorted(ms)))
    if pos != len(blob):
        raise FormatError("trailing bytes")
    deferred.sort()
    return dict(clock=clock, entries=entries, deferred=deferred)


def canonical(state):
    """The record's view of a state: no zero counters anywhere, no empty
    member clocks / deferred clocks / deferred sets (what crdt records hold)."""
    ok = all(c > 0 for c in state["clock"].values())
    ok = ok and all(d and all(c > 0 for _, c in d) for d in state["entries"].values())
    ok = ok and all(c and ms and all(x > 0 for _, x in c) for c, ms in state["deferred"])
    return ok
