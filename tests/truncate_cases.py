"""Test inputs for Causal::truncate (src/orswot.rs:159-172): canonical Orswot
states (not necessarily reachable by ops: deferred clocks may cover member
dots, so apply_deferred can remove dots and the final subtract can EMPTY a
member clock) and truncating clocks, as records + numpy CSR clock batches,
plus the pure-Python restatement's result (oracle/crdts_ref.py)."""
import random

import numpy as np

import crdts_ref
import records


def random_state(rng, A, members=10, n_def=(0, 0, 1, 2, 3)):
    clock = {a: rng.randrange(1, 12) for a in range(A) if rng.random() < 0.8}
    entries = {}
    for m in rng.sample(range(1, 10_000), rng.randrange(0, members)):
        dots = {a: rng.randrange(1, c + 1) for a, c in clock.items() if rng.random() < 0.35}
        if dots:
            entries[m] = dots
    deferred = {}
    for _ in range(rng.choice(n_def)):
        d = {a: rng.randrange(1, 16) for a in range(A) if rng.random() < 0.3}
        if not d or all(clock.get(a, 0) >= c for a, c in d.items()):
            d[rng.randrange(A)] = 20 + rng.randrange(5)  # !(D <= clock): a pending remove
        ms = set(rng.sample(sorted(entries), min(len(entries), rng.randrange(1, 3)))) if entries else set()
        ms |= {rng.randrange(1, 10_000)}
        deferred[tuple(sorted(d.items()))] = ms
    return clock, entries, deferred


def truncating_clock(rng, A):
    return {a: rng.randrange(1, 14) for a in range(A) if rng.random() < 0.6}


def to_ref(state):
    clock, entries, deferred = state
    o = crdts_ref.Orswot()
    o.clock = crdts_ref.VClock(clock)
    o.entries = {m: crdts_ref.VClock(c) for m, c in entries.items()}
    o.deferred = {crdts_ref.VClock(list(k)): set(v) for k, v in deferred.items()}
    return o


def ref_state(o):
    """crdts_ref.Orswot -> (clock, entries, deferred) with sorted pairs (records.decode's shape)."""
    return (dict(o.clock.dots), {m: sorted(c.dots.items()) for m, c in o.entries.items()},
            sorted((tuple(sorted(k.dots.items())), sorted(v)) for k, v in o.deferred.items()))


def clocks_csr(clocks):
    runs = [sorted(c.items()) for c in clocks]
    ln = np.array([len(r) for r in runs], np.uint32)
    off = np.zeros(len(runs), np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    act = np.array([a for r in runs for a, _ in r] or [0], np.uint32)
    ctr = np.array([c for r in runs for _, c in r] or [1], np.uint64)
    return off, ln, act, ctr


def cases(n, A=8, seed=5, shapes=None):
    """shapes: optional list of random_state keyword sets, cycled over the n states."""
    rng = random.Random(seed)
    states = [random_state(rng, A, **(shapes[i % len(shapes)] if shapes else {})) for i in range(n)]
    clocks = [truncating_clock(rng, A) for _ in range(n)]
    recs = [records.encode(c, e, d, A) for c, e, d in states]
    return states, clocks, recs
