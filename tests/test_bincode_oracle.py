"""CPU tests of the bincode restatement (oracle/bincode_ref.py) that pins the
GPU ingest / egest codec (crdt_orswot_{from,to}_bincode), and of the
product's host-side helpers for it. SURVEY.md §8(f) rank 1."""
import os
import random
import struct
import sys

import pytest

import records

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import bincode_ref as BC  # noqa: E402

WIDTHS = [(1, 8), (2, 8), (4, 4), (8, 8)]


def _states(n=200, seed=1, sparse=False):
    import crdts_hip

    if sparse:
        (b, o), _ = crdts_hip.generate_replicas(n, 2, threads=4)
    else:
        (b, o), _ = crdts_hip.generate_orswot(n, first_obj=seed, threads=4)
    return [records.decode(r) for r in records.unpack_batch(b, o)]


def small_members(st):
    """The same state with member keys replaced by their rank (order kept)."""
    keys = sorted(set(st["entries"]) | {m for _, ms in st["deferred"] for m in ms})
    r = {k: i + 1 for i, k in enumerate(keys)}
    return dict(clock=st["clock"], entries={r[m]: d for m, d in st["entries"].items()},
                deferred=[(c, [r[m] for m in ms]) for c, ms in st["deferred"]])


def _fits(st, wa, wm):
    amax, mmax = (1 << (8 * wa)) - 1, (1 << (8 * wm)) - 1
    acts = list(st["clock"]) + [a for d in st["entries"].values() for a, _ in d] + \
        [a for c, _ in st["deferred"] for a, _ in c]
    mems = list(st["entries"]) + [m for _, ms in st["deferred"] for m in ms]
    return all(a <= amax for a in acts) and all(m <= mmax for m in mems)


def test_doc_example_bytes():
    """src/lib.rs:53-60: Orswot<u8, u8> after one add of member 1 by actor 1.
    Bytes derived from the format restatement (not from reference output)."""
    st = dict(clock={1: 1}, entries={1: [(1, 1)]}, deferred=[])
    b = BC.encode(st, 1, 1)
    exp = (struct.pack("<Q", 1) + b"\x01" + struct.pack("<Q", 1) +      # clock {1: 1}
           struct.pack("<Q", 1) + b"\x01" + struct.pack("<Q", 1) + b"\x01" + struct.pack("<Q", 1) +  # entries
           struct.pack("<Q", 0))                                        # deferred {}
    assert b == exp and len(b) == 51
    assert BC.decode(b, 1, 1) == st


@pytest.mark.parametrize("wa,wm", WIDTHS)
def test_round_trip_generator_states(wa, wm):
    rng = random.Random(wa * 10 + wm)
    n = 0
    for st in _states(300, seed=wa):
        st = st if wm == 8 else small_members(st)
        if not _fits(st, wa, wm):
            continue
        n += 1
        want = dict(clock=st["clock"], entries=st["entries"], deferred=st["deferred"])
        assert BC.decode(BC.encode(want, wa, wm), wa, wm) == want
        assert BC.decode(BC.encode(want, wa, wm, rng=rng), wa, wm) == want  # any HashMap order
    assert n > 100


def test_round_trip_sparse_states():
    for st in _states(100, sparse=True):
        want = dict(clock=st["clock"], entries=st["entries"], deferred=st["deferred"])
        assert BC.decode(BC.encode(want, 2, 8, rng=random.Random(3)), 2, 8) == want


def test_deferred_states_present():
    sts = _states(2000)
    assert sum(1 for s in sts if s["deferred"]) > 20


@pytest.mark.parametrize("damage", ["truncate", "trailing", "dup_member", "clock_order", "dup_set"])
def test_malformed(damage):
    st = dict(clock={1: 3, 2: 4}, entries={7: [(1, 3)], 9: [(2, 4)]}, deferred=[([(3, 1)], [5, 6])])
    b = bytearray(BC.encode(st, 1, 1))
    if damage == "truncate":
        b = b[:-1]
    elif damage == "trailing":
        b += b"\x00"
    elif damage == "dup_member":
        b[8 + 2 * 9 + 8 + 18] = 7          # second member key := 7
    elif damage == "clock_order":
        b[8], b[17] = 2, 1                  # BTreeMap keys 2, 1
    elif damage == "dup_set":
        b[-1] = 5                            # set {5, 5}
    with pytest.raises(BC.FormatError):
        BC.decode(bytes(b), 1, 1)


def test_record_form_agrees():
    """decode(encode(record state)) re-encodes to the same canonical record."""
    for st in _states(200, seed=9):
        back = BC.decode(BC.encode(st, 1, 8, rng=random.Random(1)), 1, 8)
        rec = records.encode(back["clock"], {m: dict(d) for m, d in back["entries"].items()},
                             {tuple(c): set(ms) for c, ms in back["deferred"]}, 16)
        assert records.decode(rec)["entries"] == st["entries"]
        assert records.decode(rec)["deferred"] == st["deferred"]


def test_cpp_restatement_agrees(oracle):
    """The C++ restatement (the CPU baseline's) and the Python one decode every
    blob to the same canonical record, for dense and sparse states."""
    rng = random.Random(11)
    for st in _states(300, seed=21):
        blob = BC.encode(dict(clock=st["clock"], entries=st["entries"], deferred=st["deferred"]), 1, 8, rng=rng)
        assert oracle.bincode_to_record(blob, 1, 8, 16) == records.encode(
            st["clock"], {m: dict(d) for m, d in st["entries"].items()},
            {tuple(c): set(ms) for c, ms in st["deferred"]}, 16)
    for st in _states(100, sparse=True):
        blob = BC.encode(dict(clock=st["clock"], entries=st["entries"], deferred=st["deferred"]), 2, 8, rng=rng)
        assert oracle.bincode_to_record(blob, 2, 8, 1024, 1) == records.encode(
            st["clock"], {m: dict(d) for m, d in st["entries"].items()},
            {tuple(c): set(ms) for c, ms in st["deferred"]}, 1024, True)


def extreme_state(rng, A, wa, wm):
    """A state stressing one bound term or another: many one-dot members,
    big deferred sets of narrow members, several deferred clocks, or empty."""
    alim = min(A, 1 << (8 * wa)) if wa < 8 else A
    acts = rng.sample(range(alim), rng.choice([1, 2, min(5, alim), min(16, alim)]))
    mlim = 1 << (8 * wm) if wm < 8 else 1 << 40
    ents = {}
    for _ in range(rng.choice([0, 1, 40])):
        ents[rng.randrange(mlim)] = sorted((a, rng.randrange(1, 9))
                                           for a in rng.sample(acts, rng.randrange(1, len(acts) + 1)))
    clock = {}
    for d in ents.values():
        for a, c in d:
            clock[a] = max(clock.get(a, 0), c)
    deferred, seen = [], set()
    for _ in range(rng.choice([0, 1, 8])):
        dc = tuple(sorted((a, rng.randrange(10, 20)) for a in rng.sample(acts, rng.randrange(1, len(acts) + 1))))
        if dc not in seen:
            seen.add(dc)
            deferred.append((list(dc), sorted({rng.randrange(mlim) for _ in range(rng.choice([1, 30]))})))
    return dict(clock=clock, entries=ents, deferred=deferred)


def bincode_record_bound(L, wa, wm, A, sparse):
    """Mirror of bc_record_bound (rust-crdt_amd/csrc/bincode.hip): the record
    bytes of any blob of L bytes are at most 48 + 8 A (dense) + ceil(c L),
    c = max(12 / (wa + 8), 12 / (wm + 8), 8 / wm), rounded up to 16."""
    c = max(-(-12 * L // (wa + 8)), -(-12 * L // (wm + 8)), -(-8 * L // wm))
    return (48 + (0 if sparse else 8 * A) + c + 15) // 16 * 16


@pytest.mark.parametrize("wa,wm", [(1, 1), (1, 8), (2, 2), (8, 1), (8, 8), (4, 2)])
@pytest.mark.parametrize("sparse", [False, True])
def test_record_bound_holds(wa, wm, sparse):
    """The placement bound behind crdt_orswot_bincode_record_bounds, against
    the real record size, on shapes that stress each of its terms."""
    import random

    rng = random.Random(wa * 10 + wm + sparse)
    A = 256 if sparse else 16
    for _ in range(2000):
        st = extreme_state(rng, A, wa, wm)
        L = len(BC.encode(st, wa, wm))
        rec = records.encode(st["clock"], {m: dict(d) for m, d in st["entries"].items()},
                             {tuple(c): set(ms) for c, ms in st["deferred"]}, A, sparse)
        assert len(rec) <= bincode_record_bound(L, wa, wm, A, sparse), (len(rec), L, st)
