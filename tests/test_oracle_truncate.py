"""CPU: the C++ oracle's Causal::truncate (oracle/ref_cpu.cpp Orswot::truncate,
src/orswot.rs:159-172) against the independent Python restatement
(oracle/crdts_ref.py) on random canonical states — including states whose
deferred clocks cover member dots, where truncate leaves a member with an
EMPTY clock (the record carries CRDT_ORSWOT_EMPTY_MEMBER_CLOCK)."""
import numpy as np

import oracle_ffi
import records
import truncate_cases as T


def _decode_all(ob, oo):
    return [records.decode(r) for r in records.unpack_batch(ob, oo)]


def test_cpp_oracle_matches_python_restatement():
    states, clocks, recs = T.cases(3000)
    lb, lo = records.pack_batch(recs)
    ob, oo = oracle_ffi.orswot_truncate_batch(lb, lo, T.clocks_csr(clocks), 8)
    got = _decode_all(ob, oo)
    empties = 0
    for st, c, g in zip(states, clocks, got):
        o = T.to_ref(st)
        o.truncate(oracle_ffi_clock(c))
        clock, entries, deferred = T.ref_state(o)
        assert g["clock"] == clock
        assert {m: list(v) for m, v in g["entries"].items()} == entries
        assert sorted((tuple(k), sorted(v)) for k, v in g["deferred"]) == deferred
        empties += any(len(v) == 0 for v in entries.values())
    assert empties > 20  # the empty-member-clock case is exercised
    flags = [int(np.frombuffer(r[28:32], np.uint32)[0]) for r in records.unpack_batch(ob, oo)]
    assert sum(f & 2 for f in flags) // 2 == empties


def oracle_ffi_clock(c):
    import crdts_ref

    return crdts_ref.VClock(c)
