"""The roofline numerator (bench.py): SURVEY.md §8(d)'s compact algorithmic
bytes, computed from record headers (crdts_hip.record.batch_compact_bytes on
the host, OrswotBatch.compact_bytes on the device), equal the formula applied
to the oracle's decoded states — inputs and the oracle's merged outputs, dense
(config 3) and sparse (config 5) — on a sample."""
import numpy as np

import records


def _formula(d, A, sparse):
    """bytes(side) = top + 4 + 4 + Σ_members(8 + 4 + 12·dots) + Σ_deferred(4 + 12·dots + 4 + 8·members)."""
    top = 4 + 12 * len(d["clock"]) if sparse else 8 * A
    mem = sum(8 + 4 + 12 * len(c) for c in d["entries"].values())
    dfr = sum(4 + 12 * len(p) + 4 + 8 * len(m) for p, m in d["deferred"])
    return top + 8 + mem + dfr


def _check(base, off, A, sparse):
    from crdts_hip.record import batch_compact_bytes

    want = sum(_formula(records.decode(r), A, sparse) for r in records.unpack_batch(base, off))
    assert batch_compact_bytes(base, off) == want
    return want


def test_config3_sample(oracle):
    import crdts_hip

    n = 3000
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(n, threads=8)
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, 16, threads=8)
    tot = _check(lb, lo, 16, False) + _check(rb, ro, 16, False) + _check(ob, oo, 16, False)
    assert 2700 < tot / n < 2950  # ~2 818 B per merge at full size


def test_config5_sample(oracle):
    import crdts_hip

    U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
    reps = crdts_hip.generate_replicas(1500, 2, threads=8)
    ob, oo = oracle.orswot_merge_batch(reps[0][0], reps[0][1], reps[1][0], reps[1][1], U, threads=8, flags=SP)
    for b, o in (reps[0], reps[1], (ob, oo)):
        _check(b, o, U, True)


def test_device_form_matches_host():
    import crdts_hip
    from crdts_hip.record import batch_compact_bytes

    (lb, lo), _ = crdts_hip.generate_orswot(500, threads=4)
    B = crdts_hip.OrswotBatch.from_host(lb, lo, 16, device="cpu")
    assert B.compact_bytes() == batch_compact_bytes(lb, lo)
