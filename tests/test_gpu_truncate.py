"""GPU parity: batched Causal::truncate for Orswot (crdt_orswot_truncate,
src/orswot.rs:159-172) vs the oracle's Orswot::truncate, byte-exact: random
canonical states incl. deferred clocks that cover member dots, where truncate
leaves members with EMPTY clocks (CRDT_ORSWOT_EMPTY_MEMBER_CLOCK, kept as in
the reference); config-3 states truncated by the other replica's top clock
(the Map case: the remover's clock) and by partial clocks; CSR (config 5)
records; and a record with an empty member clock rejected by the merge."""
import random

import numpy as np
import pytest

import records
import truncate_cases as T

pytestmark = pytest.mark.gpu


def _check(gpu, oracle, lb, lo, clocks_np, A, flags=0):
    import crdts_hip

    B = crdts_hip.OrswotBatch.from_host(lb, lo, A, flags=flags)
    C = crdts_hip.ClockBatch.from_host(*clocks_np)
    out = gpu.orswot_truncate(B, C)
    got = out.records()
    ob, oo = oracle.orswot_truncate_batch(lb, lo, clocks_np, A, flags, threads=16)
    exp = records.unpack_batch(ob, oo)
    bad = [i for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not bad, f"{len(bad)}/{len(exp)} differ; first {bad[0]}: {records.decode(got[bad[0]])} vs " \
                    f"{records.decode(exp[bad[0]])}"
    assert (out.off.cpu().numpy().view(np.uint64) == lo.astype(np.uint64)).all()  # written in place of the input
    return exp


def test_random_states_incl_empty_member_clocks(gpu, oracle):
    states, clocks, recs = T.cases(20_000, seed=9)
    lb, lo = records.pack_batch(recs)
    exp = _check(gpu, oracle, lb, lo, T.clocks_csr(clocks), 8)
    flags = [int(np.frombuffer(r[28:32], np.uint32)[0]) for r in exp]
    assert sum(1 for f in flags if f & 2) > 100  # empty member clocks occur and match


@pytest.mark.parametrize("A", [8, 40])
def test_both_kernel_forms_in_one_batch(gpu, oracle, A):
    """The kernel stages a record in LDS when it is dense, A <= 32, <= 4 KB and
    has <= 8 deferred clocks, else reads it from HBM: at A = 8 one batch mixes
    ordinary records with ones of 9-12 deferred clocks and > 4 KB ones (150-300
    members); at A = 40 every record takes the HBM form."""
    shapes = [{}, {"n_def": (9, 10, 12)}, {"members": 300}, {}]
    states, clocks, recs = T.cases(4_000, A=A, seed=17, shapes=shapes)
    assert max(len(r) for r in recs) > 4096 and max(len(s[2]) for s in states) > 8
    lb, lo = records.pack_batch(recs)
    _check(gpu, oracle, lb, lo, T.clocks_csr(clocks), A)


def test_config3_truncated_by_the_other_replicas_clock(gpu, oracle):
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(50_000, threads=16, seed=12)
    rng = random.Random(3)
    clocks = []
    for i, r in enumerate(records.unpack_batch(rb, ro)):
        c = records.decode(r)["clock"]
        if i % 3 == 1:  # a partial clock: some actors dropped, some counters lowered
            c = {a: max(1, v - rng.randrange(3)) for a, v in c.items() if rng.random() < 0.7}
        elif i % 3 == 2:
            c = {}
        clocks.append(c)
    _check(gpu, oracle, lb, lo, T.clocks_csr(clocks), 16)


def test_sparse_records(gpu, oracle):
    import crdts_hip

    U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
    reps = crdts_hip.generate_replicas(20_000, 2, threads=16)
    clocks = [records.decode(r)["clock"] for r in records.unpack_batch(*reps[1])]
    _check(gpu, oracle, reps[0][0], reps[0][1], T.clocks_csr(clocks), U, SP)


def test_empty_member_clock_rejected_by_merge(gpu, oracle):
    import crdts_hip
    from crdts_hip._lib import CRDT_ENONCANON

    # entry {a:5, b:1}, deferred {a:6} naming it (pending: a:6 > clock's a:5), c = {a:3, b:2}:
    # the deferred subtract removes a:5, the final subtract b:1 -> an empty clock
    rec = records.encode({0: 5, 1: 1}, {7: {0: 5, 1: 1}}, {((0, 6),): {7}}, 4)
    lb, lo = records.pack_batch([rec])
    exp = _check(gpu, oracle, lb, lo, T.clocks_csr([{0: 3, 1: 2}]), 4)
    d = records.decode(exp[0])
    assert d["entries"] == {7: []} and d["flags"] & 2
    B = crdts_hip.OrswotBatch.from_host(*records.pack_batch(exp), 4)
    with pytest.raises(crdts_hip.CrdtError) as e:
        gpu.orswot_merge(B, B)
    assert e.value.code == CRDT_ENONCANON


@pytest.mark.parametrize("A,shape", [(4, {"members": 90, "n_def": (0,)}), (16, {"members": 12, "n_def": (0,)}),
                                     (8, {"members": 10, "n_def": (0, 1)})])
def test_single_pass_form_and_its_limits(gpu, oracle, A, shape):
    """Records without deferred removes, <= 64 members of <= 4 dots take the
    single-pass LDS form (output assembled over the stage, 16-B copy-out);
    past 64 members (A = 4, up to 89 members in < 4 KB) or with a member of
    more than 4 dots (A = 16) the two-pass form — mixed in one batch with
    records that have deferred removes."""
    states, clocks, recs = T.cases(6_000, A=A, seed=23 + A, shapes=[shape, {}])
    n_mem = [len(s[1]) for s in states]
    most = [max((len(c) for c in s[1].values()), default=0) for s in states]
    if A == 4:
        assert sum(1 for n, r in zip(n_mem, recs) if n > 64 and len(r) <= 4096) > 100
    if A == 16:
        assert sum(1 for m in most if m > 4) > 100
    lb, lo = records.pack_batch(recs)
    _check(gpu, oracle, lb, lo, T.clocks_csr(clocks), A)


@pytest.mark.parametrize("A,shapes", [(8, None), (40, None), (8, [{}, {"members": 300}])])
def test_truncate_twice(gpu, oracle, A, shapes):
    """A record truncate wrote (possibly with empty member clocks, header flag
    bit 1) is a valid input of truncate: the reference's Map calls
    val.truncate again on a nested Orswot (src/map.rs apply_rm / truncate) and
    drops the empty-clock members then (empty <= c). Both kernel forms (A = 8:
    LDS and HBM; A = 40: HBM), byte-exact vs the oracle's second truncate."""
    import crdts_hip

    states, clocks, recs = T.cases(6_000, A=A, seed=31 + A, shapes=shapes)
    lb, lo = records.pack_batch(recs)
    first = _check(gpu, oracle, lb, lo, T.clocks_csr(clocks), A)
    assert sum(1 for r in first if np.frombuffer(r[28:32], np.uint32)[0] & 2) > 50
    rng = random.Random(A)
    again = [{a: v + rng.randrange(3) for a, v in c.items() if rng.random() < 0.8} for c in clocks]
    lb2, lo2 = records.pack_batch(first)
    second = _check(gpu, oracle, lb2, lo2, T.clocks_csr(again), A)
    # the handmade case of test_empty_member_clock_rejected_by_merge, truncated again
    rec = records.encode({0: 5, 1: 1}, {7: {0: 5, 1: 1}}, {((0, 6),): {7}}, 4)
    one = _check(gpu, oracle, *records.pack_batch([rec]), T.clocks_csr([{0: 3, 1: 2}]), 4)
    two = _check(gpu, oracle, *records.pack_batch(one), T.clocks_csr([{1: 1}]), 4)
    assert records.decode(two[0])["entries"] == {} and not records.decode(two[0])["flags"] & 2
    B = crdts_hip.OrswotBatch.from_host(*records.pack_batch(two), 4)
    assert gpu.orswot_merge(B, B).records() == two  # canonical again: the merge takes it


@pytest.mark.parametrize("A", [8, 40])
@pytest.mark.parametrize("bad", ["unsorted", "duplicate", "zero", "unsorted_past_64"])
def test_noncanonical_clock_run_rejected(gpu, A, bad):
    """A truncating clock run whose actors are not strictly increasing or that
    holds a zero counter latches CRDT_ENONCANON (crdts_hip.h), in the LDS form
    (A = 8) and the HBM form (A = 40); a run longer than 64 entries is checked
    past its first 64 too."""
    import crdts_hip
    from crdts_hip._lib import CRDT_ENONCANON

    states, clocks, recs = T.cases(200, A=A, seed=41)
    off, ln, act, ctr = T.clocks_csr(clocks)
    k = 117
    if bad == "unsorted_past_64":
        run = [(a, 3) for a in range(70)]
        run[66], run[67] = run[67], run[66]
    else:
        run = [(0, 2), (2, 5), (5, 1)]
        if bad == "unsorted":
            run[1], run[2] = run[2], run[1]
        elif bad == "duplicate":
            run[2] = (2, 7)
        else:
            run[1] = (2, 0)
    runs = [sorted(c.items()) for c in clocks]
    runs[k] = run
    ln = np.array([len(r) for r in runs], np.uint32)
    off = np.zeros(len(runs), np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    act = np.array([a for r in runs for a, _ in r], np.uint32)
    ctr = np.array([c for r in runs for _, c in r], np.uint64)
    lb, lo = records.pack_batch(recs)
    B = crdts_hip.OrswotBatch.from_host(lb, lo, A)
    C = crdts_hip.ClockBatch.from_host(off, ln, act, ctr)
    with pytest.raises(crdts_hip.CrdtError) as e:
        gpu.orswot_truncate(B, C)
    assert e.value.code == CRDT_ENONCANON


def test_out_aliasing_the_input_rejected(gpu):
    """crdt_orswot_truncate is not in place: an output range overlapping the
    input records is CRDT_EINVAL (checked before any launch)."""
    import crdts_hip
    from crdts_hip._lib import CRDT_EINVAL

    states, clocks, recs = T.cases(300, A=40, seed=3)
    B = crdts_hip.OrswotBatch.from_host(*records.pack_batch(recs), 40)
    C = crdts_hip.ClockBatch.from_host(*T.clocks_csr(clocks))
    with pytest.raises(crdts_hip.CrdtError) as e:
        gpu.orswot_truncate(B, C, out=B)
    assert e.value.code == CRDT_EINVAL
    gpu.orswot_truncate(B, C)  # the context is still usable


@pytest.mark.parametrize("A", [8, 16, 32])
def test_fast_form_with_deferred_clocks(gpu, oracle, A):
    """The streaming fast form (orswot_truncate_fast_kernel) takes dense
    records of <= 64 members / dots with up to 8 deferred clocks: deferred
    clocks that cover member dots (dots killed, members kept with an EMPTY
    clock), clocks re-deferred or dropped against max(T, c) — mixed in one
    batch with records past its limits (9-12 deferred clocks, 100+ members)
    that the general form takes; byte-exact vs the oracle."""
    shapes = [{"n_def": (1, 2, 3, 8)}, {}, {"n_def": (9, 12)}, {"members": 120}]
    states, clocks, recs = T.cases(8_000, A=A, seed=61 + A, shapes=shapes)
    n_def = [len(s[2]) for s in states]
    assert sum(1 for d in n_def if 1 <= d <= 8) > 2000 and sum(1 for d in n_def if d > 8) > 500
    lb, lo = records.pack_batch(recs)
    exp = _check(gpu, oracle, lb, lo, T.clocks_csr(clocks), A)
    assert sum(1 for r in exp if np.frombuffer(r[28:32], np.uint32)[0] & 2) > 100
    try:  # the records the fast form leaves reach the general form listed, or (list full) by their flags
        for cap in (8, 0):
            gpu.set_list_cap(cap)
            _check(gpu, oracle, lb, lo, T.clocks_csr(clocks), A)
    finally:
        gpu.set_list_cap(65536)
