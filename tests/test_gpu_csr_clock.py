"""GPU parity: sparse (CSR) VClock / GCounter / PNCounter merge through the C
ABI (crdt_vclock_csr_merge / crdt_gcounter_csr_merge / crdt_pncounter_csr_merge)
vs the oracle (VClock::merge over std::map, src/vclock.rs:131-137), byte-exact:
the reference's merge KATs in CSR form, a 1024-actor universe with ~48 actors
per clock, empty and > 64-entry runs (the chunked path), gapped inputs (a
merge output merged again), non-canonical and misplaced runs, and at full
size the properties the join has (idempotent, commutative: VClock::merge is a
pointwise max)."""
import json
import os

import numpy as np
import pytest

from test_oracle_csr import csr, dict_merge, unpack, witnessed

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _gpu_merge(gpu, s, o, kind="vclock"):
    import crdts_hip

    S = crdts_hip.ClockBatch.from_host(*s)
    O = crdts_hip.ClockBatch.from_host(*o)
    return gpu.clock_csr_merge(S, O, kind=kind)


def test_reference_kats_csr_on_gpu(gpu):
    kats = [k for k in json.load(open(os.path.join(GOLDEN, "kat_vclock_counters.json")))["vclock_binop"]
            if k["op"] == "merge"]
    out = _gpu_merge(gpu, csr([witnessed(k["a"]) for k in kats]), csr([witnessed(k["b"]) for k in kats]))
    for k, g in zip(kats, out.clocks()):
        assert g == [tuple(x) for x in k["expect"]], k["name"]


@pytest.mark.parametrize("kind", ["vclock", "gcounter"])
def test_universe_1024_vs_oracle(gpu, oracle, kind):
    import crdts_hip

    s, o = crdts_hip.generate_clocks_csr(100_003, seed=11)
    out = _gpu_merge(gpu, s, o, kind)
    eo, el, ea, ec = oracle.vclock_csr_merge(s, o, threads=16)
    go, gl, ga, gc = out.to_host()
    assert (go == eo).all() and (gl == el).all()
    used = np.zeros(len(ea), bool)  # compare the written entries only (gaps are unspecified)
    idx = np.repeat(eo.astype(np.int64), el.astype(np.int64)) + (
        np.arange(int(el.sum())) - np.repeat(np.cumsum(el.astype(np.int64)) - el.astype(np.int64), el.astype(np.int64)))
    used[idx] = True
    assert (ga[used] == ea[used]).all() and (gc[used] == ec[used]).all()


def test_empty_long_and_edge_runs(gpu, oracle):
    rng = np.random.default_rng(7)

    def rnd(n, universe=100_000):
        return {int(x): int(rng.integers(1, 1 << 62)) for x in rng.choice(universe, n, replace=False)}

    A = [{}, {5: 1}, {}, rnd(64), rnd(65), rnd(700), rnd(1000), rnd(3), rnd(64), {0: 1, (1 << 32) - 1: 2}]
    B = [{}, {}, {7: 2}, rnd(64), rnd(64), rnd(900), rnd(10), rnd(1000), rnd(65), {(1 << 32) - 1: 5}]
    A[8].update({k: v + 1 for k, v in list(B[8].items())[:30]})  # equal actors across the chunk boundary
    B[6].update({k: v for k, v in list(A[6].items())[:5]})
    out = _gpu_merge(gpu, csr(A), csr(B))
    assert out.clocks() == [dict_merge(a, b) for a, b in zip(A, B)]
    assert out.clocks() == unpack(oracle.vclock_csr_merge(csr(A), csr(B)))


def test_gapped_input_and_chained_fold(gpu, oracle):
    """A merge output (runs at s.off + o.off, gaps between them) is a valid
    input: ((a ⊔ b) ⊔ c) on the GPU equals the oracle's fold."""
    import crdts_hip

    a, b = crdts_hip.generate_clocks_csr(20_000, seed=21)
    c, _ = crdts_hip.generate_clocks_csr(20_000, seed=22)
    ab = _gpu_merge(gpu, a, b)
    abc = gpu.clock_csr_merge(ab, crdts_hip.ClockBatch.from_host(*c))
    e_ab = oracle.vclock_csr_merge(a, b)
    e_abc = oracle.vclock_csr_merge(e_ab, c)
    assert abc.clocks() == unpack(e_abc)


def test_properties_full_size(gpu):
    """1M clocks per side: x ⊔ x = x, and a ⊔ b = b ⊔ a entry for entry
    (VClock::merge is a pointwise max over the actor union)."""
    import torch

    import crdts_hip

    s, o = crdts_hip.generate_clocks_csr(1_000_000, seed=31)
    S, O = crdts_hip.ClockBatch.from_host(*s), crdts_hip.ClockBatch.from_host(*o)
    xx = gpu.clock_csr_merge(S, S)
    assert torch.equal(xx.len, S.len)
    ab, ba = gpu.clock_csr_merge(S, O), gpu.clock_csr_merge(O, S)
    assert torch.equal(ab.len, ba.len)
    ha, hb = ab.to_host(), ba.to_host()
    ln = ha[1].astype(np.int64)
    start = np.repeat(np.cumsum(ln) - ln, ln)
    k = np.arange(int(ln.sum())) - start
    ia = np.repeat(ha[0].astype(np.int64), ln) + k
    ib = np.repeat(hb[0].astype(np.int64), ln) + k
    assert (ha[2][ia] == hb[2][ib]).all() and (ha[3][ia] == hb[3][ib]).all()
    hs = S.to_host()
    ixx = np.repeat(xx.to_host()[0].astype(np.int64), hs[1].astype(np.int64)) + (
        np.arange(int(hs[1].sum())) - np.repeat(np.cumsum(hs[1].astype(np.int64)) - hs[1].astype(np.int64),
                                                hs[1].astype(np.int64)))
    hx = xx.to_host()
    assert (hx[2][ixx] == hs[2]).all() and (hx[3][ixx] == hs[3]).all()


def test_pncounter_csr(gpu, oracle):
    import crdts_hip

    sp, op = crdts_hip.generate_clocks_csr(5_000, seed=41)
    sn, on = crdts_hip.generate_clocks_csr(5_000, seed=42)
    B = crdts_hip.ClockBatch.from_host
    outp, outn = gpu.pncounter_csr_merge(B(*sp), B(*sn), B(*op), B(*on))
    assert outp.clocks() == unpack(oracle.vclock_csr_merge(sp, op))
    assert outn.clocks() == unpack(oracle.vclock_csr_merge(sn, on))


@pytest.mark.parametrize("bad", ["zero", "unsorted"])
def test_noncanonical_run_rejected(gpu, bad):
    import crdts_hip
    from crdts_hip._lib import CRDT_ENONCANON

    A = [{1: 1, 2: 2}, {1: 1, 2: 2, 3: 3}, {4: 4}]
    s = csr(A)
    if bad == "zero":
        s[3][3] = 0
    else:
        s[2][[2, 3]] = s[2][[3, 2]]
    with pytest.raises(crdts_hip.CrdtError) as e:
        _gpu_merge(gpu, s, csr([{}, {}, {5: 5}]))
    assert e.value.code == CRDT_ENONCANON
    gpu.status()  # cleared
    assert _gpu_merge(gpu, csr(A), csr([{}, {}, {5: 5}])).clocks()[2] == [(4, 4), (5, 5)]


def test_misplaced_runs_rejected(gpu):
    import crdts_hip
    from crdts_hip._lib import CRDT_EINVAL

    off, ln, act, ctr = csr([{1: 1, 2: 2}, {3: 3}, {4: 4}])
    off = off.copy()
    off[1] = 1  # overlaps object 0's run
    with pytest.raises(crdts_hip.CrdtError) as e:
        _gpu_merge(gpu, (off, ln, act, ctr), csr([{}, {}, {}]))
    assert e.value.code == CRDT_EINVAL
