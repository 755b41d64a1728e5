"""MVReg merge and VClock partial order: the
oracle restatement pinned to the reference's MVReg KATs (test/mvreg.rs) and
VClock order KATs, and GPU parity of crdt_mvreg_merge / crdt_vclock_partial_cmp
against it on random batches."""
import numpy as np
import pytest

A8 = 8


def _slab(regs, cap, A):
    n = len(regs)
    cnt = np.zeros(n, np.uint32)
    clk = np.zeros((n, cap, A), np.uint64)
    val = np.zeros((n, cap), np.uint64)
    for i, r in enumerate(regs):
        cnt[i] = len(r)
        for k, (c, v) in enumerate(r):
            for a, x in c.items():
                clk[i, k, a] = x
            val[i, k] = v
    return cnt, clk, val


def _unslab(cnt, clk, val):
    out = []
    for i in range(len(cnt)):
        out.append([({a: int(x) for a, x in enumerate(clk[i, k]) if x}, int(val[i, k])) for k in range(cnt[i])])
    return out


def test_mvreg_kats(oracle):
    """test/mvreg.rs:36-57 (same value, concurrent: both kept) and :82-103 (multi val)."""
    r1 = [({4: 1}, 23)]
    r2 = [({7: 1}, 23)]
    got = _unslab(*oracle.mvreg_merge(*_slab([r1], 2, A8), *_slab([r2], 2, A8), A8, 4))
    assert got == [[({4: 1}, 23), ({7: 1}, 23)]]
    got = _unslab(*oracle.mvreg_merge(*_slab([[({1: 1}, 32)]], 1, A8), *_slab([[({2: 1}, 82)]], 1, A8), A8, 2))
    assert [v for _, v in got[0]] in ([32, 82], [82, 32])
    # dominated values are dropped; an equal clock is kept once (self's)
    got = _unslab(*oracle.mvreg_merge(*_slab([[({1: 1}, 5), ({2: 2}, 6)]], 2, A8),
                                      *_slab([[({1: 2}, 7), ({2: 2}, 9)]], 2, A8), A8, 4))
    assert got == [[({2: 2}, 6), ({1: 2}, 7)]]


def test_partial_cmp_kats(oracle):
    """test/vclock.rs:134-175 (test_vclock_ordering), actor "A" -> 0, "B" -> 1:
    {} == {}; {A:2} > {A:1}; {A:2} < {A:3}; {A:2,B:1} || {A:3}; {A:3,B:1} > {A:3}."""
    a = np.array([[0, 0], [2, 0], [2, 0], [2, 1], [3, 1]], np.uint64)
    b = np.array([[0, 0], [1, 0], [3, 0], [3, 0], [3, 0]], np.uint64)
    assert oracle.partial_cmp_rows(a, b, 2).tolist() == [0, 1, -1, 2, 1]


def _random_regs(rng, n, cap, A, hi):
    regs = []
    for _ in range(n):
        k = int(rng.integers(0, cap + 1))
        r = []
        for _ in range(k):
            c = {a: int(x) for a, x in enumerate(rng.integers(0, hi, A)) if x}
            r.append((c, int(rng.integers(0, 1 << 62))))
        regs.append(r)
    return regs


@pytest.mark.gpu
@pytest.mark.parametrize("A,cap,hi", [(8, 4, 3), (16, 8, 2), (64, 3, 4), (5, 16, 2)])
def test_gpu_mvreg_merge(gpu, oracle, A, cap, hi):
    import torch

    rng = np.random.default_rng(A * 100 + cap)
    n = 20_000
    S = _slab(_random_regs(rng, n, cap, A, hi), cap, A)
    O = _slab(_random_regs(rng, n, cap, A, hi), cap, A)
    exp = oracle.mvreg_merge(*S, *O, A, 2 * cap)

    def dev(t):
        t = np.ascontiguousarray(t)
        return torch.from_numpy(t.view(np.int32 if t.dtype == np.uint32 else np.int64)).to("cuda:0")

    got = gpu.mvreg_merge(tuple(dev(x) for x in S), tuple(dev(x) for x in O), A)
    gn = got[0].cpu().numpy().view(np.uint32)
    gc = got[1].cpu().numpy().view(np.uint64)
    gv = got[2].cpu().numpy().view(np.uint64)
    assert (gn == exp[0]).all()
    assert (gc == exp[1]).all() and (gv == exp[2]).all()
    assert len(set(exp[0].tolist())) > 3  # a spread of survivor counts


@pytest.mark.gpu
@pytest.mark.parametrize("A,cap,hi,n", [(8, 100, 3, 3000), (16, 300, 2, 300), (512, 16, 2, 2000)])
def test_gpu_mvreg_merge_big(gpu, oracle, A, cap, hi, n):
    """Registers past the fast kernel's limits take the one-wave kernel:
    more than 64 slots per side (100, 300), or rows too large for its LDS
    (16 slots x 512 actors: 128 KB per wave). Exact vs the oracle."""
    import torch

    rng = np.random.default_rng(A * 1000 + cap)
    S = _slab(_random_regs(rng, n, cap, A, hi), cap, A)
    O = _slab(_random_regs(rng, n, cap, A, hi), cap, A)
    exp = oracle.mvreg_merge(*S, *O, A, 2 * cap)

    def dev(t):
        t = np.ascontiguousarray(t)
        return torch.from_numpy(t.view(np.int32 if t.dtype == np.uint32 else np.int64)).to("cuda:0")

    got = gpu.mvreg_merge(tuple(dev(x) for x in S), tuple(dev(x) for x in O), A)
    gn = got[0].cpu().numpy().view(np.uint32)
    assert (gn == exp[0]).all()
    assert (got[1].cpu().numpy().view(np.uint64) == exp[1]).all()
    assert (got[2].cpu().numpy().view(np.uint64) == exp[2]).all()
    assert exp[0].max() > (64 if cap > 64 else 8)


@pytest.mark.gpu
@pytest.mark.parametrize("A", [1, 8, 16, 64, 100, 300])
def test_gpu_partial_cmp(gpu, oracle, A):
    import torch

    rng = np.random.default_rng(A)
    n = 100_000
    a = rng.integers(0, 3, (n, A)).astype(np.uint64)
    b = a.copy()
    sel = rng.random(n)
    b[sel < 0.25] += rng.integers(0, 2, (int((sel < 0.25).sum()), A)).astype(np.uint64)   # b >= a
    m = (sel >= 0.25) & (sel < 0.5)
    b[m] = a[m] - (rng.integers(0, 2, (int(m.sum()), A)).astype(np.uint64) * (a[m] > 0))  # b <= a
    m = sel >= 0.75
    b[m] = rng.integers(0, 3, (int(m.sum()), A)).astype(np.uint64)                          # random
    b[(sel >= 0.5) & (sel < 0.6)] = a[(sel >= 0.5) & (sel < 0.6)]                             # equal
    exp = oracle.partial_cmp_rows(a, b, A)
    ta = torch.from_numpy(a.view(np.int64)).to("cuda:0")
    tb = torch.from_numpy(b.view(np.int64)).to("cuda:0")
    got = gpu.vclock_partial_cmp(ta, tb, A).cpu().numpy()
    assert (got == exp).all()
    assert len(set(exp.tolist())) == 4 or A == 1
