"""GPU parity for records at offsets past 2 GiB / 4 GiB.

Batches are plain byte buffers addressed by u64 offsets (include/crdts_hip.h);
a 1M-object fold over CSR records (config 5) outgrows 2^31 bytes by its second
step. Here both inputs sit behind a gap that puts their records on either side
of 2^31 and their output slots (self.off + other.off) on either side of 2^32,
for the dense (config 3) and the sparse (config 5) join, checked byte-exact
against the oracle.
"""
import numpy as np
import pytest

import records

pytestmark = pytest.mark.gpu

GAP = (1 << 31) - (1 << 19)  # records straddle 2 GiB; output slots straddle 4 GiB


def _shifted(base, off, n_actors, flags):
    import torch

    import crdts_hip

    base = np.ascontiguousarray(base, dtype=np.uint8)
    nb = GAP + (base.nbytes + 15) // 16 * 16
    b = torch.empty(nb, dtype=torch.uint8, device="cuda:0")
    b[GAP:GAP + base.nbytes].copy_(torch.from_numpy(base))
    o = np.ascontiguousarray(off, dtype=np.uint64) + np.uint64(GAP)
    ot = torch.from_numpy(o.view(np.int64)).to("cuda:0")
    return crdts_hip.OrswotBatch(b, ot, n_actors, nb, flags)


def _check(gpu, oracle, lb, lo, rb, ro, n_actors, flags):
    L = _shifted(lb, lo, n_actors, flags)
    R = _shifted(rb, ro, n_actors, flags)
    out = gpu.orswot_merge(L, R)
    got_off = out.off.cpu().numpy().view(np.uint64)
    exp_off = L.off.cpu().numpy().view(np.uint64) + R.off.cpu().numpy().view(np.uint64)
    assert (got_off == exp_off).all()
    assert got_off.min() < (1 << 32) < got_off.max()
    ob, oo = oracle.orswot_merge_batch(lb, lo, rb, ro, n_actors, threads=16, flags=flags)
    exp = records.unpack_batch(ob, oo)
    first = int(got_off.min())
    host = out.base[first:int(got_off.max()) + max(map(len, exp))].cpu().numpy()
    bad = 0
    for i, e in enumerate(exp):
        s = int(got_off[i]) - first
        if host[s:s + len(e)].tobytes() != e:
            bad += 1
    assert bad == 0, f"{bad} / {len(exp)} objects differ"
    del out, L, R


def test_dense_records_past_2gib(gpu, oracle):
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(4_000, first_obj=123, threads=16)
    assert int(lo[-1]) + GAP > (1 << 31) > int(lo[0]) + GAP
    _check(gpu, oracle, lb, lo, rb, ro, crdts_hip.CONFIG3["n_actors"], 0)


def test_sparse_records_past_2gib(gpu, oracle):
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_replicas(3_000, 2, first_obj=77, threads=16)
    assert int(lo[-1]) + GAP > (1 << 31) > int(lo[0]) + GAP
    _check(gpu, oracle, lb, lo, rb, ro, crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK)
