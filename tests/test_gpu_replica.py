"""GPU: replica anti-entropy through the C ABI (SURVEY.md §8(b),(e);
BASELINE.json configs[3], configs[4]).

- RCCL at world size 1 (one GPU on the test box): crdt_comm_init,
  crdt_replica_allreduce_max and crdt_orswot_replica_join driven through the
  same Python front end bench.py uses (crdts_hip.replica), bytes compared
  with the oracle;
- crdt_orswot_replica_join_local: the owner-sharded exchange and rank-order
  fold with 2..8 replicas as virtual ranks on the one GPU (the code below the
  transport is the RCCL path's), byte-exact against the oracle's fold
  ((r0 ⊔ r1) ⊔ r2) ⊔ ... (src/orswot.rs:87-157 applied in rank order),
  dense and CSR records, more ranks than objects, a misordered batch.
"""
import numpy as np
import pytest

import records

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm1():
    """An engine whose context owns a 1-rank RCCL communicator."""
    import crdts_hip

    eng = crdts_hip.Engine(0)
    eng.comm_init(crdts_hip.Engine.comm_unique_id(), 1, 0)
    yield eng
    eng.comm_destroy()


def _oracle_fold(oracle, reps, A, flags=0):
    acc = reps[0]
    for b, o in reps[1:]:
        acc = oracle.orswot_merge_batch(acc[0], acc[1], b, o, A, threads=16, flags=flags)
    return records.unpack_batch(*acc)


def test_rccl_world1_dense_allreduce_max(comm1):
    import torch

    from crdts_hip import replica

    g = torch.Generator(device="cuda:0")
    g.manual_seed(4)
    rows = torch.randint(-(1 << 62), 1 << 62, (1 << 20, 8), dtype=torch.int64, device="cuda:0", generator=g)
    rows[:7] = -1  # u64 values >= 2^63 must survive unchanged (no sign trick anywhere)
    before = rows.clone()
    replica.dense_allreduce_max(rows, engine=comm1)
    torch.cuda.synchronize()
    assert torch.equal(rows, before)


def test_rccl_world1_reduce_scatter_max(comm1):
    """crdt_replica_reduce_scatter_max at world size 1: the owner shard is
    every word, unchanged (u64 values >= 2^63 included)."""
    import torch

    from crdts_hip import replica

    rows = torch.randint(-(1 << 62), 1 << 62, (4096, 8), dtype=torch.int64, device="cuda:0")
    rows[:5] = -3
    shard = replica.dense_reduce_scatter_max(rows, engine=comm1)
    torch.cuda.synchronize()
    assert torch.equal(shard, rows.reshape(-1))


def test_rccl_world1_orswot_replica_join(comm1, oracle):
    import crdts_hip
    from crdts_hip import replica

    (lb, lo), _ = crdts_hip.generate_orswot(20_000, threads=16, seed=31)
    B = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    out = replica.orswot_anti_entropy(comm1, B)
    assert out.records() == records.unpack_batch(lb, lo)  # the fold of one replica is itself, packed
    assert out.bytes <= B.bytes


@pytest.mark.parametrize("R", [2, 3, 8])
def test_local_join_dense_matches_oracle_fold(gpu, oracle, R):
    import crdts_hip

    reps = [crdts_hip.generate_orswot(5_000, threads=16, seed=40 + r)[r % 2] for r in range(R)]
    batches = [crdts_hip.OrswotBatch.from_host(b, o, 16) for b, o in reps]
    out = gpu.orswot_replica_join_local(batches)
    exp = _oracle_fold(oracle, reps, 16)
    got = out.records()
    bad = [i for i, (x, y) in enumerate(zip(got, exp)) if x != y]
    assert not bad, f"{len(bad)} / {len(exp)} differ, first {bad[0]}"
    assert len(got) == len(exp)


def test_local_join_sparse_config5_matches_oracle_fold(gpu, oracle):
    import crdts_hip

    U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
    reps = crdts_hip.generate_replicas(4_000, 8, threads=16)
    batches = [crdts_hip.OrswotBatch.from_host(b, o, U, flags=SP) for b, o in reps]
    out = gpu.orswot_replica_join_local(batches)
    assert out.records() == _oracle_fold(oracle, reps, U, SP)


def test_local_join_gapped_inputs_and_tiny(gpu, oracle):
    """Replicas that are merge outputs (gaps between records), and more
    virtual ranks than objects (empty ranges)."""
    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(3_000, threads=16, seed=51)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    Rb = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    gapped = gpu.orswot_merge(L, Rb)  # offsets self.off + other.off: a batch with gaps
    out = gpu.orswot_replica_join_local([gapped, L, Rb])
    gb, go = gapped.to_host()
    exp = _oracle_fold(oracle, [(gb, go), (lb, lo), (rb, ro)], 16)
    assert out.records() == exp
    small = [crdts_hip.generate_orswot(3, threads=1, seed=60 + r)[0] for r in range(5)]
    out = gpu.orswot_replica_join_local([crdts_hip.OrswotBatch.from_host(b, o, 16) for b, o in small])
    assert out.records() == _oracle_fold(oracle, small, 16)


def test_local_join_rejects_misordered_replica(gpu):
    import crdts_hip
    from crdts_hip._lib import CRDT_EINVAL

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(1_000, threads=16, seed=70)
    perm = lo.copy()
    perm[[0, 999]] = perm[[999, 0]]
    with pytest.raises(crdts_hip.CrdtError) as e:
        gpu.orswot_replica_join_local([crdts_hip.OrswotBatch.from_host(lb, perm, 16),
                                       crdts_hip.OrswotBatch.from_host(rb, ro, 16)])
    assert e.value.code == CRDT_EINVAL
    # the context is usable afterwards
    out = gpu.orswot_replica_join_local([crdts_hip.OrswotBatch.from_host(lb, lo, 16),
                                         crdts_hip.OrswotBatch.from_host(rb, ro, 16)])
    assert out.n_obj == 1_000
