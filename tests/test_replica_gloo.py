"""CPU, world_size 2-3 over gloo: the replica anti-entropy exchange (§8(e)).

- dense: u64-exact all-reduce(max) via the sign flip, including counters
  >= 2^63 (where a plain signed max would be wrong);
- Orswot: the OWNER-SHARDED join (rank j folds range j of every replica in
  rank order, the folded ranges are all-gathered); with the oracle as the fold
  (no GPU here) every rank ends with the oracle's ((r0 ⊔ r1) ⊔ r2) bytes,
  identical on every rank, having folded only its 1/N of the objects.
The same Python front end drives the C ABI over RCCL (crdt_orswot_replica_join,
crdt_replica_allreduce_max) when the engine owns a communicator: bench.py at
N > 1, and tests/test_gpu_replica.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import sys

    for p in (os.path.join(REPO, "rust-crdt_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _dense_worker(rank, world, port, q):
    _init(rank, world, port)
    from crdts_hip import replica

    rng = np.random.default_rng(100 + rank)
    rows = rng.integers(0, np.iinfo(np.uint64).max, size=(258, 16), dtype=np.uint64, endpoint=True)
    rows[rng.random(rows.shape) < 0.25] = 0
    t = torch.from_numpy(rows.view(np.int64).copy())
    shard = replica.dense_reduce_scatter_max(t.clone())  # the owner-shard variant, before the in-place join
    replica.dense_allreduce_max(t, chunk_elems=1000)
    q.put((rank, rows, t.numpy().view(np.uint64).copy(), shard.numpy().view(np.uint64).copy()))
    dist.destroy_process_group()


def _orswot_worker(rank, world, port, q):
    _init(rank, world, port)
    import crdts_hip
    import oracle_ffi
    from crdts_hip import replica

    n = 300
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(n, threads=2, seed=77)
    (xb, xo), _ = crdts_hip.generate_orswot(n, threads=2, seed=78)
    mine = [(lb, lo), (rb, ro), (xb, xo)][rank]
    B = crdts_hip.OrswotBatch(torch.from_numpy(mine[0].copy()), torch.from_numpy(mine[1].view(np.int64).copy()), 16,
                              mine[0].nbytes)

    def oracle_merge(L, R):
        ob, oo = oracle_ffi.orswot_merge_batch(L.base.numpy(), L.off.numpy().view(np.uint64), R.base.numpy(),
                                               R.off.numpy().view(np.uint64), 16, threads=2)
        return crdts_hip.OrswotBatch(torch.from_numpy(ob), torch.from_numpy(oo.view(np.int64)), 16, ob.nbytes)

    stats = {}
    out = replica.orswot_anti_entropy(None, B, merge_fn=oracle_merge, stats=stats)
    b = replica.ranges(n, world)
    assert stats["objects_folded"] == b[rank + 1] - b[rank]  # owner-sharded: 1/N of the objects
    assert stats["merges"] == (b[rank + 1] - b[rank]) * (world - 1)
    dg = replica.digest(out)
    d = torch.tensor([dg - (1 << 64) if dg >= (1 << 63) else dg], dtype=torch.int64)
    ds = [torch.zeros_like(d) for _ in range(world)]
    dist.all_gather(ds, d)
    # reference fold, computed locally from the generator
    acc = (lb, lo)
    for b, o in [(rb, ro), (xb, xo)][: world - 1]:
        acc = oracle_ffi.orswot_merge_batch(acc[0], acc[1], b, o, 16, threads=2)
    ref = crdts_hip.OrswotBatch(torch.from_numpy(acc[0]), torch.from_numpy(acc[1].view(np.int64)), 16, acc[0].nbytes)
    q.put((rank, [int(x.item()) % (1 << 64) for x in ds], replica.digest(ref), out.records() == ref.records()))
    dist.destroy_process_group()


def _orswot_sparse_worker(rank, world, port, q):
    """Config-5 shape: every rank holds replica `rank` of the same objects
    (CSR top clocks, 1024-actor universe)."""
    _init(rank, world, port)
    import crdts_hip
    import oracle_ffi
    from crdts_hip import replica

    U, SP = 1024, crdts_hip.SPARSE_CLOCK
    reps = crdts_hip.generate_replicas(250, world, threads=2)
    mine = reps[rank]
    B = crdts_hip.OrswotBatch(torch.from_numpy(mine[0].copy()), torch.from_numpy(mine[1].view(np.int64).copy()), U,
                              mine[0].nbytes, SP)

    def oracle_merge(L, R):
        assert L.flags == R.flags == SP
        ob, oo = oracle_ffi.orswot_merge_batch(L.base.numpy(), L.off.numpy().view(np.uint64), R.base.numpy(),
                                               R.off.numpy().view(np.uint64), U, threads=2, flags=SP)
        return crdts_hip.OrswotBatch(torch.from_numpy(ob), torch.from_numpy(oo.view(np.int64)), U, ob.nbytes, SP)

    out = replica.orswot_anti_entropy(None, B, merge_fn=oracle_merge)
    acc = reps[0]
    for b, o in reps[1:]:
        acc = oracle_ffi.orswot_merge_batch(acc[0], acc[1], b, o, U, threads=2, flags=SP)
    ref = crdts_hip.OrswotBatch(torch.from_numpy(acc[0]), torch.from_numpy(acc[1].view(np.int64)), U, acc[0].nbytes)
    dg = replica.digest(out)
    d = torch.tensor([dg - (1 << 64) if dg >= (1 << 63) else dg], dtype=torch.int64)
    ds = [torch.zeros_like(d) for _ in range(world)]
    dist.all_gather(ds, d)
    q.put((rank, [int(x.item()) % (1 << 64) for x in ds], replica.digest(ref), out.records() == ref.records()))
    dist.destroy_process_group()


def _orswot_tiny_worker(rank, world, port, q):
    """More ranks than objects: some ranges are empty."""
    _init(rank, world, port)
    import crdts_hip
    import oracle_ffi
    from crdts_hip import replica

    gens = [crdts_hip.generate_orswot(2, threads=1, seed=90 + r)[0] for r in range(world)]
    lb, lo = gens[rank]
    B = crdts_hip.OrswotBatch(torch.from_numpy(lb.copy()), torch.from_numpy(lo.view(np.int64).copy()), 16, lb.nbytes)

    def oracle_merge(L, R):
        ob, oo = oracle_ffi.orswot_merge_batch(L.base.numpy(), L.off.numpy().view(np.uint64), R.base.numpy(),
                                               R.off.numpy().view(np.uint64), 16, threads=1)
        return crdts_hip.OrswotBatch(torch.from_numpy(ob), torch.from_numpy(oo.view(np.int64)), 16, ob.nbytes)

    out = replica.orswot_anti_entropy(None, B, merge_fn=oracle_merge)
    acc = gens[0]
    for b, o in gens[1:]:
        acc = oracle_ffi.orswot_merge_batch(acc[0], acc[1], b, o, 16, threads=1)
    ref = crdts_hip.OrswotBatch(torch.from_numpy(acc[0]), torch.from_numpy(acc[1].view(np.int64)), 16, acc[0].nbytes)
    q.put((rank, None, None, out.records() == ref.records()))
    dist.destroy_process_group()


def _guarded(fn, rank, world, port, q):
    try:
        fn(rank, world, port, q)
    except BaseException:  # report instead of leaving the peers blocked in a collective
        import traceback

        q.put(("error", rank, traceback.format_exc()))
        raise


def _run(fn, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guarded, args=(fn, r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    for _ in range(world):
        item = q.get(timeout=240)
        if item[0] == "error":
            for p in procs:
                p.kill()
            raise AssertionError(f"rank {item[1]} failed:\n{item[2]}")
        res.append(item)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda x: x[0])


def test_dense_allreduce_max_u64_exact_gloo():
    res = _run(_dense_worker, 2)
    exp = np.maximum(res[0][1], res[1][1])
    assert (exp >= np.uint64(1 << 63)).any()  # the sign-flip matters on this data
    half = exp.size // 2
    for r, _, got, shard in res:
        assert (got == exp).all()
        assert (shard == exp.reshape(-1)[r * half:(r + 1) * half]).all()  # rank r owns words [r n/N, (r+1) n/N)


@pytest.mark.parametrize("world", [2, 3])
def test_orswot_anti_entropy_gloo(world):
    res = _run(_orswot_worker, world)
    for rank, digests, ref_digest, same in res:
        assert same, f"rank {rank} fold differs from the oracle's rank-order fold"
        assert len(set(digests)) == 1 and digests[0] == ref_digest


def test_orswot_sparse_anti_entropy_gloo():
    res = _run(_orswot_sparse_worker, 3)
    for rank, digests, ref_digest, same in res:
        assert same, f"rank {rank} sparse fold differs from the oracle's rank-order fold"
        assert len(set(digests)) == 1 and digests[0] == ref_digest


def test_orswot_anti_entropy_more_ranks_than_objects_gloo():
    for rank, _, _, same in _run(_orswot_tiny_worker, 3):
        assert same, f"rank {rank}: fold with empty ranges differs"
