"""GPU, one process per rank: the PRODUCT's owner-sharded Orswot replica join
(C++ `orswot_join_rank`, rust-crdt_amd/csrc/replica.hip) with ranks as real
processes, world 1-3, all on the test box's one MI355X.

RCCL cannot put two ranks on one GPU, so the ranks talk through
crdt_orswot_replica_join_transport with a gloo transport (crdts_hip.replica.
GlooTransport: host-staged all-gathers and point-to-point transfers). Every
line of the join above the transport — slice bounds, the symmetric verdicts,
the arena plan, the rank-order fold with the batched merge kernel, compaction,
the result exchange and rebase — is the code crdt_orswot_replica_join runs
over RCCL. Checked: every rank ends with the oracle's rank-order fold
((r0 ⊔ r1) ⊔ r2) (src/orswot.rs:87-157, order fixed by :98-103 vs :132-138)
byte for byte; a non-canonical record in the middle of a slice makes EVERY
rank return the same error (none left in a collective), and the next join on
the same contexts succeeds. Config 4's dense all-reduce (max) over the same
transport (crdt_replica_allreduce_max_transport) equals the pointwise max of
every rank's rows on every rank, and its owner-shard variant
(crdt_replica_reduce_scatter_max_transport) each rank's slice of it. One rank whose arena cannot grow
(crdt_ctx_set_arena_limit) makes every rank of either exchange return
CRDT_ECAPACITY before any data moves.
"""
import os
import socket

import numpy as np
import pytest

import records

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_fold(oracle_ffi, reps, A, flags=0):
    acc = reps[0]
    for b, o in reps[1:]:
        acc = oracle_ffi.orswot_merge_batch(acc[0], acc[1], b, o, A, threads=4, flags=flags)
    return records.unpack_batch(*acc)


CRDT_EINVAL, CRDT_ECAPACITY, CRDT_ENONCANON = -1, -4, -2  # include/crdts_hip.h


def _worker(rank, world, port, q):
    import sys

    for p in (os.path.join(REPO, "rust-crdt_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    import crdts_hip
    import oracle_ffi
    from crdts_hip import replica

    eng = crdts_hip.Engine(0)
    T = replica.GlooTransport()
    res = {"rank": rank}

    # 1. dense records (config-3 shape), one distinct replica per rank
    reps = [crdts_hip.generate_orswot(4_000, threads=4, seed=140 + r)[r % 2] for r in range(world)]
    B = crdts_hip.OrswotBatch.from_host(*reps[rank], 16)
    out = eng.orswot_replica_join_transport(B, T)
    res["dense_ok"] = out.records() == _oracle_fold(oracle_ffi, reps, 16)
    res["dense_digest"] = replica.digest(out)

    # 2. CSR records, config-5 shape (replica r of the same objects on rank r)
    U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
    sreps = crdts_hip.generate_replicas(3_000, world, threads=4)
    SB = crdts_hip.OrswotBatch.from_host(*sreps[rank], U, flags=SP)
    sout = eng.orswot_replica_join_transport(SB, T)
    res["sparse_ok"] = sout.records() == _oracle_fold(oracle_ffi, sreps, U, SP)
    res["sparse_digest"] = replica.digest(sout)

    # 3. a non-canonical record (n_clk != n_actors) in the MIDDLE of the last
    #    rank's slice of range 0: every rank must return the same error
    bad_b, bad_o = reps[rank][0].copy(), reps[rank][1]
    if rank == world - 1:
        i = len(bad_o) // (2 * world)
        o = int(bad_o[i])
        bad_b[o + 4:o + 8] = np.frombuffer(np.uint32(17).tobytes(), np.uint8)
    try:
        eng.orswot_replica_join_transport(crdts_hip.OrswotBatch.from_host(bad_b, bad_o, 16), T)
        res["bad_code"] = 0
    except crdts_hip.CrdtError as e:
        res["bad_code"] = e.code
    # 4. the contexts are clean afterwards: the good join again
    out2 = eng.orswot_replica_join_transport(B, T)
    res["after_ok"] = replica.digest(out2) == res["dense_digest"]
    eng.status()  # nothing left latched
    res["calls"] = dict(T.calls)
    # 5. config 4: dense u64 rows (VClock / GCounter rows) all-reduced (max) by
    #    the product over the transport (crdt_replica_allreduce_max_transport);
    #    a length no rank count divides, counters >= 2^63 and zeros
    import torch

    def rows_of(r):
        g = np.random.default_rng(300 + r)
        x = g.integers(0, np.iinfo(np.uint64).max, size=16 * 1000 + 7, dtype=np.uint64, endpoint=True)
        x[g.random(x.shape) < 0.25] = 0
        return x

    exp = np.maximum.reduce([rows_of(r) for r in range(world)])
    t = torch.from_numpy(rows_of(rank).view(np.int64).copy()).to("cuda:0")
    eng.replica_allreduce_max_transport(t, T)
    res["ar_ok"] = bool(np.array_equal(t.cpu().numpy().view(np.uint64), exp))
    # 5b. the owner-shard variant over the same transport
    #     (crdt_replica_reduce_scatter_max_transport): rank r's 1/N of the max
    w = 6000 // world
    rs = eng.replica_reduce_scatter_max_transport(
        torch.from_numpy(rows_of(rank)[:6000].view(np.int64).copy()).to("cuda:0"), T)
    res["rs_ok"] = bool(np.array_equal(rs.cpu().numpy().view(np.uint64), exp[rank * w:(rank + 1) * w]))
    # 5c. rank 0 passes a word count no rank count > 1 divides, the others a
    #     divisible one: every rank returns CRDT_EINVAL (the count is part of
    #     the all-gathered verdict), none is left in the exchange
    n5c = 6000 * world + (1 if rank == 0 else 0)
    try:
        eng.replica_reduce_scatter_max_transport(
            torch.from_numpy(np.resize(rows_of(rank), n5c).view(np.int64).copy()).to("cuda:0"), T)
        res["rs_bad_code"] = 0
    except crdts_hip.CrdtError as e:
        res["rs_bad_code"] = e.code
    # 6. one rank's arena cannot grow (a fresh context with a 1 KB arena limit
    #    on the last rank): every rank returns CRDT_ECAPACITY before any data
    #    moves (the verdicts are all-gathered first; nobody waits in an
    #    exchange), the rows are untouched, and the same contexts succeed once
    #    the limit is lifted — for the dense all-reduce and the Orswot join
    eng2 = crdts_hip.Engine(0)
    if rank == world - 1:
        eng2.set_arena_limit(1024)
    t2 = torch.from_numpy(rows_of(rank).view(np.int64).copy()).to("cuda:0")
    codes = []
    for call in (lambda: eng2.replica_allreduce_max_transport(t2, T), lambda: eng2.orswot_replica_join_transport(B, T)):
        try:
            call()
            codes.append(0)
        except crdts_hip.CrdtError as e:
            codes.append(e.code)
    res["limit_codes"] = codes
    res["limit_rows_kept"] = bool(np.array_equal(t2.cpu().numpy().view(np.uint64), rows_of(rank)))
    eng2.set_arena_limit(0)
    eng2.replica_allreduce_max_transport(t2, T)
    res["limit_after_ok"] = bool(np.array_equal(t2.cpu().numpy().view(np.uint64), exp)) and \
        replica.digest(eng2.orswot_replica_join_transport(B, T)) == res["dense_digest"]
    eng2.status()
    # 7. a status latched on rank 0's context by an earlier launch (a rejected
    #    record, merged with check_status=False) and never read is that rank's
    #    error in the next join: every rank returns it; the join after that
    #    succeeds (the status was cleared)
    if rank == 0:
        bb = reps[0][0].copy()
        o0 = int(reps[0][1][0])
        bb[o0 + 4:o0 + 8] = np.frombuffer(np.uint32(17).tobytes(), np.uint8)
        Bb = crdts_hip.OrswotBatch.from_host(bb, reps[0][1], 16)
        eng2.orswot_merge(Bb, Bb, check_status=False)
    try:
        eng2.orswot_replica_join_transport(B, T)
        res["latched_code"] = 0
    except crdts_hip.CrdtError as e:
        res["latched_code"] = e.code
    res["latched_after_ok"] = replica.digest(eng2.orswot_replica_join_transport(B, T)) == res["dense_digest"]
    q.put(res)
    dist.destroy_process_group()


def _guarded(rank, world, port, q):
    try:
        _worker(rank, world, port, q)
    except BaseException:  # report instead of leaving the peers blocked in a collective
        import traceback

        q.put({"error": traceback.format_exc(), "rank": rank})
        raise


@pytest.mark.parametrize("world", [1, 2, 3])
def test_product_join_across_processes(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guarded, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(world):
            item = q.get(timeout=150)
            if "error" in item:
                raise AssertionError(f"rank {item['rank']} failed:\n{item['error']}")
            res.append(item)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    res.sort(key=lambda r: r["rank"])
    for r in res:
        assert r["dense_ok"], f"rank {r['rank']}: dense join differs from the oracle's rank-order fold"
        assert r["sparse_ok"], f"rank {r['rank']}: CSR join differs from the oracle's rank-order fold"
        assert r["bad_code"] != 0, f"rank {r['rank']}: a non-canonical record was accepted"
        assert r["after_ok"], f"rank {r['rank']}: the join after a failed one differs"
    assert len({r["dense_digest"] for r in res}) == 1
    assert len({r["sparse_digest"] for r in res}) == 1
    assert len({r["bad_code"] for r in res}) == 1, [r["bad_code"] for r in res]
    for r in res:  # 2 exchanges per completed join; the failed one stops after the first
        assert r["calls"]["exchange"] == 2 + 2 + 1 + 2, r["calls"]
        assert r["ar_ok"], f"rank {r['rank']}: the transport all-reduce differs from the pointwise max"
        assert r["rs_ok"], f"rank {r['rank']}: the transport reduce-scatter differs from its slice of the max"
        assert r["rs_bad_code"] == (0 if world == 1 else CRDT_EINVAL), r["rs_bad_code"]
        assert r["limit_codes"] == ([0, CRDT_ECAPACITY] if world == 1 else [CRDT_ECAPACITY, CRDT_ECAPACITY]), r["limit_codes"]
        assert r["limit_rows_kept"] or world == 1
        assert r["limit_after_ok"], f"rank {r['rank']}: the calls after the arena failure differ"
        assert r["latched_code"] == CRDT_ENONCANON, r["latched_code"]
        assert r["latched_after_ok"], f"rank {r['rank']}: the join after the latched status differs"
