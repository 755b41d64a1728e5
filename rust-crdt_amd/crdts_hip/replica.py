"""Replica anti-entropy across GPUs: the
Python front end.

One process per GPU; every rank holds a full replica of the same objects and
after anti-entropy every rank holds the join of all replicas, bit-identical.

On GPUs the work is done by the C ABI over RCCL (rust-crdt_amd/csrc/replica.hip):
`init_comm` gives the Engine's context an RCCL communicator (the 128-byte id
is broadcast over the torch.distributed group), then
- `dense_allreduce_max` -> crdt_replica_allreduce_max: one in-place
  ncclAllReduce(ncclUint64, ncclMax). The join is VClock::merge
  (src/vclock.rs:131-137), a pointwise max: exact in any reduction order.
  `dense_reduce_scatter_max` -> crdt_replica_reduce_scatter_max: the
  owner-shard variant (each rank keeps its 1/N of the joined words).
- `orswot_anti_entropy` -> crdt_orswot_replica_join: OWNER-SHARDED. The join
  is structurally NON-commutative (src/orswot.rs:98-103 vs :132-138), so the
  result is the rank-order fold ((r0 ⊔ r1) ⊔ r2) ⊔ ...; the n objects are
  split into N contiguous ranges, rank j receives every replica's slice of
  range j (point-to-point), folds it in rank order, compacts it, and the folded
  ranges are exchanged back. Per rank: n/N objects folded N-1 times and about
  2(N-1)/N of one replica's bytes on the wire.

Without a communicator (CPU tensors over gloo, tests) the same two functions
run the same algorithm over torch.distributed (all_to_all_single /
all_gather) with a caller-supplied merge (the oracle in the CPU tests): the
dense max reduces int64 after flipping bit 63 (x -> x ^ 2^63 maps u64 order
onto i64 order), since gloo's MAX is signed.
"""
from __future__ import annotations

import numpy as np

SIGN = -(1 << 63)  # int64 with only bit 63 set


def _torch():
    import torch

    return torch


def init_comm(engine, group=None):
    """Collective: rank 0 draws an RCCL id, the group broadcasts it, and every
    rank's engine context creates its communicator (crdt_comm_init)."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    box = [engine.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0, group=group)
    engine.comm_init(box[0], world, rank)
    return engine


def _has_comm(engine):
    return engine is not None and getattr(engine, "has_comm", False)


def dense_allreduce_max(rows, group=None, chunk_elems=1 << 28, engine=None, stream=None):
    """In place: rows = max over ranks (u64 semantics) of rows.

    `rows` is an int64 tensor holding u64 counters (any shape). With an engine
    whose context owns a communicator: crdt_replica_allreduce_max (RCCL,
    native ncclUint64 + ncclMax, no extra passes). Otherwise (gloo, CPU):
    torch.distributed all-reduce through the sign flip, chunked.
    """
    if _has_comm(engine):
        return engine.replica_allreduce_max(rows, stream=stream)
    torch = _torch()
    import torch.distributed as dist

    flat = rows.view(-1)
    sign = torch.tensor(SIGN, dtype=torch.int64, device=flat.device)
    for s in range(0, flat.numel(), chunk_elems):
        part = flat[s:s + chunk_elems]
        part.bitwise_xor_(sign)
        dist.all_reduce(part, op=dist.ReduceOp.MAX, group=group)
        part.bitwise_xor_(sign)
    return rows


def dense_reduce_scatter_max(rows, group=None, engine=None, stream=None):
    """The owner-shard variant: this rank's
    1/N of the rows' words, maxed over ranks (u64 order). With an engine that
    owns a communicator: crdt_replica_reduce_scatter_max (one
    ncclReduceScatter, ncclUint64 + ncclMax). Otherwise (gloo, CPU): the
    all-reduce above, then this rank's slice."""
    if _has_comm(engine):
        return engine.replica_reduce_scatter_max(rows, stream=stream)
    import torch.distributed as dist

    world, me = dist.get_world_size(group), dist.get_rank(group)
    flat = rows.reshape(-1).clone()
    if flat.numel() % world:
        raise ValueError("reduce_scatter: word count not a multiple of the rank count")
    dense_allreduce_max(flat, group=group)
    w = flat.numel() // world
    return flat[me * w:(me + 1) * w].clone()


def _gather_bytes(buf_u8, group=None):
    """All-gather a variable-length uint8 tensor: sizes first, then padded blobs."""
    torch = _torch()
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = torch.tensor([buf_u8.numel()], dtype=torch.int64, device=buf_u8.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    cap = max(sizes) if sizes else 0
    pad = torch.zeros(cap, dtype=torch.uint8, device=buf_u8.device)
    pad[: buf_u8.numel()] = buf_u8
    outs = [torch.empty(cap, dtype=torch.uint8, device=buf_u8.device) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return [o[:s] for o, s in zip(outs, sizes)]


def ranges(n, world):
    """Object range owned by each rank: [b_j, b_{j+1}), b_j = j*n // N (the C
    ABI's split, crdt_orswot_replica_join)."""
    return [n * j // world for j in range(world + 1)]


def _record_sizes(base, off):
    b = base.cpu().numpy()
    o = off.cpu().numpy().view(np.uint64)
    return np.array([int(b[x:x + 4].view(np.uint32)[0]) for x in o.tolist()], dtype=np.int64)


def orswot_anti_entropy(engine, batch, group=None, merge_fn=None, stats=None):
    """Join the Orswot replicas of all ranks: returns an OrswotBatch equal to
    ((r0 ⊔ r1) ⊔ r2) ⊔ ... on every rank.

    With an engine that owns a communicator and no merge_fn: the C ABI
    (crdt_orswot_replica_join over RCCL, the batched GPU merge as the fold).
    Otherwise the same owner-sharded algorithm over torch.distributed, folding
    with merge_fn(L, R) -> OrswotBatch (default engine.orswot_merge). `stats`,
    if a dict, receives this rank's exchange and fold counts.
    """
    if merge_fn is None and _has_comm(engine):
        return engine.orswot_replica_join(batch)
    torch = _torch()
    import torch.distributed as dist

    from . import OrswotBatch

    merge = merge_fn or (lambda L, R: engine.orswot_merge(L, R))
    R_, me = dist.get_world_size(group), dist.get_rank(group)
    n, fl, A = batch.n_obj, getattr(batch, "flags", 0), batch.n_actors
    b = ranges(n, R_)
    off = batch.off.cpu().numpy().view(np.uint64)
    sizes = _record_sizes(batch.base, batch.off)
    # 1. byte extent of my slice of every range, all-gathered
    bounds = np.zeros(2 * R_, dtype=np.int64)
    for j in range(R_):
        if b[j + 1] > b[j]:
            bounds[2 * j] = int(off[b[j]])
            bounds[2 * j + 1] = int(off[b[j + 1] - 1]) + int(sizes[b[j + 1] - 1])
    mine = torch.from_numpy(bounds).to(batch.base.device)
    G = [torch.zeros_like(mine) for _ in range(R_)]
    dist.all_gather(G, mine, group=group)
    G = [g.cpu().numpy() for g in G]
    # 2. every replica's slice of my range (records, then offsets)
    send = torch.cat([batch.base[int(bounds[2 * j]):int(bounds[2 * j + 1])] for j in range(R_)])
    in_splits = [int(bounds[2 * j + 1] - bounds[2 * j]) for j in range(R_)]
    out_splits = [int(G[p][2 * me + 1] - G[p][2 * me]) for p in range(R_)]
    recv = torch.empty(sum(out_splits), dtype=torch.uint8, device=batch.base.device)
    dist.all_to_all_single(recv, send, out_splits, in_splits, group=group)
    nr = b[me + 1] - b[me]
    roff = torch.empty(nr * R_, dtype=torch.int64, device=batch.base.device)
    dist.all_to_all_single(roff, batch.off.contiguous(), [nr] * R_, [b[j + 1] - b[j] for j in range(R_)], group=group)
    pos = np.concatenate([[0], np.cumsum(out_splits)]).astype(np.int64)
    pieces = []
    for p in range(R_):
        po = roff[p * nr:(p + 1) * nr] - int(G[p][2 * me])
        pieces.append(OrswotBatch(recv[int(pos[p]):int(pos[p + 1])].contiguous(), po.contiguous(), A,
                                  out_splits[p], fl))
    # 3. rank-order fold of my range, compacted
    acc = pieces[0]
    for piece in pieces[1:]:
        acc = merge(acc, piece) if nr else acc
    shard = OrswotBatch.from_records(acc.records(), A, device=None, flags=fl) if nr else None
    sb = shard.base[: shard.bytes] if shard is not None else torch.empty(0, dtype=torch.uint8)
    so = shard.off if shard is not None else torch.empty(0, dtype=torch.int64)
    # 4. the folded ranges, all-gathered and rebased
    bases = _gather_bytes(sb.to(batch.base.device), group)
    offs = _gather_bytes(so.to(batch.base.device).view(torch.uint8), group)
    P = np.concatenate([[0], np.cumsum([x.numel() for x in bases])]).astype(np.int64)
    out_off = torch.cat([o.view(torch.int64) + int(P[q]) for q, o in enumerate(offs)])
    out_base = torch.cat(bases) if int(P[-1]) else torch.zeros(16, dtype=torch.uint8)
    if isinstance(stats, dict):
        stats.update(objects_folded=nr, merges=nr * (R_ - 1), bytes_sent=sum(in_splits) + int(sb.numel()) * (R_ - 1),
                     bytes_received=sum(out_splits) + int(P[-1]) - int(sb.numel()))
    return OrswotBatch(out_base, out_off, A, max(16, int(P[-1])), fl)


class GlooTransport:
    """A crdt_transport over a torch.distributed group (e.g. gloo): the C
    ABI's owner-sharded join (crdt_orswot_replica_join_transport) with every
    rank a process, RCCL not involved. Device data is staged through host
    memory (hipMemcpy), so this is a test / fallback transport — the product
    multi-GPU path is RCCL (crdt_orswot_replica_join). Any transport failure
    (a torch.distributed error, a self transfer that does not pair up) ends
    the process with exit code 70 instead of returning CRDT_ECOMM: its peers
    may already have posted their side, and only a closed connection releases
    them."""

    def __init__(self, group=None):
        import ctypes as C

        import torch.distributed as dist

        from ._lib import ALLGATHER_FN, EXCHANGE_FN, TransportC, hip_runtime

        self.group = group
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        self._hip = hip_runtime()  # the HIP runtime already loaded (torch's)
        self._hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self._hip.hipStreamSynchronize.argtypes = [C.c_void_p]
        self.calls = {"allgather": 0, "exchange": 0, "bytes_sent": 0, "bytes_received": 0}
        self._ag = ALLGATHER_FN(self._allgather)
        self._ex = EXCHANGE_FN(self._exchange)
        self.c = TransportC(self.world, self.rank, None, self._ag, self._ex)

    def _memcpy(self, dst, src, n):
        if n and self._hip.hipMemcpy(dst, src, n, 4) != 0:  # hipMemcpyDefault
            raise RuntimeError("hipMemcpy failed")

    def _allgather(self, user, h_in, n, h_out):
        try:
            import torch
            import torch.distributed as dist

            mine = torch.from_numpy(np.ctypeslib.as_array(h_in, shape=(n,)).view(np.int64).copy())
            parts = [torch.empty(n, dtype=torch.int64) for _ in range(self.world)]
            dist.all_gather(parts, mine, group=self.group)
            out = np.ctypeslib.as_array(h_out, shape=(n * self.world,)).view(np.int64)
            out[:] = torch.cat(parts).numpy()
            self.calls["allgather"] += 1
            return 0
        except Exception as e:  # noqa: BLE001 - peers may be inside the collective
            self._abandon("allgather", e)

    @staticmethod
    def _abandon(what, e):
        """A transport failure after the peers may have posted their side of the
        collective: they would wait forever, so this process exits (non-zero)
        and its peers' waits fail on the closed connection — no rank is left
        waiting in a collective another has left."""
        import os
        import sys

        print(f"GlooTransport.{what}: {e!r}; exiting so that no peer waits forever", file=sys.stderr, flush=True)
        os._exit(70)

    def _exchange(self, user, sends, ns, recvs, nr, stream):
        # the local checks first. A mismatch ends the process as any other
        # transport failure does (_abandon): the peers post their side of this
        # exchange concurrently, so returning an error here would leave them
        # waiting for transfers this rank never makes
        S = [sends[k] for k in range(ns)]
        Rv = [recvs[k] for k in range(nr)]
        me = self.rank
        self_s = [x for x in S if x.peer == me]
        self_r = [y for y in Rv if y.peer == me]
        if len(self_s) != len(self_r) or any(x.bytes != y.bytes for x, y in zip(self_s, self_r)):
            self._abandon("exchange", ValueError("self transfers do not pair up"))
        try:
            import ctypes as C

            import torch
            import torch.distributed as dist

            if self._hip.hipStreamSynchronize(stream) != 0:  # the sends' data is produced on `stream`
                raise RuntimeError("hipStreamSynchronize failed")
            for x, y in zip(self_s, self_r):  # k-th self send -> k-th self recv
                self._memcpy(y.dst, x.src, x.bytes)
            reqs, landing = [], []
            tag = {}
            for x in S:  # tags: position among this pair's transfers (the same on both ends)
                t = tag[("s", x.peer)] = tag.get(("s", x.peer), -1) + 1
                if x.peer == me or not x.bytes:
                    continue
                h = np.empty(x.bytes, np.uint8)
                self._memcpy(h.ctypes.data_as(C.c_void_p), x.src, x.bytes)
                reqs.append(dist.isend(torch.from_numpy(h), x.peer, group=self.group, tag=t))
                self.calls["bytes_sent"] += x.bytes
            for y in Rv:
                t = tag[("r", y.peer)] = tag.get(("r", y.peer), -1) + 1
                if y.peer == me or not y.bytes:
                    continue
                h = torch.empty(y.bytes, dtype=torch.uint8)
                reqs.append(dist.irecv(h, y.peer, group=self.group, tag=t))
                landing.append((y, h))
            for r in reqs:
                r.wait()
            for y, h in landing:
                self._memcpy(y.dst, C.c_void_p(h.data_ptr()), y.bytes)
                self.calls["bytes_received"] += y.bytes
            self.calls["exchange"] += 1
            return 0
        except Exception as e:  # noqa: BLE001 - peers may be inside the collective
            self._abandon("exchange", e)


def digest(batch) -> int:
    """Checksum of a batch's records in object order (offsets and gaps
    excluded, so gapped and compact batches of the same states agree):
    sum over the concatenated records' u64 words w_k of w_k * (2k + 1), mod 2^64."""
    base = batch.base.cpu().numpy() if hasattr(batch.base, "cpu") else np.asarray(batch.base, dtype=np.uint8)
    off = batch.off.cpu().numpy().view(np.uint64) if hasattr(batch.off, "cpu") else np.asarray(batch.off, np.uint64)
    parts = []
    for o in off.tolist():
        size = int(base[o:o + 4].view(np.uint32)[0])
        parts.append(base[o:o + size])
    if not parts:
        return 0
    cat = np.concatenate(parts)
    words = cat.view(np.uint64)  # every record is a multiple of 16 bytes
    k = np.arange(words.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int((words * (k * np.uint64(2) + np.uint64(1))).sum(dtype=np.uint64))
