"""Replica anti-entropy across GPUs.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI).
Every rank holds a full replica of the same objects; after anti-entropy every
rank holds the join of all replicas, bit-identical on every rank.

Dense counters (VClock / GCounter / PNCounter rows): the join is the
pointwise u64 max (src/vclock.rs:131-137), associative and commutative, so a
single all-reduce(max) is exact in any reduction order. RCCL/gloo reduce
int64 with a signed max; flipping bit 63 maps unsigned order onto signed
order (x -> x ^ 2^63 is monotone from u64 to i64), so
    max_u64(xs) = max_i64(xs ^ 2^63) ^ 2^63
bit-exactly, for every u64 value.

Orswot: the join is NOT commutative structurally (src/orswot.rs:98-103 vs
:132-138), so replicas are exchanged (all-gather of per-rank byte sizes, then
of size-padded record blobs and offsets) and every rank folds them locally
in rank order ((r0 ⊔ r1) ⊔ r2) ⊔ ... with the batched merge kernel, which
gives identical bytes on every rank.
"""
from __future__ import annotations

import numpy as np

SIGN = -(1 << 63)  # int64 with only bit 63 set


def _torch():
    import torch

    return torch


_NATIVE_U64 = {}


def native_u64_max(device, group=None):
    """Whether this backend reduces torch.uint64 with MAX natively (RCCL's
    ncclUint64 + ncclMax); probed once per device with a 2-element collective
    whose answer needs unsigned order."""
    torch = _torch()
    import torch.distributed as dist

    key = (str(device), id(group))
    if key not in _NATIVE_U64:
        ok = False
        try:
            rank = dist.get_rank(group)
            t = torch.tensor([(1 << 63) + 5 if rank == 0 else 7, 3], dtype=torch.uint64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            ok = int(t[0].item()) == (1 << 63) + 5
        except (RuntimeError, TypeError, ValueError):
            ok = False
        _NATIVE_U64[key] = ok
    return _NATIVE_U64[key]


def dense_allreduce_max(rows, group=None, chunk_elems=1 << 28, native=None):
    """In place: rows = max over ranks (u64 semantics) of rows.

    `rows` is an int64 tensor holding u64 counters (any shape), on the
    process's GPU for nccl or on the CPU for gloo. Where the backend reduces
    uint64 natively (RCCL ncclUint64/ncclMax; `native`, probed when None) the
    rows are reduced as uint64 directly; otherwise through the sign flip
    below. Chunked so collectives stay <= 2 GiB.
    """
    torch = _torch()
    import torch.distributed as dist

    flat = rows.view(-1)
    if native is None:
        native = native_u64_max(flat.device, group)
    if native:
        u = flat.view(torch.uint64)
        for s in range(0, u.numel(), chunk_elems):
            dist.all_reduce(u[s:s + chunk_elems], op=dist.ReduceOp.MAX, group=group)
        return rows
    sign = torch.tensor(SIGN, dtype=torch.int64, device=flat.device)
    for s in range(0, flat.numel(), chunk_elems):
        part = flat[s:s + chunk_elems]
        part.bitwise_xor_(sign)
        dist.all_reduce(part, op=dist.ReduceOp.MAX, group=group)
        part.bitwise_xor_(sign)
    return rows


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


def orswot_gather(batch_base, batch_off, group=None):
    """All-gather every rank's Orswot record batch (base: uint8 tensor,
    off: int64 tensor of byte offsets; same n_obj on every rank).
    Returns [(base_r, off_r)] in rank order, on the input's device."""
    torch = _torch()
    bases = _gather_bytes(batch_base, group)
    offs = _gather_bytes(batch_off.view(torch.uint8), group)
    return [(b, o.view(torch.int64)) for b, o in zip(bases, offs)]


def orswot_anti_entropy(engine, batch, group=None, merge_fn=None):
    """Join the Orswot replicas of all ranks: returns an OrswotBatch equal to
    ((r0 ⊔ r1) ⊔ r2) ⊔ ... on every rank.

    `merge_fn(L, R) -> OrswotBatch` defaults to engine.orswot_merge (the GPU
    kernel); the gloo tests on CPU pass the oracle instead.
    """
    from . import OrswotBatch

    parts = orswot_gather(batch.base, batch.off, group)
    merge = merge_fn or (lambda L, R: engine.orswot_merge(L, R))
    fl = getattr(batch, "flags", 0)  # dense or CSR top clocks, the same on every rank
    acc = OrswotBatch(parts[0][0], parts[0][1], batch.n_actors, parts[0][0].numel(), fl)
    for base, off in parts[1:]:
        acc = merge(acc, OrswotBatch(base, off, batch.n_actors, base.numel(), fl))
    return acc


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
