"""Canonical Orswot record codec (layout: include/crdts_hip.h), host side.

Used by the Python mirror types to read states back; the hot path never goes
through here.
"""
from __future__ import annotations

import struct

HDR = 32
SPARSE_CLOCK = 1  # header flags bit 0: CSR top clock (CRDT_ORSWOT_SPARSE_CLOCK)


def _pad(x, a):
    return (x + a - 1) // a * a


def _clock_bytes(n_clk, sparse):
    return _pad(12 * n_clk, 8) if sparse else 8 * n_clk


def record_bytes(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, sparse=False):
    b = _pad(HDR + _clock_bytes(n_clk, sparse) + 12 * (n_mem + n_dot), 8)
    return _pad(b + 12 * n_def_dot + 8 * n_def_mem + 8 * n_def, 16)


def decode_record(rec):
    """-> dict(clock={actor: ctr}, entries={member: [(actor, ctr)]}, deferred=[([(a, c)], [members])])."""
    rec = bytes(rec)
    size, n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, flags = struct.unpack_from("<8I", rec, 0)
    o = HDR
    sparse = bool(flags & SPARSE_CLOCK)
    clk = struct.unpack_from(f"<{n_clk}Q", rec, o)
    cact = struct.unpack_from(f"<{n_clk}I", rec, o + 8 * n_clk) if sparse else range(n_clk)
    o += _clock_bytes(n_clk, sparse)
    keys = struct.unpack_from(f"<{n_mem}Q", rec, o); o += 8 * n_mem
    dctr = struct.unpack_from(f"<{n_dot}Q", rec, o); o += 8 * n_dot
    dact = struct.unpack_from(f"<{n_dot}I", rec, o); o += 4 * n_dot
    dend = struct.unpack_from(f"<{n_mem}I", rec, o); o = _pad(o + 4 * n_mem, 8)
    fctr = struct.unpack_from(f"<{n_def_dot}Q", rec, o); o += 8 * n_def_dot
    fkey = struct.unpack_from(f"<{n_def_mem}Q", rec, o); o += 8 * n_def_mem
    fact = struct.unpack_from(f"<{n_def_dot}I", rec, o); o += 4 * n_def_dot
    fdend = struct.unpack_from(f"<{n_def}I", rec, o); o += 4 * n_def
    fmend = struct.unpack_from(f"<{n_def}I", rec, o)
    entries, s = {}, 0
    for m, e in zip(keys, dend):
        entries[m] = list(zip(dact[s:e], dctr[s:e]))
        s = e
    deferred, s, t = [], 0, 0
    for de, me in zip(fdend, fmend):
        deferred.append((list(zip(fact[s:de], fctr[s:de])), list(fkey[t:me])))
        s, t = de, me
    return dict(size=size, clock={a: c for a, c in zip(cact, clk) if c}, entries=entries, deferred=deferred)


def encode_record(clock, entries, deferred, n_actors, sparse=False):
    """clock {a: c}; entries {m: {a: c}}; deferred {tuple(sorted (a, c)): iterable(m)}.
    sparse: CSR top clock of the clock's nonzero actors (else n_actors dense slots)."""
    mems = sorted(entries)
    runs = [sorted(entries[m].items()) for m in mems]
    defs = sorted((tuple(k), sorted(v)) for k, v in deferred.items())
    n_mem, n_dot, n_def = len(mems), sum(map(len, runs)), len(defs)
    n_def_dot = sum(len(d[0]) for d in defs)
    n_def_mem = sum(len(d[1]) for d in defs)
    cl = sorted((a, c) for a, c in clock.items() if c)
    n_clk = len(cl) if sparse else n_actors
    size = record_bytes(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, sparse)
    out = bytearray(size)
    struct.pack_into("<8I", out, 0, size, n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem,
                     SPARSE_CLOCK if sparse else 0)
    o = HDR
    if sparse:
        struct.pack_into(f"<{n_clk}Q", out, o, *[c for _, c in cl])
        struct.pack_into(f"<{n_clk}I", out, o + 8 * n_clk, *[a for a, _ in cl])
    else:
        clk = [0] * n_actors
        for a, c in cl:
            clk[a] = c
        struct.pack_into(f"<{n_actors}Q", out, o, *clk)
    o += _clock_bytes(n_clk, sparse)
    struct.pack_into(f"<{n_mem}Q", out, o, *mems); o += 8 * n_mem
    struct.pack_into(f"<{n_dot}Q", out, o, *[c for r in runs for _, c in r]); o += 8 * n_dot
    struct.pack_into(f"<{n_dot}I", out, o, *[a for r in runs for a, _ in r]); o += 4 * n_dot
    e, ends = 0, []
    for r in runs:
        e += len(r)
        ends.append(e)
    struct.pack_into(f"<{n_mem}I", out, o, *ends); o = _pad(o + 4 * n_mem, 8)
    struct.pack_into(f"<{n_def_dot}Q", out, o, *[c for d in defs for _, c in d[0]]); o += 8 * n_def_dot
    struct.pack_into(f"<{n_def_mem}Q", out, o, *[m for d in defs for m in d[1]]); o += 8 * n_def_mem
    struct.pack_into(f"<{n_def_dot}I", out, o, *[a for d in defs for a, _ in d[0]]); o += 4 * n_def_dot
    de, me, a, b = [], [], 0, 0
    for d in defs:
        a += len(d[0]); b += len(d[1])
        de.append(a); me.append(b)
    struct.pack_into(f"<{n_def}I", out, o, *de); o += 4 * n_def
    struct.pack_into(f"<{n_def}I", out, o, *me)
    return bytes(out)


def compact_bytes(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, sparse=False):
    """SURVEY.md §8(d)'s algorithmic bytes of one Orswot side in the compact
    layout (no header, no padding): top + 4 + 4 + Σ_members(8 key + 4 dot-off +
    12·dots) + Σ_deferred(4 + 12·dots + 4 + 8·members), top = 8·A dense or
    4 + 12·nnz sparse. Works elementwise on numpy arrays of header counts."""
    top = 4 + 12 * n_clk if sparse else 8 * n_clk
    return top + 8 + 12 * n_mem + 12 * n_dot + 8 * n_def + 12 * n_def_dot + 8 * n_def_mem


def batch_compact_bytes(base, off):
    """Σ compact_bytes over a batch's records, read from their headers
    (base: uint8 numpy buffer, off: record offsets; flags bit 0 per record)."""
    import numpy as np

    w = np.asarray(base)[: len(base) // 4 * 4].view(np.uint32)
    i = (np.asarray(off, dtype=np.uint64) // np.uint64(4)).astype(np.int64)
    h = [w[i + k].astype(np.int64) for k in range(8)]
    sp = (h[7] & SPARSE_CLOCK) != 0
    top = np.where(sp, 4 + 12 * h[1], 8 * h[1])
    return int((top + 8 + 12 * h[2] + 12 * h[3] + 8 * h[4] + 12 * h[5] + 8 * h[6]).sum())
