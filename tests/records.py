"""Pure-Python codec of the canonical Orswot record (layout: include/crdts_hip.h).

Test infrastructure: lets tests build records from the pure-Python restatement
and decode kernel outputs for readable diffs. Independent of the oracle's and
the product's codecs.
"""
from __future__ import annotations

import struct

import numpy as np

HDR = 32


def _pad(x, a):
    return (x + a - 1) // a * a


def record_bytes(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, sparse=False):
    # sparse (CSR) top clock: u64 ctr[n_clk] + u32 act[n_clk], padded to 8
    b = HDR + (_pad(12 * n_clk, 8) if sparse else 8 * n_clk) + 12 * (n_mem + n_dot)
    b = _pad(b, 8)
    b += 12 * n_def_dot + 8 * n_def_mem + 8 * n_def
    return _pad(b, 16)


def _clock_key(pairs):
    return tuple(pairs)  # lexicographic over (actor, counter), prefix first == tuple order


def encode(clock, entries, deferred, n_actors, sparse=False):
    """clock: {a: c}; entries: {m: {a: c}}; deferred: {tuple(sorted pairs): set(m)}.
    sparse: the top clock as CSR (header flags bit 0), n_clk = its nnz."""
    mems = sorted(entries)
    runs = [sorted(entries[m].items()) for m in mems]
    defs = sorted(((tuple(sorted(k)) if not isinstance(k, tuple) else k), sorted(v)) for k, v in deferred.items())
    n_mem, n_dot = len(mems), sum(len(r) for r in runs)
    n_def = len(defs)
    n_def_dot = sum(len(d[0]) for d in defs)
    n_def_mem = sum(len(d[1]) for d in defs)
    pairs = sorted((a, c) for a, c in clock.items() if c)
    n_clk = len(pairs) if sparse else n_actors
    size = record_bytes(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, sparse)
    out = bytearray(size)
    struct.pack_into("<8I", out, 0, size, n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, 1 if sparse else 0)
    o = HDR
    if sparse:
        struct.pack_into(f"<{n_clk}Q", out, o, *[c for _, c in pairs])
        struct.pack_into(f"<{n_clk}I", out, o + 8 * n_clk, *[a for a, _ in pairs])
        o += _pad(12 * n_clk, 8)
    else:
        clk = [0] * n_actors
        for a, c in pairs:
            clk[a] = c
        struct.pack_into(f"<{n_actors}Q", out, o, *clk)
        o += 8 * n_actors
    struct.pack_into(f"<{n_mem}Q", out, o, *mems)
    o += 8 * n_mem
    struct.pack_into(f"<{n_dot}Q", out, o, *[c for r in runs for _, c in r])
    o += 8 * n_dot
    struct.pack_into(f"<{n_dot}I", out, o, *[a for r in runs for a, _ in r])
    o += 4 * n_dot
    ends, e = [], 0
    for r in runs:
        e += len(r)
        ends.append(e)
    struct.pack_into(f"<{n_mem}I", out, o, *ends)
    o = _pad(o + 4 * n_mem, 8)
    struct.pack_into(f"<{n_def_dot}Q", out, o, *[c for d in defs for _, c in d[0]])
    o += 8 * n_def_dot
    struct.pack_into(f"<{n_def_mem}Q", out, o, *[m for d in defs for m in d[1]])
    o += 8 * n_def_mem
    struct.pack_into(f"<{n_def_dot}I", out, o, *[a for d in defs for a, _ in d[0]])
    o += 4 * n_def_dot
    de, me, dd, mm = [], [], 0, 0
    for d in defs:
        dd += len(d[0])
        mm += len(d[1])
        de.append(dd)
        me.append(mm)
    struct.pack_into(f"<{n_def}I", out, o, *de)
    o += 4 * n_def
    struct.pack_into(f"<{n_def}I", out, o, *me)
    return bytes(out)


def decode(rec):
    """Returns dict(clock={a:c}, entries={m:[(a,c)..]}, deferred=[(pairs, members)..], size=)."""
    rec = bytes(rec)
    size, n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem, flags = struct.unpack_from("<8I", rec, 0)
    o = HDR
    clk = struct.unpack_from(f"<{n_clk}Q", rec, o)
    if flags & 1:
        cact = struct.unpack_from(f"<{n_clk}I", rec, o + 8 * n_clk)
        o += _pad(12 * n_clk, 8)
    else:
        cact = range(n_clk)
        o += 8 * n_clk
    keys = struct.unpack_from(f"<{n_mem}Q", rec, o)
    o += 8 * n_mem
    dctr = struct.unpack_from(f"<{n_dot}Q", rec, o)
    o += 8 * n_dot
    dact = struct.unpack_from(f"<{n_dot}I", rec, o)
    o += 4 * n_dot
    dend = struct.unpack_from(f"<{n_mem}I", rec, o)
    o = _pad(o + 4 * n_mem, 8)
    fctr = struct.unpack_from(f"<{n_def_dot}Q", rec, o)
    o += 8 * n_def_dot
    fkey = struct.unpack_from(f"<{n_def_mem}Q", rec, o)
    o += 8 * n_def_mem
    fact = struct.unpack_from(f"<{n_def_dot}I", rec, o)
    o += 4 * n_def_dot
    fdend = struct.unpack_from(f"<{n_def}I", rec, o)
    o += 4 * n_def
    fmend = struct.unpack_from(f"<{n_def}I", rec, o)
    entries, s = {}, 0
    for m, e in zip(keys, dend):
        entries[m] = list(zip(dact[s:e], dctr[s:e]))
        s = e
    deferred, s, t = [], 0, 0
    for de, me in zip(fdend, fmend):
        deferred.append((list(zip(fact[s:de], fctr[s:de])), list(fkey[t:me])))
        s, t = de, me
    return dict(size=size, flags=flags, clock={a: c for a, c in zip(cact, clk) if c},
                entries=entries, deferred=deferred)


def from_py(orswot, n_actors, sparse=False):
    """Encode a crdts_ref.Orswot."""
    return encode(dict(orswot.clock.dots), {m: dict(c.dots) for m, c in orswot.entries.items()},
                  {tuple(sorted(c.dots.items())): set(s) for c, s in orswot.deferred.items()}, n_actors, sparse)


def pack_batch(records, align=16):
    """list of bytes -> (u8 base, u64 offsets)."""
    offs, pos = [], 0
    for r in records:
        offs.append(pos)
        pos += _pad(len(r), align)
    base = np.zeros(max(pos, 16), dtype=np.uint8)
    for o, r in zip(offs, records):
        base[o:o + len(r)] = np.frombuffer(r, dtype=np.uint8)
    return base, np.array(offs, dtype=np.uint64)


def unpack_batch(base, offs):
    base = np.asarray(base, dtype=np.uint8)
    out = []
    for o in np.asarray(offs, dtype=np.uint64).tolist():
        size = int(np.frombuffer(base[o:o + 4].tobytes(), dtype=np.uint32)[0])
        out.append(base[o:o + size].tobytes())
    return out
