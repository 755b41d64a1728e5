"""crdts_hip — MI355X batched state-based CRDT merge (host side, Python).

Mirrors the reference's `CvRDT::merge(&mut self, &other)` (src/traits.rs:9-12)
for VClock / GCounter / PNCounter / Orswot, executed on the GPU through the C
ABI of libcrdts_hip.so (include/crdts_hip.h):

    eng = Engine(0)
    out = eng.orswot_merge(self_batch, other_batch)      # batch join on HBM
    a.merge(b)                                           # one pair, same kernel

Device memory and streams come from torch (plumbing only).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import (CRDT_COMM_ID_BYTES, CRDT_ECAPACITY, CRDT_ENONCANON, CRDT_OK, EXPORTS, LIB_PATH, SPARSE_CLOCK, Batch, CrdtError,
                   GenParams, RepParams, check, lib)
from .record import decode_record, encode_record, record_bytes

__all__ = [
    "Engine", "OrswotBatch", "GenParams", "CrdtError", "generate_orswot", "generate_dense", "HostOrswot",
    "Orswot", "VClock", "GCounter", "PNCounter", "merge_batch", "decode_record", "encode_record",
    "record_bytes", "CONFIG3", "EXPORTS", "LIB_PATH", "CONFIG5", "SPARSE_CLOCK", "generate_replicas", "ClockBatch",
    "generate_clocks_csr", "MapMapSlab",
]

# SURVEY.md §8(d) config 3 / BASELINE.json configs[2].
CONFIG3 = dict(n_actors=16, member_universe=64, ancestor_adds=32, min_div_ops=4, max_div_ops=16, pct_add=60,
               pct_future_rm=10, pct_deferred_obj=8, pct_shared_actor=5)
CONFIG3_SEED = 0xC0FFEE03
# SURVEY.md §8(d) config 5 / BASELINE.json configs[4]: 1024-actor universe, CSR top clocks, 8 replicas.
CONFIG5 = dict(universe=1024, pool_actors=48, own_actors=2, member_universe=64, ancestor_adds=48, min_div_ops=4,
               max_div_ops=16, pct_add=60, pct_future_rm=10, pct_deferred_obj=8)
CONFIG5_SEED = 0xC0FFEE05


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _torch():
    import torch

    return torch


class ClockBatch:
    """A batch of sparse (CSR) clocks (include/crdts_hip.h crdt_clock_csr):
    object i's clock is entries [off[i], off[i] + len[i]) of (act, ctr) —
    actors strictly increasing, counters > 0. Tensors: off int64, len int32,
    act int32, ctr int64 (u64 bits); host numpy or device torch."""

    def __init__(self, off, len_, act, ctr, n_entries=None):
        self.off, self.len, self.act, self.ctr = off, len_, act, ctr
        self.n_obj = int(off.shape[0])
        self.n_entries = int(act.shape[0]) if n_entries is None else int(n_entries)

    @classmethod
    def from_host(cls, off, len_, act, ctr, device=0):
        torch = _torch()
        dev = f"cuda:{device}"

        def t(x, dt, ndt):
            x = np.ascontiguousarray(x, dtype=ndt)
            return torch.from_numpy(x.view(dt) if x.size else np.zeros(1, dt)).to(dev)

        return cls(t(off, np.int64, np.uint64)[: len(off)], t(len_, np.int32, np.uint32)[: len(len_)],
                   t(act, np.int32, np.uint32), t(ctr, np.int64, np.uint64), n_entries=len(act))

    @classmethod
    def from_lists(cls, clocks, device=0):
        """clocks: list of {actor: counter} dicts (or sorted (actor, counter) lists)."""
        runs = [sorted(dict(c).items()) for c in clocks]
        lens = np.array([len(r) for r in runs], np.uint32)
        off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if len(runs) else np.zeros(0, np.uint64)
        act = np.array([a for r in runs for a, _ in r], np.uint32)
        ctr = np.array([c for r in runs for _, c in r], np.uint64)
        return cls.from_host(off, lens, act, ctr, device)

    def cstruct(self):
        from ._lib import ClockCsr

        return ClockCsr(self.off.data_ptr(), self.len.data_ptr(), self.act.data_ptr(), self.ctr.data_ptr(),
                        self.n_obj, self.n_entries)

    def to_host(self):
        return (self.off.cpu().numpy().view(np.uint64), self.len.cpu().numpy().view(np.uint32),
                self.act[: self.n_entries].cpu().numpy().view(np.uint32),
                self.ctr[: self.n_entries].cpu().numpy().view(np.uint64))

    def clocks(self):
        """Host list of sorted (actor, counter) lists, one per object."""
        off, ln, act, ctr = self.to_host()
        return [list(zip(act[o:o + n].tolist(), ctr[o:o + n].tolist())) for o, n in zip(off.tolist(), ln.tolist())]


class OrswotBatch:
    """A batch of canonical Orswot records resident on one GPU.

    base: torch.uint8 device tensor; off: torch.int64 device tensor (u64 offsets).
    flags: 0 (dense top clocks, n_actors slots) or SPARSE_CLOCK (CSR top clocks
    over an actor universe of n_actors ids).
    """

    def __init__(self, base, off, n_actors, nbytes=None, flags=0):
        self.base = base
        self.off = off
        self.flags = int(flags)
        self.n_actors = int(n_actors)
        self.n_obj = int(off.numel())
        self.bytes = int(nbytes if nbytes is not None else base.numel())

    def cbatch(self):
        return Batch(self.base.data_ptr(), self.off.data_ptr(), self.n_obj, self.bytes)

    @classmethod
    def from_host(cls, base, off, n_actors, device=0, flags=0):
        """device: a GPU index, or None / "cpu" for host tensors (the CPU tests' gloo path)."""
        torch = _torch()
        dev = "cpu" if device is None or device == "cpu" else (device if isinstance(device, str) else f"cuda:{device}")
        base = np.ascontiguousarray(base, dtype=np.uint8)
        nb = max(16, (base.nbytes + 15) // 16 * 16)
        b = torch.zeros(nb, dtype=torch.uint8, device=dev)
        if base.nbytes:
            b[: base.nbytes].copy_(torch.from_numpy(base))
        o = torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint64).view(np.int64)).to(dev)
        return cls(b, o, n_actors, nb, flags)

    @classmethod
    def from_records(cls, records, n_actors, device=0, flags=0):
        offs, pos = [], 0
        for r in records:
            offs.append(pos)
            pos += (len(r) + 15) // 16 * 16
        base = np.zeros(max(pos, 16), dtype=np.uint8)
        for o, r in zip(offs, records):
            base[o:o + len(r)] = np.frombuffer(r, dtype=np.uint8)
        return cls.from_host(base, np.array(offs, dtype=np.uint64), n_actors, device, flags)

    def to_host(self):
        base = self.base.cpu().numpy()
        off = self.off.cpu().numpy().view(np.uint64)
        return base, off

    def compact_bytes(self):
        """Σ over the records of SURVEY.md §8(d)'s compact algorithmic bytes
        (record.compact_bytes), from the headers gathered on the device."""
        torch = _torch()
        w = self.base[: self.base.numel() // 4 * 4].view(torch.int32)
        h = w[(self.off // 4)[:, None] + torch.arange(8, device=self.off.device)[None, :]].to(torch.int64)
        sp = (h[:, 7] & SPARSE_CLOCK) != 0
        top = torch.where(sp, 4 + 12 * h[:, 1], 8 * h[:, 1])
        return int((top + 8 + 12 * h[:, 2] + 12 * h[:, 3] + 8 * h[:, 4] + 12 * h[:, 5] + 8 * h[:, 6]).sum().item())

    def records(self):
        base, off = self.to_host()
        out = []
        for o in off.tolist():
            size = int(base[o:o + 4].view(np.uint32)[0])
            out.append(base[o:o + size].tobytes())
        return out


class OrswotOps:
    """A batch of Orswot ops (Op::Add / Op::Rm, src/orswot.rs:38-53) on the
    device, grouped per object in order (crdt_orswot_ops)."""

    ADD, RM = 0, 1

    def __init__(self, obj_end, kind, member, actor, counter, clk_end, clk_act, clk_ctr):
        self.t = (obj_end, kind, member, actor, counter, clk_end, clk_act, clk_ctr)
        self.n_ops = int(kind.numel())
        self.n_clk = int(clk_act.numel())

    def cops(self):
        from ._lib import Ops

        p = [C.c_void_p(t.data_ptr()) if t.numel() else None for t in self.t]
        return Ops(*p, self.n_ops, self.n_clk)

    @classmethod
    def from_lists(cls, per_obj, device=0):
        """per_obj[i] = [("add", actor, counter, member) | ("rm", member, [(actor, counter), ...]), ...]"""
        torch = _torch()
        ends, kind, mem, act, ctr, cend, cact, cctr = [], [], [], [], [], [], [], []
        for ops in per_obj:
            for op in ops:
                if op[0] == "add":
                    kind.append(cls.ADD); act.append(op[1]); ctr.append(op[2]); mem.append(op[3])
                else:
                    kind.append(cls.RM); act.append(0); ctr.append(0); mem.append(op[1])
                    for a, c in op[2]:
                        cact.append(a); cctr.append(c)
                cend.append(len(cact))
            ends.append(len(kind))
        dev = f"cuda:{device}"

        def u64(x):
            return torch.from_numpy(np.asarray(x, dtype=np.uint64).view(np.int64)).to(dev)

        def u32(x):
            return torch.from_numpy(np.asarray(x, dtype=np.uint32).view(np.int32)).to(dev)

        return cls(u64(ends), u32(kind), u64(mem), u32(act), u64(ctr), u64(cend), u32(cact), u64(cctr))


class MapSlab:
    """Dense fixed-capacity slab of Map<u64, MVReg<u64, A>, A> states
    (crdt_map_mvreg_slab, include/crdts_hip.h). Arrays are numpy (host) or
    torch (device) with the shapes below; dtypes u32 / u64 (torch: int32 / int64)."""

    FIELDS = ("clock", "n_keys", "keys", "eclock", "mv_n", "mv_clock", "mv_val", "n_def", "dclock", "dset_n", "dset")

    def __init__(self, arrays, kcap, mcap, dcap, scap):
        self.a = dict(arrays)
        self.kcap, self.mcap, self.dcap, self.scap = kcap, mcap, dcap, scap

    @staticmethod
    def shapes(n, A, kcap, mcap, dcap, scap):
        return {"clock": (n, A), "n_keys": (n,), "keys": (n, kcap), "eclock": (n, kcap, A), "mv_n": (n, kcap),
                "mv_clock": (n, kcap, mcap, A), "mv_val": (n, kcap, mcap), "n_def": (n,), "dclock": (n, dcap, A),
                "dset_n": (n, dcap), "dset": (n, dcap, scap)}

    @classmethod
    def alloc(cls, n, A, kcap, mcap, dcap, scap, device=None):
        out = {}
        for f, shp in cls.shapes(n, A, kcap, mcap, dcap, scap).items():
            u32 = f in ("n_keys", "mv_n", "n_def", "dset_n")
            if device is None:
                out[f] = np.zeros(shp, np.uint32 if u32 else np.uint64)
            else:
                torch = _torch()
                out[f] = torch.zeros(shp, dtype=torch.int32 if u32 else torch.int64, device=device)
        return cls(out, kcap, mcap, dcap, scap)

    def to(self, device):
        torch = _torch()
        return MapSlab({f: torch.from_numpy(np.ascontiguousarray(v).view(np.int32 if v.dtype == np.uint32 else np.int64))
                        .to(device) for f, v in self.a.items()}, self.kcap, self.mcap, self.dcap, self.scap)

    def host(self):
        return MapSlab({f: (v.cpu().numpy().view(np.uint32 if v.dtype.itemsize == 4 else np.uint64)
                            if hasattr(v, "cpu") else v) for f, v in self.a.items()},
                       self.kcap, self.mcap, self.dcap, self.scap)

    def used_masks(self):
        """Per field, a boolean array of its shape: the slots the state uses
        (keys below n_keys, values below mv_n, deferred below n_def, set
        elements below dset_n). Host slabs."""
        a = self.host().a
        key = np.arange(self.kcap)[None, :] < a["n_keys"][:, None]  # [n, kcap]
        val = key[:, :, None] & (np.arange(self.mcap)[None, None, :] < a["mv_n"][:, :, None])  # [n, kcap, mcap]
        dfr = np.arange(self.dcap)[None, :] < a["n_def"][:, None]  # [n, dcap]
        dset = dfr[..., None] & (np.arange(self.scap)[None, None, :] < a["dset_n"][..., None])
        full = lambda f: np.ones(a[f].shape, bool)  # noqa: E731
        per = {"clock": full("clock"), "n_keys": full("n_keys"), "n_def": full("n_def"), "keys": key,
               "eclock": key[..., None], "mv_n": key, "mv_clock": val[..., None], "mv_val": val,
               "dclock": dfr[..., None], "dset_n": dfr, "dset": dset}
        return {f: np.broadcast_to(m, a[f].shape) for f, m in per.items()}

    def canonical(self):
        """Host copy with every slot past its count zeroed (the merge writes
        only the used slots, include/crdts_hip.h)."""
        a = {f: np.array(v, copy=True) for f, v in self.host().a.items()}
        for f, m in self.used_masks().items():
            a[f][~m] = 0
        return MapSlab(a, self.kcap, self.mcap, self.dcap, self.scap)

    def used_bytes(self):
        """Bytes of the used slots (the state's own bytes, not its capacity)."""
        h = self.host().a
        return int(sum(int(m.sum()) * h[f].dtype.itemsize for f, m in self.used_masks().items()))

    def cstruct(self):
        from ._lib import MapSlabC

        ptr = [C.c_void_p(v.data_ptr() if hasattr(v, "data_ptr") else v.ctypes.data) for v in
               (self.a[f] for f in self.FIELDS)]
        return MapSlabC(*ptr, self.kcap, self.mcap, self.dcap, self.scap)


class MapMapSlab:
    """Dense slab of Map<u64, Map<u64, MVReg<u64, A>, A>, A> states — the
    reference's TestMap (crdt_map_map_slab, include/crdts_hip.h): the outer
    map's arrays (shapes below) and `inner`, a MapSlab of n * kcap nested
    maps (key slot k of object i: inner object i * kcap + k)."""

    FIELDS = ("clock", "n_keys", "keys", "eclock", "n_def", "dclock", "dset_n", "dset")

    def __init__(self, arrays, kcap, dcap, scap, inner):
        self.a = dict(arrays)
        self.kcap, self.dcap, self.scap = kcap, dcap, scap
        self.inner = inner

    @property
    def n(self):
        return int(self.a["n_keys"].shape[0])

    @staticmethod
    def shapes(n, A, kcap, dcap, scap):
        return {"clock": (n, A), "n_keys": (n,), "keys": (n, kcap), "eclock": (n, kcap, A), "n_def": (n,),
                "dclock": (n, dcap, A), "dset_n": (n, dcap), "dset": (n, dcap, scap)}

    @classmethod
    def alloc(cls, n, A, kcap, dcap, scap, inner_caps, device=None):
        """inner_caps: (kcap, mcap, dcap, scap) of the nested maps."""
        out = {}
        for f, shp in cls.shapes(n, A, kcap, dcap, scap).items():
            u32 = f in ("n_keys", "n_def", "dset_n")
            if device is None:
                out[f] = np.zeros(shp, np.uint32 if u32 else np.uint64)
            else:
                torch = _torch()
                out[f] = torch.zeros(shp, dtype=torch.int32 if u32 else torch.int64, device=device)
        return cls(out, kcap, dcap, scap, MapSlab.alloc(n * kcap, A, *inner_caps, device=device))

    @property
    def inner_caps(self):
        return (self.inner.kcap, self.inner.mcap, self.inner.dcap, self.inner.scap)

    def to(self, device):
        torch = _torch()
        return MapMapSlab({f: torch.from_numpy(np.ascontiguousarray(v).view(np.int32 if v.dtype == np.uint32
                                                                              else np.int64)).to(device)
                           for f, v in self.a.items()}, self.kcap, self.dcap, self.scap, self.inner.to(device))

    def host(self):
        return MapMapSlab({f: (v.cpu().numpy().view(np.uint32 if v.dtype.itemsize == 4 else np.uint64)
                               if hasattr(v, "cpu") else v) for f, v in self.a.items()},
                          self.kcap, self.dcap, self.scap, self.inner.host())

    def canonical(self):
        """Host copy with every slot past its count zeroed, outer and inner
        (nested maps of unused key slots zeroed whole)."""
        h = self.host()
        a = {f: np.array(v, copy=True) for f, v in h.a.items()}
        key = np.arange(self.kcap)[None, :] < a["n_keys"][:, None]
        dfr = np.arange(self.dcap)[None, :] < a["n_def"][:, None]
        dset = dfr[..., None] & (np.arange(self.scap)[None, None, :] < a["dset_n"][..., None])
        for f, m in (("keys", key), ("eclock", key[..., None]), ("dclock", dfr[..., None]), ("dset_n", dfr),
                     ("dset", dset)):
            a[f][~np.broadcast_to(m, a[f].shape)] = 0
        inner = h.inner.canonical()
        dead = ~key.reshape(-1)
        for f, v in inner.a.items():
            v[dead] = 0
        return MapMapSlab(a, self.kcap, self.dcap, self.scap, inner)

    def used_bytes(self):
        """Bytes of the used slots: the outer map's, and the nested maps' of
        its used key slots (the state's own bytes, not the capacity)."""
        h = self.host()
        a = h.a
        key = np.arange(self.kcap)[None, :] < a["n_keys"][:, None]
        dfr = np.arange(self.dcap)[None, :] < a["n_def"][:, None]
        dset = dfr[..., None] & (np.arange(self.scap)[None, None, :] < a["dset_n"][..., None])
        A = a["clock"].shape[1]
        outer = 8 * A * self.n + 8 * self.n + int(key.sum()) * (8 + 8 * A) + int(dfr.sum()) * (8 * A + 4) + \
            int(dset.sum()) * 8
        used = key.reshape(-1)
        inner = int(sum(int((m.reshape(m.shape[0], -1)[used]).sum()) * h.inner.a[f].dtype.itemsize
                        for f, m in h.inner.used_masks().items()))
        return outer + inner

    def cstruct(self):
        from ._lib import MAP_MAP_FIELDS, MapMapSlabC

        ptr = [C.c_void_p(self.a[f].data_ptr() if hasattr(self.a[f], "data_ptr") else self.a[f].ctypes.data)
               for f in MAP_MAP_FIELDS]
        return MapMapSlabC(*ptr, self.kcap, self.dcap, self.scap, self.inner.cstruct())


class MapOrswotSlab:
    """Dense fixed-capacity slab of Map<u64, Orswot<u64, A>, A> states
    (crdt_map_orswot_slab, include/crdts_hip.h): numpy (host) or torch
    (device) arrays with the shapes below; dtypes u32 / u64 (torch: int32 /
    int64). `caps` = dict(kcap, mcap, vdcap, vscap, dcap, scap)."""

    U32 = ("n_keys", "vn_mem", "vn_def", "vdset_n", "n_def", "dset_n")

    def __init__(self, arrays, caps):
        self.a = dict(arrays)
        self.caps = dict(caps)

    @staticmethod
    def shapes(n, A, kcap, mcap, vdcap, vscap, dcap, scap):
        return {"clock": (n, A), "n_keys": (n,), "keys": (n, kcap), "eclock": (n, kcap, A), "vclock": (n, kcap, A),
                "vn_mem": (n, kcap), "vmem": (n, kcap, mcap), "vmclock": (n, kcap, mcap, A), "vn_def": (n, kcap),
                "vdclock": (n, kcap, vdcap, A), "vdset_n": (n, kcap, vdcap), "vdset": (n, kcap, vdcap, vscap),
                "n_def": (n,), "dclock": (n, dcap, A), "dset_n": (n, dcap), "dset": (n, dcap, scap)}

    @classmethod
    def alloc(cls, n, A, device=None, **caps):
        out = {}
        for f, shp in cls.shapes(n, A, **caps).items():
            u32 = f in cls.U32
            if device is None:
                out[f] = np.zeros(shp, np.uint32 if u32 else np.uint64)
            else:
                torch = _torch()
                out[f] = torch.zeros(shp, dtype=torch.int32 if u32 else torch.int64, device=device)
        return cls(out, caps)

    @property
    def n(self):
        return int(self.a["n_keys"].shape[0])

    def to(self, device):
        torch = _torch()
        return MapOrswotSlab({f: torch.from_numpy(np.ascontiguousarray(v).view(np.int32 if v.dtype == np.uint32
                                                                                 else np.int64)).to(device)
                              for f, v in self.a.items()}, self.caps)

    def host(self):
        return MapOrswotSlab({f: (v.cpu().numpy().view(np.uint32 if v.dtype.itemsize == 4 else np.uint64)
                                  if hasattr(v, "cpu") else v) for f, v in self.a.items()}, self.caps)

    def used_masks(self):
        """Per field, a boolean array of its shape: the slots the state uses
        (key slots below n_keys, members below vn_mem, deferred below vn_def /
        n_def, set elements below their sizes; clocks and counts of used
        slots). Host slabs."""
        a = self.host().a
        kcap, mcap, vdcap, vscap, dcap, scap = (self.caps[k] for k in ("kcap", "mcap", "vdcap", "vscap", "dcap",
                                                                      "scap"))
        key = np.arange(kcap)[None, :] < a["n_keys"][:, None]  # [n, kcap]
        mem = key[:, :, None] & (np.arange(mcap)[None, None, :] < a["vn_mem"][:, :, None])  # [n, kcap, mcap]
        vdef = key[:, :, None] & (np.arange(vdcap)[None, None, :] < a["vn_def"][:, :, None])  # [n, kcap, vdcap]
        vset = vdef[..., None] & (np.arange(vscap)[None, None, None, :] < a["vdset_n"][..., None])
        dfr = np.arange(dcap)[None, :] < a["n_def"][:, None]  # [n, dcap]
        dset = dfr[..., None] & (np.arange(scap)[None, None, :] < a["dset_n"][..., None])
        full = lambda f: np.ones(a[f].shape, bool)  # noqa: E731
        per = {"clock": full("clock"), "n_keys": full("n_keys"), "n_def": full("n_def"), "keys": key,
               "eclock": key[..., None], "vclock": key[..., None], "vn_mem": key, "vn_def": key, "vmem": mem,
               "vmclock": mem[..., None], "vdclock": vdef[..., None], "vdset_n": vdef, "vdset": vset,
               "dclock": dfr[..., None], "dset_n": dfr, "dset": dset}
        return {f: np.broadcast_to(m, a[f].shape) for f, m in per.items()}

    def canonical(self):
        """Host copy with every slot past its count zeroed: the merge writes
        only the used slots (include/crdts_hip.h), so two slabs hold the same
        states iff their canonical forms are equal."""
        a = {f: np.array(v, copy=True) for f, v in self.host().a.items()}
        for f, m in self.used_masks().items():
            a[f][~m] = 0
        return MapOrswotSlab(a, self.caps)

    def used_bytes(self):
        """Bytes of the used slots (the state's own bytes, not its capacity)."""
        h = self.host().a
        return int(sum(int(m.sum()) * h[f].dtype.itemsize for f, m in self.used_masks().items()))

    def cstruct(self):
        from ._lib import MAP_ORSWOT_CAPS, MAP_ORSWOT_FIELDS, MapOrswotSlabC

        ptr = [C.c_void_p(self.a[f].data_ptr() if hasattr(self.a[f], "data_ptr") else self.a[f].ctypes.data)
               for f in MAP_ORSWOT_FIELDS]
        return MapOrswotSlabC(*ptr, *[self.caps[k] for k in MAP_ORSWOT_CAPS])


class Engine:
    """One crdt_ctx bound to a device. All merges run on the GPU."""

    def __init__(self, device=0):
        torch = _torch()
        if not torch.cuda.is_available():
            raise CrdtError(-6, "Engine needs a visible gfx950 GPU")
        self.device = int(device)
        torch.cuda.set_device(self.device)
        ctx = C.c_void_p()
        check(lib.crdt_ctx_create(C.byref(ctx), self.device), "crdt_ctx_create")
        self.ctx = ctx

    def __del__(self):
        if getattr(self, "ctx", None) is not None and lib is not None:
            lib.crdt_ctx_destroy(self.ctx)
            self.ctx = None

    def _stream(self, stream=None):
        torch = _torch()
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return C.c_void_p(s.cuda_stream)

    @staticmethod
    def _diag(name):
        if not hasattr(lib, name):
            raise RuntimeError(f"{name}: diagnostic build only (make -C rust-crdt_amd diag; CRDTS_HIP_DIAG=1)")
        return getattr(lib, name)

    def set_blocks_per_cu(self, k):
        """Diagnostic build only: workgroups per CU of the Orswot kernel."""
        check(self._diag("crdt_ctx_set_blocks_per_cu")(self.ctx, int(k)), "set_blocks_per_cu")

    def set_variant(self, v):
        """Diagnostic build only: Orswot kernel variant (0 = the product kernel)."""
        check(self._diag("crdt_ctx_set_variant")(self.ctx, int(v)), "set_variant")

    def set_list_cap(self, cap):
        """Test knob: capacity of the general-path object list (overflow -> full scan)."""
        check(lib.crdt_ctx_set_list_cap(self.ctx, int(cap)), "set_list_cap")

    def status(self, stream=None):
        rc = lib.crdt_ctx_status(self.ctx, self._stream(stream))
        check(rc, "kernel status")

    # ---------------------------------------------------------------- Orswot
    def orswot_alloc_out(self, L: OrswotBatch, R: OrswotBatch):
        torch = _torch()
        nb = L.bytes + R.bytes
        base = torch.empty(nb, dtype=torch.uint8, device=f"cuda:{self.device}")
        off = torch.empty(L.n_obj, dtype=torch.int64, device=f"cuda:{self.device}")
        return OrswotBatch(base, off, L.n_actors, nb, L.flags)

    def orswot_merge(self, L: OrswotBatch, R: OrswotBatch, out: OrswotBatch | None = None, stream=None,
                     check_status=True):
        """out[i] = L[i].merge(&R[i])  (src/orswot.rs:87-157). Async unless check_status."""
        if L.n_actors != R.n_actors or L.n_obj != R.n_obj or L.flags != R.flags:
            raise CrdtError(-1, "batch shapes differ")
        if out is None:
            out = self.orswot_alloc_out(L, R)
        lb, rb = L.cbatch(), R.cbatch()
        out.flags = L.flags
        rc = lib.crdt_orswot_merge_ex(self.ctx, C.byref(lb), C.byref(rb), C.c_void_p(out.base.data_ptr()),
                                      C.c_void_p(out.off.data_ptr()), out.bytes, L.n_actors, L.flags,
                                      self._stream(stream))
        check(rc, "crdt_orswot_merge")
        if check_status:
            self.status(stream)
        return out

    def orswot_fold(self, batches, out: OrswotBatch | None = None, stream=None, check_status=True):
        """((b0 ⊔ b1) ⊔ b2) ⊔ ... of batches of the same objects (crdt_orswot_fold:
        the rank-order fold of replica anti-entropy, R - 1 batched merges).
        Returns an OrswotBatch (`out`, reused, when given: at least the
        batches' bytes together and n_obj offsets)."""
        torch = _torch()
        B0 = batches[0]
        total = sum(B.bytes for B in batches)
        if out is None:
            out = OrswotBatch(torch.empty(max(16, total), dtype=torch.uint8, device=B0.base.device),
                              torch.empty(B0.n_obj, dtype=torch.int64, device=B0.base.device), B0.n_actors,
                              max(16, total), B0.flags)
        arr = (Batch * len(batches))(*[B.cbatch() for B in batches])
        check(lib.crdt_orswot_fold(self.ctx, arr, len(batches), B0.n_actors, B0.flags,
                                   C.c_void_p(out.base.data_ptr()), C.c_void_p(out.off.data_ptr()), out.bytes,
                                   self._stream(stream)), "orswot_fold")
        if check_status:
            self.status(stream)
        return out

    def orswot_validate(self, B: OrswotBatch, stream=None):
        b = B.cbatch()
        check(lib.crdt_orswot_validate_ex(self.ctx, C.byref(b), B.n_actors, B.flags, self._stream(stream)),
              "validate")
        self.status(stream)

    def orswot_compact(self, B: OrswotBatch, stream=None):
        torch = _torch()
        dev = f"cuda:{self.device}"
        scratch = torch.empty(int(lib.crdt_orswot_compact_scratch_bytes(B.n_obj)), dtype=torch.uint8, device=dev)
        dst = torch.empty(B.bytes, dtype=torch.uint8, device=dev)
        doff = torch.empty(B.n_obj, dtype=torch.int64, device=dev)
        b = B.cbatch()
        check(lib.crdt_orswot_compact(self.ctx, C.byref(b), C.c_void_p(dst.data_ptr()),
                                      C.c_void_p(doff.data_ptr()), B.bytes, C.c_void_p(scratch.data_ptr()),
                                      self._stream(stream)), "compact")
        torch.cuda.synchronize(self.device)
        used = 0
        if B.n_obj:
            last = int(doff[-1].item())
            used = last + int(dst[last:last + 4].cpu().numpy().view(np.uint32)[0])
        return OrswotBatch(dst, doff, B.n_actors, max(16, (used + 15) // 16 * 16), B.flags)

    # ------------------------------------------------ replica anti-entropy (RCCL)
    @staticmethod
    def comm_unique_id() -> bytes:
        """crdt_comm_unique_id: the RCCL id rank 0 hands to every rank."""
        buf = (C.c_uint8 * CRDT_COMM_ID_BYTES)()
        check(lib.crdt_comm_unique_id(buf), "comm_unique_id")
        return bytes(buf)

    def comm_init(self, uid: bytes, n_ranks: int, rank: int):
        """crdt_comm_init (collective): this context owns an RCCL communicator."""
        if len(uid) != CRDT_COMM_ID_BYTES:
            raise CrdtError(-1, "comm id must be CRDT_COMM_ID_BYTES bytes")
        buf = (C.c_uint8 * CRDT_COMM_ID_BYTES).from_buffer_copy(uid)
        check(lib.crdt_comm_init(self.ctx, buf, int(n_ranks), int(rank)), "comm_init")
        self.n_ranks, self.rank = int(n_ranks), int(rank)

    @property
    def has_comm(self):
        return getattr(self, "n_ranks", 0) > 0

    def comm_destroy(self):
        check(lib.crdt_comm_destroy(self.ctx), "comm_destroy")
        self.n_ranks = 0

    def replica_allreduce_max(self, rows, stream=None):
        """In place: rows := max over ranks (u64 order), ncclUint64 + ncclMax
        (src/vclock.rs:131-137 across replicas). rows: int64 device tensor of u64."""
        check(lib.crdt_replica_allreduce_max(self.ctx, C.c_void_p(rows.data_ptr()), rows.numel(),
                                             self._stream(stream)), "replica_allreduce_max")
        return rows

    def replica_reduce_scatter_max(self, rows, stream=None):
        """The owner shard of the u64 max over ranks: rank r gets words
        [r n/N, (r+1) n/N) (crdt_replica_reduce_scatter_max). Returns a new
        int64 device tensor of n/N words."""
        torch = _torch()
        flat = rows.reshape(-1)
        n_ranks = self.n_ranks
        if flat.numel() % n_ranks:
            raise CrdtError(-1, "reduce_scatter: word count not a multiple of the rank count")
        out = torch.empty(flat.numel() // n_ranks, dtype=torch.int64, device=flat.device)
        check(lib.crdt_replica_reduce_scatter_max(self.ctx, C.c_void_p(flat.data_ptr()), flat.numel(),
                                                  C.c_void_p(out.data_ptr()), self._stream(stream)),
              "replica_reduce_scatter_max")
        return out

    def set_arena_limit(self, max_bytes):
        """Largest replica-exchange arena the context may allocate (0: no limit; crdt_ctx_set_arena_limit)."""
        check(lib.crdt_ctx_set_arena_limit(self.ctx, int(max_bytes)), "set_arena_limit")

    def host_syncs(self):
        """Host synchronisations the context's replica joins made so far (crdt_ctx_host_syncs)."""
        return int(lib.crdt_ctx_host_syncs(self.ctx))

    def comm_count(self):
        """Ranks of the context's RCCL communicator (ncclCommCount)."""
        n = C.c_int(0)
        check(lib.crdt_comm_count(self.ctx, C.byref(n)), "comm_count")
        return n.value

    def orswot_replica_join_bound(self, B: OrswotBatch, stream=None):
        """Output bytes that suffice for crdt_orswot_replica_join (collective:
        the sum of every rank's replica bytes)."""
        b = B.cbatch()
        bound = C.c_size_t(0)
        check(lib.crdt_orswot_replica_join_bound(self.ctx, C.byref(b), C.byref(bound), self._stream(stream)),
              "replica_join_bound")
        return max(16, bound.value)

    def orswot_replica_alloc_out(self, B: OrswotBatch, bound: int):
        torch = _torch()
        dev = f"cuda:{self.device}"
        return OrswotBatch(torch.empty(max(16, bound), dtype=torch.uint8, device=dev),
                           torch.empty(B.n_obj, dtype=torch.int64, device=dev), B.n_actors, max(16, bound), B.flags)

    def orswot_replica_join(self, B: OrswotBatch, out: OrswotBatch | None = None, stream=None):
        """((r0 ⊔ r1) ⊔ ...) of every rank's replica, owner-sharded over RCCL;
        the same packed batch on every rank (crdt_orswot_replica_join). `out`
        (from orswot_replica_alloc_out with a bound from
        orswot_replica_join_bound) is reused when given, so a repeated join
        runs no bound collective and allocates nothing."""
        if out is None:
            out = self.orswot_replica_alloc_out(B, self.orswot_replica_join_bound(B, stream))
        b = B.cbatch()
        used = C.c_size_t(0)
        check(lib.crdt_orswot_replica_join(self.ctx, C.byref(b), B.n_actors, B.flags,
                                           C.c_void_p(out.base.data_ptr()), C.c_void_p(out.off.data_ptr()),
                                           out.base.numel(), C.byref(used), self._stream(stream)),
              "orswot_replica_join")
        return OrswotBatch(out.base, out.off, B.n_actors, max(16, used.value), B.flags)

    def orswot_replica_join_transport(self, B: OrswotBatch, transport, out: OrswotBatch | None = None,
                                      out_bytes: int | None = None, stream=None):
        """The same owner-sharded join over a caller transport
        (crdt_orswot_replica_join_transport; `transport` has a `.c` TransportC,
        e.g. replica.GlooTransport). out_bytes defaults to world x this
        replica's bytes rounded up (enough when replicas are of similar size;
        pass the all-reduced sum otherwise)."""
        if out is None:
            cap = out_bytes if out_bytes is not None else transport.world * ((B.bytes + 15) // 16 * 16 + 16)
            out = self.orswot_replica_alloc_out(B, cap)
        b = B.cbatch()
        used = C.c_size_t(0)
        check(lib.crdt_orswot_replica_join_transport(self.ctx, C.byref(transport.c), C.byref(b), B.n_actors,
                                                     B.flags, C.c_void_p(out.base.data_ptr()),
                                                     C.c_void_p(out.off.data_ptr()), out.base.numel(),
                                                     C.byref(used), self._stream(stream)),
              "orswot_replica_join_transport")
        return OrswotBatch(out.base, out.off, B.n_actors, max(16, used.value), B.flags)

    def replica_allreduce_max_transport(self, rows, transport, stream=None):
        """rows (a device int64 tensor read as u64) := its max over ranks, in
        place, over a caller transport (crdt_replica_allreduce_max_transport:
        owner-sharded reduce-scatter with the dense max kernel + all-gather;
        `transport` has a `.c` TransportC, e.g. replica.GlooTransport)."""
        check(lib.crdt_replica_allreduce_max_transport(self.ctx, C.byref(transport.c), C.c_void_p(rows.data_ptr()),
                                                       rows.numel(), self._stream(stream)),
              "replica_allreduce_max_transport")
        return rows

    def replica_reduce_scatter_max_transport(self, rows, transport, stream=None):
        """The owner shard of the u64 max over ranks over a caller transport
        (crdt_replica_reduce_scatter_max_transport): rank r gets words
        [r n/N, (r+1) n/N). Returns a new int64 device tensor of n/N words.
        A word count N does not divide is CRDT_EINVAL on EVERY rank: the C ABI
        checks it with the peers (a local early return here would leave them
        waiting in the exchange)."""
        torch = _torch()
        flat = rows.reshape(-1)
        out = torch.empty(max(1, flat.numel() // transport.world), dtype=torch.int64, device=flat.device)
        check(lib.crdt_replica_reduce_scatter_max_transport(self.ctx, C.byref(transport.c),
                                                            C.c_void_p(flat.data_ptr()), flat.numel(),
                                                            C.c_void_p(out.data_ptr()), self._stream(stream)),
              "replica_reduce_scatter_max_transport")
        return out[: flat.numel() // transport.world]

    def orswot_replica_join_local(self, batches, stream=None):
        """The same owner-sharded join with every replica a virtual rank on this
        device (crdt_orswot_replica_join_local)."""
        torch = _torch()
        arr = (Batch * len(batches))(*[x.cbatch() for x in batches])
        cap = sum((x.bytes + 15) // 16 * 16 for x in batches)
        dev = f"cuda:{self.device}"
        base = torch.empty(max(16, cap), dtype=torch.uint8, device=dev)
        off = torch.empty(batches[0].n_obj, dtype=torch.int64, device=dev)
        used = C.c_size_t(0)
        check(lib.crdt_orswot_replica_join_local(self.ctx, arr, len(batches), batches[0].n_actors, batches[0].flags,
                                                 C.c_void_p(base.data_ptr()), C.c_void_p(off.data_ptr()),
                                                 base.numel(), C.byref(used), self._stream(stream)),
              "orswot_replica_join_local")
        return OrswotBatch(base, off, batches[0].n_actors, max(16, used.value), batches[0].flags)

    # ---------------------------------------------------------------- dense
    # ------------------------------------------------ VClock order / MVReg
    def vclock_partial_cmp(self, a_rows, b_rows, n_actors, stream=None):
        """partial_cmp of dense rows (src/vclock.rs:59-71): int8 tensor of
        0 Equal, 1 Greater, -1 Less, 2 None."""
        torch = _torch()
        n = int(a_rows.numel()) // n_actors
        out = torch.empty(n, dtype=torch.int8, device=a_rows.device)
        check(lib.crdt_vclock_partial_cmp(self.ctx, C.c_void_p(a_rows.data_ptr()), C.c_void_p(b_rows.data_ptr()), n,
                                          n_actors, C.c_void_p(out.data_ptr()), self._stream(stream)),
              "vclock_partial_cmp")
        return out

    def mvreg_merge(self, self_slab, other_slab, n_actors, out_cap=None, stream=None, check_status=True):
        """MVReg<u64, A>::merge (src/mvreg.rs:121-153) over slabs (n, clocks[n][cap][A], vals[n][cap])
        of int32 / int64 device tensors; returns the output slab."""
        torch = _torch()
        sn, sc, sv = self_slab
        on, oc, ov = other_slab
        n_obj, scap, ocap = int(sn.numel()), int(sv.shape[1]), int(ov.shape[1])
        cap = out_cap or scap + ocap
        dev = sn.device
        outn = torch.empty(n_obj, dtype=torch.int32, device=dev)
        outc = torch.empty((n_obj, cap, n_actors), dtype=torch.int64, device=dev)
        outv = torch.empty((n_obj, cap), dtype=torch.int64, device=dev)
        p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        check(lib.crdt_mvreg_merge(self.ctx, p(sn), p(sc), p(sv), scap, p(on), p(oc), p(ov), ocap, p(outn), p(outc),
                                   p(outv), cap, n_obj, n_actors, self._stream(stream)), "mvreg_merge")
        if check_status:
            self.status(stream)
        return outn, outc, outv

    # ------------------------------------------------ Map<u64, MVReg<u64>>
    def map_mvreg_merge(self, S: "MapSlab", O: "MapSlab", n_actors, stream=None, check_status=True, out=None):
        """Map::merge (src/map.rs:191-268) of device slabs; returns the output slab
        (capacities = the sums of the inputs'). Only the used slots of the
        output are written (`out`, if given, is reused as it is)."""
        n = int(S.a["n_keys"].shape[0])
        R = out if out is not None else MapSlab.alloc(n, n_actors, S.kcap + O.kcap, S.mcap + O.mcap,
                                                      S.dcap + O.dcap, S.scap + O.scap, device=S.a["clock"].device)
        s, o, r = S.cstruct(), O.cstruct(), R.cstruct()
        check(lib.crdt_map_mvreg_merge(self.ctx, C.byref(s), C.byref(o), C.byref(r), n, n_actors,
                                       self._stream(stream)), "map_mvreg_merge")
        if check_status:
            self.status(stream)
        return R

    # ------------------------------------------------ Map<u64, Map<u64, MVReg<u64>>>
    def map_map_merge(self, S: "MapMapSlab", O: "MapMapSlab", n_actors, stream=None, check_status=True, out=None):
        """Map::merge of nested maps (src/map.rs:191-268 with the inner map as
        the value: its merge and Causal::truncate) of device slabs; returns
        the output slab (capacities: the sums of the inputs', outer and inner)."""
        torch = _torch()
        n = S.n
        R = out if out is not None else MapMapSlab.alloc(
            n, n_actors, S.kcap + O.kcap, S.dcap + O.dcap, S.scap + O.scap,
            tuple(x + y for x, y in zip(S.inner_caps, O.inner_caps)), device=S.a["clock"].device)
        s, o, r = S.cstruct(), O.cstruct(), R.cstruct()
        nb = int(lib.crdt_map_map_merge_scratch_bytes(C.byref(r), n, n_actors))
        # the engine keeps the scratch (grown as needed): a launch in flight on
        # another stream never sees it freed
        sc = getattr(self, "_map_map_scratch", None)
        if sc is None or sc.numel() < nb or sc.device != S.a["clock"].device:
            sc = self._map_map_scratch = torch.empty(max(16, nb), dtype=torch.uint8, device=S.a["clock"].device)
        check(lib.crdt_map_map_merge(self.ctx, C.byref(s), C.byref(o), C.byref(r), n, n_actors,
                                     C.c_void_p(sc.data_ptr()), int(sc.numel()), self._stream(stream)),
              "map_map_merge")
        if check_status:
            self.status(stream)
        return R

    # ------------------------------------------------ Map<u64, Orswot<u64>>
    def map_orswot_merge(self, S: "MapOrswotSlab", O: "MapOrswotSlab", n_actors, out_caps=None, stream=None,
                         check_status=True, out=None):
        """Map::merge with Orswot values (src/map.rs:192-269) of device slabs;
        returns the output slab (default capacities: the sums of the inputs').
        Only the used slots of the output are written (`out`, if given, is
        reused as it is: compare `.canonical()` forms)."""
        n = S.n
        caps = out_caps or {k: S.caps[k] + O.caps[k] for k in S.caps}
        R = out if out is not None else MapOrswotSlab.alloc(n, n_actors, device=S.a["clock"].device, **caps)
        s, o, r = S.cstruct(), O.cstruct(), R.cstruct()
        check(lib.crdt_map_orswot_merge(self.ctx, C.byref(s), C.byref(o), C.byref(r), n, n_actors,
                                        self._stream(stream)), "map_orswot_merge")
        if check_status:
            self.status(stream)
        return R

    # ------------------------------------------------ batched op path
    def orswot_apply(self, B: "OrswotBatch", ops: "OrswotOps", stream=None, check_status=True):
        """out[i] = B[i] after CmRDT::apply of object i's ops in order
        (src/orswot.rs:61-85). Returns an OrswotBatch."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        per_op = 48 if B.flags & SPARSE_CLOCK else 32  # include/crdts_hip.h: output reservation per op
        cap = B.bytes + per_op * ops.n_ops + 16 * ops.n_clk + 32 * B.n_obj
        base = torch.empty(max(16, cap), dtype=torch.uint8, device=dev)
        off = torch.empty(B.n_obj, dtype=torch.int64, device=dev)
        b = B.cbatch()
        o = ops.cops()
        check(lib.crdt_orswot_apply(self.ctx, C.byref(b), C.byref(o), B.n_actors, B.flags,
                                    C.c_void_p(base.data_ptr()), C.c_void_p(off.data_ptr()), int(base.numel()),
                                    self._stream(stream)), "orswot_apply")
        if check_status:
            self.status(stream)
        return OrswotBatch(base, off, B.n_actors, int(base.numel()), B.flags)

    # ------------------------------------------------ bincode ingest / egest
    def orswot_from_bincode(self, blobs, blob_off, blob_len, n_actors, actor_bytes, member_bytes, flags=0,
                            stream=None, check_status=True, packed=True):
        """Records from the reference's binary form (`from_binary`, src/lib.rs:78-83).

        blobs: torch.uint8 device tensor; blob_off / blob_len: torch.int64 device
        tensors (u64). Returns an OrswotBatch of canonical records: packed
        (a sizes pass walks every blob first), or with packed=False placed by
        crdt_orswot_bincode_record_bounds (blob lengths only: every blob is
        read once; the batch has gaps)."""
        torch = _torch()
        n = int(blob_off.numel())
        dev = f"cuda:{self.device}"
        st = self._stream(stream)
        sizes = torch.empty(n, dtype=torch.int64, device=dev)
        if packed:
            check(lib.crdt_orswot_bincode_record_sizes(self.ctx, C.c_void_p(blobs.data_ptr()), int(blobs.numel()),
                                                       C.c_void_p(blob_off.data_ptr()),
                                                       C.c_void_p(blob_len.data_ptr()), n, actor_bytes, member_bytes,
                                                       n_actors, flags, C.c_void_p(sizes.data_ptr()), st),
                  "bincode_record_sizes")
        else:
            check(lib.crdt_orswot_bincode_record_bounds(self.ctx, C.c_void_p(blob_len.data_ptr()), n, actor_bytes,
                                                        member_bytes, n_actors, flags, C.c_void_p(sizes.data_ptr()),
                                                        st), "bincode_record_bounds")
        with torch.cuda.stream(stream) if stream is not None else _nullctx():
            ends = torch.cumsum(sizes, 0)
            total = int(ends[-1].item()) if n else 0
            off = ends - sizes
        base = torch.empty(max(16, total), dtype=torch.uint8, device=dev)
        check(lib.crdt_orswot_from_bincode(self.ctx, C.c_void_p(blobs.data_ptr()), int(blobs.numel()),
                                           C.c_void_p(blob_off.data_ptr()), C.c_void_p(blob_len.data_ptr()), n,
                                           actor_bytes, member_bytes, n_actors, flags, C.c_void_p(base.data_ptr()),
                                           C.c_void_p(off.data_ptr()), int(base.numel()), st), "from_bincode")
        if check_status:
            self.status(stream)
        return OrswotBatch(base, off, n_actors, int(base.numel()), flags)

    def orswot_to_bincode(self, B: "OrswotBatch", actor_bytes, member_bytes, stream=None, check_status=True):
        """The reference's binary form (`to_binary`, src/lib.rs:62-64) of every
        record: (blobs uint8, blob_off int64, blob_len int64) device tensors;
        blob i starts 16-B aligned and is zero-padded to 16."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        st = self._stream(stream)
        b = B.cbatch()
        lens = torch.empty(B.n_obj, dtype=torch.int64, device=dev)
        check(lib.crdt_orswot_bincode_sizes(self.ctx, C.byref(b), B.n_actors, B.flags, actor_bytes, member_bytes,
                                            C.c_void_p(lens.data_ptr()), st), "bincode_sizes")
        with torch.cuda.stream(stream) if stream is not None else _nullctx():
            padded = (lens + 15) // 16 * 16
            ends = torch.cumsum(padded, 0)
            total = int(ends[-1].item()) if B.n_obj else 0
            off = ends - padded
        out = torch.empty(max(16, total), dtype=torch.uint8, device=dev)
        check(lib.crdt_orswot_to_bincode(self.ctx, C.byref(b), B.n_actors, B.flags, actor_bytes, member_bytes,
                                         C.c_void_p(out.data_ptr()), C.c_void_p(off.data_ptr()), int(out.numel()),
                                         st), "to_bincode")
        if check_status:
            self.status(stream)
        return out, off, lens

    def orswot_truncate(self, B: OrswotBatch, clocks: "ClockBatch", out: "OrswotBatch | None" = None, stream=None,
                        check_status=True):
        """out[i] = B[i] after Causal::truncate(&clocks[i]) (src/orswot.rs:159-172),
        written at B.off[i] (crdt_orswot_truncate). Returns an OrswotBatch
        (`out`, reused, when given: at least B.bytes bytes and B.n_obj offsets;
        it must not share memory with B's records — the call is not in place,
        CRDT_EINVAL)."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        if out is not None:
            base, off = out.base, out.off
            if base.numel() < B.bytes or off.numel() < B.n_obj:
                raise ValueError("orswot_truncate: `out` is smaller than the input batch")
        else:
            base = torch.empty(max(16, B.bytes), dtype=torch.uint8, device=dev)
            off = torch.empty(B.n_obj, dtype=torch.int64, device=dev)
        b, c = B.cbatch(), clocks.cstruct()
        check(lib.crdt_orswot_truncate(self.ctx, C.byref(b), C.byref(c), B.n_actors, B.flags,
                                       C.c_void_p(base.data_ptr()), C.c_void_p(off.data_ptr()), base.numel(),
                                       self._stream(stream)), "orswot_truncate")
        if check_status:
            self.status(stream)
        return OrswotBatch(base, off, B.n_actors, base.numel(), B.flags)

    # ------------------------------------------------ sparse (CSR) clocks
    def clock_csr_alloc_out(self, S: "ClockBatch", O: "ClockBatch"):
        torch = _torch()
        dev = f"cuda:{self.device}"
        cap = max(1, S.n_entries + O.n_entries)
        return ClockBatch(torch.empty(S.n_obj, dtype=torch.int64, device=dev),
                          torch.empty(S.n_obj, dtype=torch.int32, device=dev),
                          torch.empty(cap, dtype=torch.int32, device=dev),
                          torch.empty(cap, dtype=torch.int64, device=dev), n_entries=cap)

    def clock_csr_merge(self, S: "ClockBatch", O: "ClockBatch", out: "ClockBatch | None" = None, kind="vclock",
                        stream=None, check_status=True):
        """out[i] = S[i].merge(&O[i]) over sparse clocks (VClock::merge
        src/vclock.rs:131-137; GCounter src/gcounter.rs:58-62): the sorted union,
        counters max'ed, placed at S.off + O.off (crdt_vclock_csr_merge)."""
        from ._lib import ClockCsrOut

        out = out or self.clock_csr_alloc_out(S, O)
        s, o = S.cstruct(), O.cstruct()
        w = ClockCsrOut(out.off.data_ptr(), out.len.data_ptr(), out.act.data_ptr(), out.ctr.data_ptr(), out.n_entries)
        fn = {"vclock": lib.crdt_vclock_csr_merge, "gcounter": lib.crdt_gcounter_csr_merge}[kind]
        check(fn(self.ctx, C.byref(s), C.byref(o), C.byref(w), self._stream(stream)), f"{kind}_csr_merge")
        if check_status:
            self.status(stream)
        return out

    def pncounter_csr_merge(self, SP, SN, OP, ON, outs=None, stream=None, check_status=True):
        """PNCounter::merge (src/pncounter.rs:90-95) over sparse P and N clocks
        (crdt_pncounter_csr_merge); returns (out_p, out_n)."""
        from ._lib import ClockCsrOut

        op, on = outs or (self.clock_csr_alloc_out(SP, OP), self.clock_csr_alloc_out(SN, ON))
        w = [ClockCsrOut(x.off.data_ptr(), x.len.data_ptr(), x.act.data_ptr(), x.ctr.data_ptr(), x.n_entries)
             for x in (op, on)]
        c = [x.cstruct() for x in (SP, SN, OP, ON)]
        check(lib.crdt_pncounter_csr_merge(self.ctx, *[C.byref(x) for x in c], C.byref(w[0]), C.byref(w[1]),
                                           self._stream(stream)), "pncounter_csr_merge")
        if check_status:
            self.status(stream)
        return op, on

    def dense_merge(self, self_rows, other_rows, n_actors, kind="gcounter", stream=None):
        """In place: self_rows = max(self_rows, other_rows) (src/vclock.rs:131-137).

        Rows are torch int64 device tensors holding u64 counters; shape
        [n_obj, n_actors] (vclock / gcounter) or [n_obj, 2*n_actors] (pncounter).
        """
        fn = {"vclock": lib.crdt_vclock_dense_merge, "gcounter": lib.crdt_gcounter_merge,
              "pncounter": lib.crdt_pncounter_merge}[kind]
        slots = n_actors * (2 if kind == "pncounter" else 1)
        if self_rows.numel() != other_rows.numel() or self_rows.numel() % slots:
            raise CrdtError(-1, "dense rows shape mismatch")
        n_obj = self_rows.numel() // slots
        check(fn(self.ctx, C.c_void_p(self_rows.data_ptr()), C.c_void_p(other_rows.data_ptr()), n_obj,
                 n_actors, self._stream(stream)), f"dense merge ({kind})")
        return self_rows


# -------------------------------------------------------------- generators
def _params(p):
    if isinstance(p, GenParams):
        return p
    d = dict(CONFIG3)
    d.update(p or {})
    return GenParams(**{k: int(v) for k, v in d.items()})


def generate_orswot(n_obj, first_obj=0, seed=CONFIG3_SEED, params=None, threads=8):
    """Host op-simulation generator (see include/crdts_hip.h). Returns
    ((L_base, L_off), (R_base, R_off)) as numpy arrays (copies)."""
    P = _params(params)
    g = C.c_void_p()
    check(lib.crdt_orswot_generate(seed, first_obj, n_obj, C.byref(P), threads, C.byref(g)), "generate")
    try:
        sides = _copy_sides(g, 2, n_obj)
        return sides[0], sides[1]
    finally:
        lib.crdt_orswot_gen_free(g)


TAIL_SEED = 0xC0FFEE06
TAIL_SIZES = (100, 300, 1000)


def generate_orswot_tail(n_obj, frac=0.05, sizes=TAIL_SIZES, first_obj=0, seed=CONFIG3_SEED, threads=8):
    """Config 3 with a heavy tail (bench.py --workload orswot_tail): object i
    is heavy iff (first_obj + i) % round(1 / frac) == 0; heavy objects take
    the sizes in turn, an object of size m being op-simulated over a member
    universe of m keys with m ancestor adds and m/8..m/4 divergent ops per
    side (so ~m members per side: the reference's entries map is unbounded,
    src/orswot.rs:26-30); the others are config-3 objects. The same object
    index gets the same pair at any batch split. Returns ((L_base, L_off),
    (R_base, R_off)) as numpy arrays."""
    def base(n, first):
        return generate_orswot(n, first_obj=first, seed=seed, threads=threads)

    def heavy_gen(n, first, m, params):
        return generate_orswot(n, first_obj=first, seed=TAIL_SEED + m, threads=threads, params=params)

    return _tail_batch(n_obj, frac, sizes, first_obj, base, heavy_gen)


def generate_orswot_csr_tail(n_obj, frac=0.05, sizes=TAIL_SIZES, first_obj=0, seed=CONFIG5_SEED, threads=8):
    """Config 5's record form with a heavy tail (bench.py --workload
    orswot_csr_tail): replicas 0 and 1 of the config-5 replica generator (CSR
    top clocks over the 1 024-actor universe) as the self and other batches,
    object i heavy iff (first_obj + i) % round(1 / frac) == 0, heavy objects
    at the sizes in turn (member universe m, m ancestor adds, m/8..m/4
    divergent ops per replica: ~m members per side; the reference's entries
    map and clock are unbounded, src/orswot.rs:26-30, src/vclock.rs:54-57).
    Split-invariant like generate_orswot_tail. Returns ((L_base, L_off),
    (R_base, R_off)) as numpy arrays, every record with the sparse-clock flag."""
    def base(n, first):
        return tuple(generate_replicas(n, 2, first_obj=first, seed=seed, threads=threads))

    def heavy_gen(n, first, m, params):
        return tuple(generate_replicas(n, 2, first_obj=first, seed=TAIL_SEED + 0x5000 + m, threads=threads,
                                       params=params))

    return _tail_batch(n_obj, frac, sizes, first_obj, base, heavy_gen)


def _tail_batch(n_obj, frac, sizes, first_obj, base, heavy_gen):
    """The heavy-tail batch assembly shared by generate_orswot_tail and
    generate_orswot_csr_tail: base(n, first) -> the ordinary pairs of objects
    [first, first + n); heavy_gen(n, first, m, params) -> n heavy pairs of size
    m (pair index first..)."""
    step = max(1, int(round(1.0 / frac)))
    ids = np.arange(first_obj, first_obj + n_obj, dtype=np.int64)
    heavy = ids % step == 0
    kind = np.where(heavy, 1 + (ids // step) % len(sizes), 0)
    parts = []  # per kind: (positions, (lb, lo), (rb, ro))
    for k in range(len(sizes) + 1):
        pos = np.nonzero(kind == k)[0]
        if pos.size == 0:
            continue
        if k == 0:  # base pairs of the objects' own ids (the heavy ids' pairs generated and dropped)
            (lb, lo), (rb, ro) = base(n_obj, first_obj)
            sides = []
            for b, o in ((lb, lo), (rb, ro)):
                end = np.append(o[1:], np.uint64(b.nbytes))
                sides.append((b, o[pos], end[pos]))
        else:  # heavy object g of size m: pair index (g // step) // len(sizes) of the size-m generator
            m = sizes[k - 1]
            sides = heavy_gen(int(pos.size), int(ids[pos[0]] // step // len(sizes)), m,
                              {"member_universe": m, "ancestor_adds": m, "min_div_ops": max(4, m // 8),
                               "max_div_ops": max(8, m // 4)})
        parts.append((pos, sides))
    out = []
    for side in (0, 1):
        # gather every object's record (16-B units) into object order
        srcs, starts, counts, order = [], [], [], []
        base_units = 0
        for pos, sides in parts:
            b, o = sides[side][0], sides[side][1]
            end = sides[side][2] if len(sides[side]) == 3 else np.append(o[1:], np.uint64(b.nbytes))
            u = b.view(np.complex128) if b.nbytes % 16 == 0 else np.frombuffer(b.tobytes() + bytes(16 - b.nbytes % 16), np.complex128)
            sz = end.astype(np.int64) - o.astype(np.int64)
            srcs.append(u)
            starts.append(o.astype(np.int64) // 16 + base_units)
            counts.append(sz // 16)
            order.append(pos)
            base_units += u.size
        src = np.concatenate(srcs)
        pos_all = np.concatenate(order)
        st = np.empty(n_obj, np.int64)
        ct = np.empty(n_obj, np.int64)
        st[pos_all] = np.concatenate(starts)
        ct[pos_all] = np.concatenate(counts)
        off_units = np.concatenate(([0], np.cumsum(ct)[:-1]))
        idx = np.repeat(st - off_units, ct) + np.arange(int(ct.sum()), dtype=np.int64)
        out.append((src[idx].view(np.uint8).copy(), (off_units * 16).astype(np.uint64)))
    return out[0], out[1]


def _copy_sides(g, n_sides, n_obj):
    sides = []
    for s in range(n_sides):
        bp, op, nb = C.c_void_p(), C.c_void_p(), C.c_size_t()
        check(lib.crdt_orswot_gen_side(g, s, C.byref(bp), C.byref(op), C.byref(nb)), "gen_side")
        base = np.ctypeslib.as_array((C.c_uint8 * max(1, nb.value)).from_address(bp.value)).copy() \
            if nb.value else np.zeros(16, np.uint8)
        off = np.ctypeslib.as_array((C.c_uint64 * max(1, n_obj)).from_address(op.value)).copy()[:n_obj] \
            if n_obj else np.zeros(0, np.uint64)
        sides.append((base, off))
    return sides


def generate_replicas(n_obj, n_replicas=8, first_obj=0, seed=CONFIG5_SEED, params=None, sparse=True, threads=8,
                      keep=None):
    """Replica sets for anti-entropy (config 5, include/crdts_hip.h): a list of
    n_replicas (base, off) batches; replica r of object i is record i of batch r.
    keep=(first, count): only replicas [first, first + count) are returned
    (crdt_orswot_generate_replicas_subset; the same bytes)."""
    d = dict(CONFIG5)
    d.update(params or {})
    P = RepParams(**{k: int(v) for k, v in d.items()})
    g = C.c_void_p()
    fl = SPARSE_CLOCK if sparse else 0
    if keep is None:
        check(lib.crdt_orswot_generate_replicas(seed, first_obj, n_obj, C.byref(P), n_replicas, fl, threads,
                                                C.byref(g)), "generate_replicas")
        count = n_replicas
    else:
        count = int(keep[1])
        check(lib.crdt_orswot_generate_replicas_subset(seed, first_obj, n_obj, C.byref(P), n_replicas, int(keep[0]),
                                                       count, fl, threads, C.byref(g)), "generate_replicas_subset")
    try:
        return _copy_sides(g, count, n_obj)
    finally:
        lib.crdt_orswot_gen_free(g)


def generate_clocks_csr(n_obj, seed, universe=1024, slots=56, p_present=6 / 7, overlap=0.75, bits=40):
    """A pair of sparse clock batches (host numpy CSR: off u64, len u32, act
    u32, ctr u64) over an actor universe of `universe` ids: each clock draws
    from `slots` evenly spaced actor bands (one actor per band), each present
    with p_present (~48 of 56 by default); the other side picks the same actor
    in a band with probability `overlap` (replicas of one clock share most
    actors), counters U[1, 2^bits)."""
    rng = np.random.default_rng(seed)
    band = universe // slots
    js = rng.integers(0, band, (n_obj, slots), dtype=np.uint32)
    jo = np.where(rng.random((n_obj, slots)) < overlap, js, rng.integers(0, band, (n_obj, slots), dtype=np.uint32))
    base = (np.arange(slots, dtype=np.uint32) * band)[None, :]
    out = []
    for j in (js, jo):
        present = rng.random((n_obj, slots)) < p_present
        act = (base + j)[present].astype(np.uint32)
        ctr = rng.integers(1, 1 << bits, act.size, dtype=np.uint64)
        ln = present.sum(1).astype(np.uint32)
        off = np.zeros(n_obj, np.uint64)
        if n_obj:
            off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
        out.append((off, ln, act, ctr))
    return out[0], out[1]


def generate_dense(n_obj, n_actors, seed, first_obj=0, bits=40, pct_zero=25, threads=8):
    rows = np.empty((n_obj, n_actors), dtype=np.uint64)
    check(lib.crdt_dense_generate(seed, first_obj, n_obj, n_actors, bits, pct_zero, threads,
                                  C.c_void_p(rows.ctypes.data)), "dense_generate")
    return rows


# -------------------------------------------------------------- op path
class HostOrswot:
    """Host Orswot built through the reference's op path (src/orswot.rs:61-85)."""

    def __init__(self, handle=None):
        self.h = C.c_void_p(handle) if handle is not None else C.c_void_p(lib.crdt_host_orswot_new())

    def __del__(self):
        if getattr(self, "h", None) is not None and lib is not None:
            lib.crdt_host_orswot_free(self.h)
            self.h = None

    def clone(self):
        return HostOrswot(lib.crdt_host_orswot_clone(self.h))

    def apply_add(self, actor, counter, member):
        check(lib.crdt_host_orswot_apply_add(self.h, actor, counter, member), "apply_add")

    def apply_rm(self, member, clock_pairs):
        n = len(clock_pairs)
        a = (C.c_uint32 * max(1, n))(*[int(x) for x, _ in clock_pairs])
        c = (C.c_uint64 * max(1, n))(*[int(y) for _, y in clock_pairs])
        check(lib.crdt_host_orswot_apply_rm(self.h, member, a, c, n), "apply_rm")

    def encode(self, n_actors, flags=0):
        cap = 1 << 14
        while True:
            buf = (C.c_uint8 * cap)()
            n = lib.crdt_host_orswot_encode_ex(self.h, n_actors, flags, buf, cap)
            if n == CRDT_ECAPACITY:
                cap *= 4
                continue
            check(n if n < 0 else 0, "encode")
            return bytes(buf[:n])

    @staticmethod
    def decode(rec: bytes):
        arr = (C.c_uint8 * len(rec)).from_buffer_copy(rec)
        h = lib.crdt_host_orswot_decode(arr, len(rec))
        if not h:
            raise CrdtError(CRDT_ENONCANON, "decode")
        return HostOrswot(h)


def build_record():
    """The loaded library's sha256 and, if present, the build record written
    by __graft_entry__.build() (rust-crdt_amd/lib/build_info.json): whether
    the library in use is the one that build produced."""
    import hashlib
    import json

    with open(LIB_PATH, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    rec = {"loaded": os.path.relpath(LIB_PATH, os.path.dirname(os.path.dirname(LIB_PATH))), "sha256": sha}
    info = os.path.join(os.path.dirname(LIB_PATH), "build_info.json")
    try:
        with open(info) as f:
            b = json.load(f)
        rec.update(built_sha256_matches=b.get("sha256") == sha, built_from=b.get("git_head"),
                   built_dirty=b.get("git_dirty"), built_at=b.get("built_at"), built_on=b.get("host"))
    except (OSError, ValueError):
        rec["build_info"] = None
    return rec


_default_engine = None


def default_engine():
    global _default_engine
    if _default_engine is None:
        _default_engine = Engine(0)
    return _default_engine


class Orswot:
    """Reference-shaped Orswot (src/orswot.rs:26-30) whose `merge` runs on the GPU.

    `n_actors` is the dense top-clock width used when the state crosses the
    C ABI (actors must be interned to ids < n_actors); with sparse=True the
    top clock crosses as CSR and n_actors is only the actor-id universe.
    """

    def __init__(self, n_actors=16, host=None, sparse=False):
        self.n_actors = n_actors
        self.sparse = bool(sparse)
        self.host = host or HostOrswot()

    @property
    def flags(self):
        return SPARSE_CLOCK if self.sparse else 0

    def clone(self):
        return Orswot(self.n_actors, self.host.clone(), self.sparse)

    def apply_add(self, actor, counter, member):  # CmRDT::apply Op::Add
        self.host.apply_add(actor, counter, member)

    def apply_rm(self, member, clock_pairs):  # CmRDT::apply Op::Rm
        self.host.apply_rm(member, clock_pairs)

    def merge(self, other: "Orswot", engine=None):  # CvRDT::merge
        merge_batch([self], [other], engine)

    def state(self):
        return decode_record(self.host.encode(self.n_actors, self.flags))

    def clock(self):
        return sorted(self.state()["clock"].items())

    def entry(self, member):
        e = self.state()["entries"].get(member)
        return None if e is None else list(e)

    def value(self):
        return sorted(self.state()["entries"])

    def deferred_len(self):
        return len(self.state()["deferred"])

    def record(self):
        return self.host.encode(self.n_actors, self.flags)


def merge_batch(selfs, others, engine=None):
    """`merge_batch(&mut [T], &[T])`: selfs[i].merge(&others[i]) for every i, one kernel launch."""
    if len(selfs) != len(others):
        raise CrdtError(-1, "merge_batch length mismatch")
    if not selfs:
        return
    eng = engine or default_engine()
    kinds = {type(x) for x in selfs} | {type(x) for x in others}
    if kinds == {Orswot}:
        n_actors = max(x.n_actors for x in list(selfs) + list(others))
        fl = SPARSE_CLOCK if any(x.sparse for x in list(selfs) + list(others)) else 0
        L = OrswotBatch.from_records([x.host.encode(n_actors, fl) for x in selfs], n_actors, eng.device, fl)
        R = OrswotBatch.from_records([x.host.encode(n_actors, fl) for x in others], n_actors, eng.device, fl)
        out = eng.orswot_merge(L, R)
        for x, rec in zip(selfs, out.records()):
            x.host = HostOrswot.decode(rec)
        return
    if kinds <= {VClock, GCounter, PNCounter} and len(kinds) == 1:
        kind = {VClock: "vclock", GCounter: "gcounter", PNCounter: "pncounter"}[kinds.pop()]
        n_actors = max(x.n_actors for x in list(selfs) + list(others))
        torch = _torch()
        a = torch.from_numpy(np.stack([x.row(n_actors) for x in selfs]).view(np.int64)).to(f"cuda:{eng.device}")
        b = torch.from_numpy(np.stack([x.row(n_actors) for x in others]).view(np.int64)).to(f"cuda:{eng.device}")
        eng.dense_merge(a, b, n_actors, kind)
        rows = a.cpu().numpy().view(np.uint64)
        for x, r in zip(selfs, rows):
            x.set_row(r, n_actors)
        return
    raise CrdtError(-1, f"merge_batch: unsupported element types {kinds}")


class VClock:
    """Reference-shaped VClock (src/vclock.rs:54-57) over interned actor ids."""

    def __init__(self, dots=None, n_actors=16):
        self.n_actors = n_actors
        self.dots = {}
        for a, c in (dots or []):
            self.witness(a, c)

    def get(self, a):
        return self.dots.get(a, 0)

    def witness(self, a, c):  # src/vclock.rs:159-163
        if not (self.get(a) >= c):
            self.dots[a] = int(c)

    def merge(self, other, engine=None):
        merge_batch([self], [other], engine)

    def row(self, n):
        r = np.zeros(n, dtype=np.uint64)
        for a, c in self.dots.items():
            r[a] = c
        return r

    def set_row(self, r, n):
        self.dots = {a: int(r[a]) for a in range(n) if r[a]}


class GCounter(VClock):
    """src/gcounter.rs:26-28 — one VClock; value() = sum (:76-78)."""

    def inc(self, actor):
        return (actor, self.get(actor) + 1)

    def apply(self, dot):
        self.witness(*dot)

    def value(self):
        return sum(self.dots.values()) & 0xFFFFFFFFFFFFFFFF


class PNCounter:
    """src/pncounter.rs:33-36 — P and N GCounters, merged together as one [P|N] row."""

    def __init__(self, n_actors=16):
        self.n_actors = n_actors
        self.p = GCounter(n_actors=n_actors)
        self.n = GCounter(n_actors=n_actors)

    def inc(self, actor):
        return (self.p.inc(actor), True)

    def dec(self, actor):
        return (self.n.inc(actor), False)

    def apply(self, op):
        dot, pos = op
        (self.p if pos else self.n).apply(dot)

    def merge(self, other, engine=None):
        merge_batch([self], [other], engine)

    def value(self):
        def i64(x):
            x &= 0xFFFFFFFFFFFFFFFF
            return x - (1 << 64) if x >= (1 << 63) else x

        return i64(i64(self.p.value()) - i64(self.n.value()))

    def row(self, n):
        return np.concatenate([self.p.row(n), self.n.row(n)])

    def set_row(self, r, n):
        self.p.set_row(r[:n], n)
        self.n.set_row(r[n:], n)
