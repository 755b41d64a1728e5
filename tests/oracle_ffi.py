"""ctypes binding of the CPU oracle (oracle/ref_cpu.cpp) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "liboracle.so")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ORACLE_DIR, "ref_cpu.cpp")
    if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
        build()
    L = C.CDLL(ORACLE_SO)
    P, U8P, U64P, U32P = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)
    L.orc_record_bytes.restype = C.c_size_t
    L.orc_record_bytes.argtypes = [C.c_uint32] * 6
    L.orc_bincode_to_record.restype = C.c_long
    L.orc_bincode_to_record.argtypes = [P, C.c_size_t, C.c_int, C.c_int, C.c_uint32, C.c_uint32, P, C.c_size_t]
    L.orc_bincode_ingest_bench.restype = C.c_double
    L.orc_bincode_ingest_bench.argtypes = [P, P, P, C.c_size_t, C.c_int, C.c_int, C.c_uint32, C.c_uint32, C.c_int,
                                           C.POINTER(C.c_int64)]
    L.orc_mvreg_merge_batch.restype = C.c_int
    L.orc_mvreg_merge_batch.argtypes = [P, P, P, C.c_uint32, P, P, P, C.c_uint32, P, P, P, C.c_uint32, C.c_size_t,
                                        C.c_uint32]
    L.orc_vclock_partial_cmp_rows.restype = None
    L.orc_vclock_partial_cmp_rows.argtypes = [P, P, C.c_size_t, C.c_uint32, P]
    L.orc_map_mvreg_merge_batch.restype = C.c_int
    L.orc_map_mvreg_merge_batch.argtypes = [P, P, P, C.c_size_t, C.c_uint32]
    L.orc_map_mvreg_generate.restype = C.c_int
    L.orc_map_mvreg_generate.argtypes = [C.c_uint64, C.c_size_t, C.c_uint32, C.c_uint32, C.c_int, P, P]
    L.orc_orswot_apply_bench.restype = C.c_double
    L.orc_orswot_apply_bench.argtypes = [P, P, C.c_size_t, C.c_size_t] + [P] * 8 + [C.c_int]
    L.orc_bincode_egest_bench.restype = C.c_double
    L.orc_bincode_egest_bench.argtypes = [P, P, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int]
    L.orc_orswot_merge_batch.restype = C.c_int
    L.orc_orswot_merge_batch.argtypes = [P, P, C.c_size_t, P, P, C.c_size_t, C.c_size_t, C.c_uint32,
                                         P, P, C.c_size_t, C.c_int, C.POINTER(C.c_int64)]
    L.orc_orswot_merge_batch_ex.restype = C.c_int
    L.orc_orswot_merge_batch_ex.argtypes = [P, P, C.c_size_t, P, P, C.c_size_t, C.c_size_t, C.c_uint32,
                                            C.c_uint32, P, P, C.c_size_t, C.c_int, C.POINTER(C.c_int64)]
    L.orc_obj_encode_ex.restype = C.c_long
    L.orc_obj_encode_ex.argtypes = [P, C.c_uint32, C.c_uint32, P, C.c_size_t]
    L.orc_orswot_bench.restype = C.c_double
    L.orc_orswot_bench.argtypes = [P, P, C.c_size_t, P, P, C.c_size_t, C.c_size_t, C.c_int]
    L.orc_dense_merge.restype = C.c_int
    L.orc_dense_merge.argtypes = [P, P, C.c_size_t, C.c_uint32, C.c_int]
    L.orc_pncounter_merge.restype = C.c_int
    L.orc_pncounter_merge.argtypes = [P, P, C.c_size_t, C.c_uint32, C.c_int]
    L.orc_dense_bench.restype = C.c_double
    L.orc_dense_bench.argtypes = [P, P, C.c_size_t, C.c_uint32, C.c_int]
    L.orc_vclock_csr_merge.restype = C.c_int
    L.orc_vclock_csr_merge.argtypes = [P] * 8 + [C.c_size_t, P, P, P, C.c_int, C.POINTER(C.c_int64)]
    L.orc_vclock_csr_bench.restype = C.c_double
    L.orc_vclock_csr_bench.argtypes = [P] * 8 + [C.c_size_t, C.c_int]
    L.orc_orswot_truncate_bench.restype = C.c_double
    L.orc_orswot_truncate_bench.argtypes = [P, P, C.c_size_t, C.c_size_t, P, P, P, P, C.c_int]
    L.orc_orswot_truncate_batch.restype = C.c_int
    L.orc_orswot_truncate_batch.argtypes = [P, P, C.c_size_t, C.c_size_t, P, P, P, P, C.c_uint32, C.c_uint32, P, P,
                                            C.c_size_t, C.c_int, C.POINTER(C.c_int64)]
    L.orc_obj_new.restype = P
    L.orc_obj_clone.restype = P
    L.orc_obj_clone.argtypes = [P]
    L.orc_obj_free.argtypes = [P]
    L.orc_obj_apply_add.argtypes = [P, C.c_uint32, C.c_uint64, C.c_uint64]
    L.orc_obj_apply_rm.argtypes = [P, C.c_uint64, U32P, U64P, C.c_uint32]
    L.orc_obj_merge.argtypes = [P, P]
    L.orc_obj_encode.restype = C.c_long
    L.orc_obj_encode.argtypes = [P, C.c_uint32, P, C.c_size_t]
    L.orc_obj_decode.restype = P
    L.orc_obj_decode.argtypes = [P, C.c_size_t]
    L.orc_obj_deferred_len.restype = C.c_long
    L.orc_obj_deferred_len.argtypes = [P]
    L.orc_obj_value.restype = C.c_long
    L.orc_obj_value.argtypes = [P, U64P, C.c_size_t]
    L.orc_obj_entry.restype = C.c_long
    L.orc_obj_entry.argtypes = [P, C.c_uint64, U32P, U64P, C.c_size_t]
    L.orc_obj_clock.restype = C.c_long
    L.orc_obj_clock.argtypes = [P, U32P, U64P, C.c_size_t]
    L.orc_vclock_binop.restype = C.c_long
    L.orc_vclock_binop.argtypes = [C.c_int, U32P, U64P, C.c_uint32, U32P, U64P, C.c_uint32, U32P, U64P,
                                   C.c_size_t]
    L.orc_vclock_partial_cmp.restype = C.c_int
    L.orc_vclock_partial_cmp.argtypes = [U32P, U64P, C.c_uint32, U32P, U64P, C.c_uint32]
    L.orc_map_orswot_merge_batch.restype = C.c_int
    L.orc_map_orswot_merge_batch.argtypes = [P, P, P, C.c_size_t, C.c_uint32]
    L.orc_map_map_merge_batch.restype = C.c_int
    L.orc_map_map_merge_batch.argtypes = [P, P, P, C.c_size_t, C.c_uint32]
    L.orc_map_map_bench.restype = C.c_double
    L.orc_map_map_bench.argtypes = [P, P, C.c_size_t, C.c_uint32, C.c_int]
    L.orc_map_orswot_order_outcomes.restype = C.c_int
    L.orc_map_orswot_order_outcomes.argtypes = [P, P, C.c_size_t, C.c_uint32, C.c_int, P]
    L.orc_map_orswot_generate.restype = C.c_int
    L.orc_map_orswot_generate.argtypes = [C.c_uint64, C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                          C.c_int, P, P]
    for pre in ("mapor", "mapmv"):
        getattr(L, f"orc_{pre}_new").restype = P
        getattr(L, f"orc_{pre}_clone").restype = P
        getattr(L, f"orc_{pre}_clone").argtypes = [P]
        getattr(L, f"orc_{pre}_free").argtypes = [P]
        getattr(L, f"orc_{pre}_merge").argtypes = [P, P]
        getattr(L, f"orc_{pre}_apply_rm").argtypes = [P, C.c_uint64, U32P, U64P, C.c_uint32]
        getattr(L, f"orc_{pre}_to_slab").restype = C.c_int
        getattr(L, f"orc_{pre}_to_slab").argtypes = [P, P, C.c_size_t, C.c_uint32]
    L.orc_mapor_apply_up.argtypes = [P, C.c_uint32, C.c_uint64, C.c_uint64, C.c_int, C.c_uint64, U32P, U64P,
                                     C.c_uint32]
    L.orc_mapmv_apply_up.argtypes = [P, C.c_uint32, C.c_uint64, C.c_uint64, U32P, U64P, C.c_uint32, C.c_uint64]
    L.orc_mapor_from_slab.restype = P
    L.orc_mapor_from_slab.argtypes = [P, C.c_size_t, C.c_uint32]
    _lib = L
    return L


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def _clock_arrays(pairs):
    a = (C.c_uint32 * max(1, len(pairs)))(*[int(x) for x, _ in pairs])
    c = (C.c_uint64 * max(1, len(pairs)))(*[int(y) for _, y in pairs])
    return a, c, len(pairs)


def _dump(fn, *args):
    cap = 4096
    a = (C.c_uint32 * cap)()
    c = (C.c_uint64 * cap)()
    n = fn(*args, a, c, cap)
    if n < 0:
        return None
    return [(int(a[i]), int(c[i])) for i in range(n)]


# ------------------------------------------------------------- VClock KATs
def vclock_binop(op, a, b):
    code = {"merge": 0, "subtract": 1, "intersection": 2}[op]
    aa, ac, an = _clock_arrays(a)
    ba, bc, bn = _clock_arrays(b)
    return _dump(lambda *r: lib().orc_vclock_binop(code, aa, ac, an, ba, bc, bn, *r))


def vclock_partial_cmp(a, b):
    aa, ac, an = _clock_arrays(a)
    ba, bc, bn = _clock_arrays(b)
    r = lib().orc_vclock_partial_cmp(aa, ac, an, ba, bc, bn)
    return {0: "Equal", 1: "Greater", -1: "Less", 2: "None"}[r]


# ------------------------------------------------------------- Orswot objects
class OracleOrswot:
    """Handle to an oracle Orswot (reference-like std::map/unordered_map)."""

    def __init__(self, handle=None):
        self.h = handle if handle is not None else lib().orc_obj_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_obj_free(self.h)
            self.h = None

    def clone(self):
        return OracleOrswot(lib().orc_obj_clone(self.h))

    def apply_add(self, actor, counter, member):
        lib().orc_obj_apply_add(self.h, actor, counter, member)

    def apply_rm(self, member, clock_pairs):
        a, c, n = _clock_arrays(clock_pairs)
        lib().orc_obj_apply_rm(self.h, member, a, c, n)

    def merge(self, other):
        lib().orc_obj_merge(self.h, other.h)

    def clock(self):
        return _dump(lambda *r: lib().orc_obj_clock(self.h, *r))

    def entry(self, member):
        return _dump(lambda *r: lib().orc_obj_entry(self.h, member, *r))

    def value(self):
        cap = 1 << 16
        buf = (C.c_uint64 * cap)()
        n = lib().orc_obj_value(self.h, buf, cap)
        return [int(buf[i]) for i in range(n)]

    def deferred_len(self):
        return int(lib().orc_obj_deferred_len(self.h))

    def encode(self, n_actors, flags=0):
        cap = 1 << 16
        while True:
            buf = np.zeros(cap, dtype=np.uint8)
            n = lib().orc_obj_encode_ex(self.h, n_actors, flags, _ptr(buf), cap)
            if n == -4:
                cap *= 4
                continue
            if n < 0:
                raise ValueError(f"encode failed: {n}")
            return buf[:n].tobytes()

    @staticmethod
    def decode(rec: bytes):
        arr = np.frombuffer(rec, dtype=np.uint8).copy()
        h = lib().orc_obj_decode(_ptr(arr), len(rec))
        if not h:
            raise ValueError("decode failed")
        return OracleOrswot(h)


# ------------------------------------------------------------- batches
def orswot_merge_batch(lbase, loff, rbase, roff, n_actors, threads=8, flags=0):
    """Merge record batches (numpy u8 bases, u64 offsets). Returns (base, off).
    flags=1: CSR top clocks (inputs and output)."""
    n = len(loff)
    cap = int(lbase.nbytes + rbase.nbytes) + 64
    obase = np.zeros(cap, dtype=np.uint8)
    ooff = np.zeros(n, dtype=np.uint64)
    bad = C.c_int64(-1)
    rc = lib().orc_orswot_merge_batch_ex(_ptr(lbase), _ptr(loff), lbase.nbytes, _ptr(rbase), _ptr(roff),
                                         rbase.nbytes, n, n_actors, flags, _ptr(obase), _ptr(ooff), cap, threads,
                                         C.byref(bad))
    if rc != 0:
        raise ValueError(f"oracle merge failed rc={rc} at object {bad.value}")
    return obase, ooff


def bincode_to_record(blob, wa, wm, n_actors, flags=0):
    """Blob -> canonical record through the C++ restatement (oracle/ref_cpu.cpp)."""
    b = np.frombuffer(bytes(blob) or b"\0", dtype=np.uint8)
    out = np.zeros(1 << 16, dtype=np.uint8)
    n = lib().orc_bincode_to_record(_ptr(b), len(blob), wa, wm, n_actors, flags, _ptr(out), out.nbytes)
    if n < 0:
        raise ValueError(f"oracle bincode decode failed rc={n}")
    return out[:n].tobytes()


def bincode_ingest_bench(blobs, off, lens, wa, wm, n_actors, flags, threads):
    bad = C.c_int64(0)
    b = np.ascontiguousarray(blobs, dtype=np.uint8)
    o = np.ascontiguousarray(off, dtype=np.uint64)
    n_ = np.ascontiguousarray(lens, dtype=np.uint64)
    secs = lib().orc_bincode_ingest_bench(_ptr(b), _ptr(o), _ptr(n_), len(o), wa, wm, n_actors, flags, threads,
                                          C.byref(bad))
    if bad.value:
        raise ValueError(f"oracle bincode ingest: {bad.value} blobs failed")
    return secs


def bincode_egest_bench(rbase, roff, wa, wm, threads):
    return lib().orc_bincode_egest_bench(_ptr(rbase), _ptr(roff), rbase.nbytes, len(roff), wa, wm, threads)


def mvreg_merge(sn, sclk, sval, on, oclk, oval, n_actors, out_cap):
    """Batch MVReg::merge through the oracle: slabs as numpy (n,), (n, cap, A), (n, cap)."""
    sn, on = (np.ascontiguousarray(x, dtype=np.uint32) for x in (sn, on))
    sclk, sval, oclk, oval = (np.ascontiguousarray(x, dtype=np.uint64) for x in (sclk, sval, oclk, oval))
    n = len(sn)
    outn = np.zeros(n, np.uint32)
    outc = np.zeros((n, out_cap, n_actors), np.uint64)
    outv = np.zeros((n, out_cap), np.uint64)
    rc = lib().orc_mvreg_merge_batch(_ptr(sn), _ptr(sclk), _ptr(sval), sval.shape[1], _ptr(on), _ptr(oclk),
                                     _ptr(oval), oval.shape[1], _ptr(outn), _ptr(outc), _ptr(outv), out_cap, n,
                                     n_actors)
    if rc:
        raise ValueError(f"oracle mvreg merge rc={rc}")
    return outn, outc, outv


def partial_cmp_rows(a, b, n_actors):
    a, b = (np.ascontiguousarray(x, dtype=np.uint64) for x in (a, b))
    out = np.zeros(a.size // n_actors, np.int8)
    lib().orc_vclock_partial_cmp_rows(_ptr(a), _ptr(b), len(out), n_actors, _ptr(out))
    return out


def map_generate(seed, n, A, keys, ops, caps):
    """Replica pairs of Map<u64, MVReg<u64>> by op simulation -> (left, right) host MapSlabs."""
    import crdts_hip

    L = crdts_hip.MapSlab.alloc(n, A, *caps)
    R = crdts_hip.MapSlab.alloc(n, A, *caps)
    l, r = L.cstruct(), R.cstruct()
    rc = lib().orc_map_mvreg_generate(seed, n, A, keys, ops, C.byref(l), C.byref(r))
    if rc:
        raise ValueError(f"map generate rc={rc} (capacity)")
    return L, R


def map_merge(S, O, A):
    """Oracle Map::merge of host MapSlabs -> output MapSlab (capacities summed)."""
    import crdts_hip

    n = S.a["n_keys"].shape[0]
    R = crdts_hip.MapSlab.alloc(n, A, S.kcap + O.kcap, S.mcap + O.mcap, S.dcap + O.dcap, S.scap + O.scap)
    s, o, r = S.cstruct(), O.cstruct(), R.cstruct()
    rc = lib().orc_map_mvreg_merge_batch(C.byref(s), C.byref(o), C.byref(r), n, A)
    if rc:
        raise ValueError(f"oracle map merge rc={rc}")
    return R


def orswot_apply_bench(rbase, roff, ops_np, threads):
    """ops_np: (obj_end, kind, member, actor, counter, clk_end, clk_act, clk_ctr) numpy arrays."""
    arrs = [np.ascontiguousarray(a) for a in ops_np]
    return lib().orc_orswot_apply_bench(_ptr(rbase), _ptr(roff), rbase.nbytes, len(roff), *[_ptr(a) for a in arrs],
                                        threads)


def orswot_bench(lbase, loff, rbase, roff, threads):
    return lib().orc_orswot_bench(_ptr(lbase), _ptr(loff), lbase.nbytes, _ptr(rbase), _ptr(roff),
                                  rbase.nbytes, len(loff), threads)


def dense_merge(self_rows, other_rows, n_actors, threads=8):
    out = np.ascontiguousarray(self_rows, dtype=np.uint64).copy()
    o = np.ascontiguousarray(other_rows, dtype=np.uint64)
    n = out.size // n_actors
    lib().orc_dense_merge(_ptr(out), _ptr(o), n, n_actors, threads)
    return out


def vclock_csr_merge(s, o, threads=8):
    """s, o: (off u64, len u32, act u32, ctr u64) numpy CSR batches of the same
    n_obj. Returns (out_off, out_len, out_act, out_ctr), entries at s.off + o.off."""
    so, sl, sa, sc = [np.ascontiguousarray(x) for x in s]
    oo, ol, oa, oc = [np.ascontiguousarray(x) for x in o]
    n = len(so)
    cap = max(1, len(sa) + len(oa))
    out_act = np.zeros(cap, np.uint32)
    out_ctr = np.zeros(cap, np.uint64)
    out_len = np.zeros(max(1, n), np.uint32)
    bad = C.c_int64(-1)
    rc = lib().orc_vclock_csr_merge(_ptr(so), _ptr(sl), _ptr(sa), _ptr(sc), _ptr(oo), _ptr(ol), _ptr(oa), _ptr(oc), n,
                                    _ptr(out_act), _ptr(out_ctr), _ptr(out_len), threads, C.byref(bad))
    if rc != 0:
        raise ValueError(f"oracle csr merge: non-canonical run at object {bad.value}")
    return (so + oo).astype(np.uint64), out_len[:n], out_act, out_ctr


def orswot_truncate_batch(lbase, loff, clocks, n_actors, flags=0, threads=8):
    """Causal::truncate of record i by clock i (clocks: numpy CSR (off, len,
    act, ctr)); returns the packed (base, off) of the truncated records."""
    lbase = np.ascontiguousarray(lbase, dtype=np.uint8)
    loff = np.ascontiguousarray(loff, dtype=np.uint64)
    co, cl, ca, cc = [np.ascontiguousarray(x) for x in clocks]
    n = len(loff)
    cap = lbase.nbytes + 16
    obase = np.zeros(cap, np.uint8)
    ooff = np.zeros(max(1, n), np.uint64)
    bad = C.c_int64(-1)
    rc = lib().orc_orswot_truncate_batch(_ptr(lbase), _ptr(loff), lbase.nbytes, n, _ptr(co), _ptr(cl), _ptr(ca),
                                         _ptr(cc), n_actors, flags, _ptr(obase), _ptr(ooff), cap, threads,
                                         C.byref(bad))
    if rc != 0:
        raise ValueError(f"oracle truncate failed rc={rc} at object {bad.value}")
    return obase, ooff[:n]


def orswot_truncate_bench(lbase, loff, clocks, threads):
    """Seconds of Orswot::truncate over the batch (decode untimed)."""
    lbase = np.ascontiguousarray(lbase, dtype=np.uint8)
    loff = np.ascontiguousarray(loff, dtype=np.uint64)
    co, cl, ca, cc = [np.ascontiguousarray(x) for x in clocks]
    return lib().orc_orswot_truncate_bench(_ptr(lbase), _ptr(loff), lbase.nbytes, len(loff), _ptr(co), _ptr(cl),
                                           _ptr(ca), _ptr(cc), threads)


def vclock_csr_bench(s, o, threads):
    so, sl, sa, sc = [np.ascontiguousarray(x) for x in s]
    oo, ol, oa, oc = [np.ascontiguousarray(x) for x in o]
    return lib().orc_vclock_csr_bench(_ptr(so), _ptr(sl), _ptr(sa), _ptr(sc), _ptr(oo), _ptr(ol), _ptr(oa), _ptr(oc),
                                      len(so), threads)


def pncounter_merge(self_rows, other_rows, n_actors, threads=8):
    out = np.ascontiguousarray(self_rows, dtype=np.uint64).copy()
    o = np.ascontiguousarray(other_rows, dtype=np.uint64)
    n = out.size // (2 * n_actors)
    lib().orc_pncounter_merge(_ptr(out), _ptr(o), n, n_actors, threads)
    return out


def dense_bench(self_rows, other_rows, n_actors, threads):
    n = self_rows.size // n_actors
    return lib().orc_dense_bench(_ptr(self_rows), _ptr(other_rows), n, n_actors, threads)


def record_bytes(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem):
    return int(lib().orc_record_bytes(n_clk, n_mem, n_dot, n_def, n_def_dot, n_def_mem))


# ------------------------------------------------------------- Map<u64, Orswot>
MAP_ORSWOT_CAPS = dict(kcap=8, mcap=8, vdcap=4, vscap=4, dcap=8, scap=8)


def map_orswot_generate(seed, n, A, keys, members, ops, pct_future, caps=None):
    """Replica pairs of Map<u64, Orswot<u64>> by op simulation -> (left, right) host slabs."""
    import crdts_hip

    caps = caps or MAP_ORSWOT_CAPS
    L = crdts_hip.MapOrswotSlab.alloc(n, A, **caps)
    R = crdts_hip.MapOrswotSlab.alloc(n, A, **caps)
    l, r = L.cstruct(), R.cstruct()
    rc = lib().orc_map_orswot_generate(seed, n, A, keys, members, ops, pct_future, C.byref(l), C.byref(r))
    if rc:
        raise ValueError(f"map-orswot generate rc={rc} (capacity)")
    return L, R


def map_orswot_merge(S, O, A, out_caps=None):
    """Oracle Map::merge (Orswot values, CLOCK ORDER apply_deferred) of host slabs."""
    import crdts_hip

    caps = out_caps or {k: S.caps[k] + O.caps[k] for k in S.caps}
    R = crdts_hip.MapOrswotSlab.alloc(S.n, A, **caps)
    s, o, r = S.cstruct(), O.cstruct(), R.cstruct()
    rc = lib().orc_map_orswot_merge_batch(C.byref(s), C.byref(o), C.byref(r), S.n, A)
    if rc:
        raise ValueError(f"oracle map-orswot merge rc={rc}")
    return R


def map_map_merge(S, O, A):
    """Oracle (C++) Map<u64, Map<u64, MVReg>>::merge of host MapMapSlabs ->
    output MapMapSlab (outer and inner capacities summed)."""
    import crdts_hip

    R = crdts_hip.MapMapSlab.alloc(S.n, A, S.kcap + O.kcap, S.dcap + O.dcap, S.scap + O.scap,
                                   tuple(x + y for x, y in zip(S.inner_caps, O.inner_caps)))
    s, o, r = S.cstruct(), O.cstruct(), R.cstruct()
    rc = lib().orc_map_map_merge_batch(C.byref(s), C.byref(o), C.byref(r), S.n, A)
    if rc:
        raise ValueError(f"oracle nested map merge rc={rc}")
    return R


def map_map_bench(S, O, A, threads):
    """Seconds for the C++ restatement's nested-map merge of the slabs' pairs (decode untimed)."""
    s, o = S.cstruct(), O.cstruct()
    return lib().orc_map_map_bench(C.byref(s), C.byref(o), S.n, A, threads)


def map_orswot_order_outcomes(S, O, A, max_k=6):
    """Per object: distinct Map::merge results over every order of the final
    apply_deferred (-1: more than max_k deferred clocks, not enumerated)."""
    out = np.zeros(S.n, dtype=np.int32)
    s, o = S.cstruct(), O.cstruct()
    lib().orc_map_orswot_order_outcomes(C.byref(s), C.byref(o), S.n, A, max_k, _ptr(out))
    return out


class OracleMap:
    """Handle to an oracle Map<u64, Orswot<u64>> (kind "orswot") or Map<u64, MVReg<u64>> (kind "mvreg")."""

    def __init__(self, kind, handle=None):
        self.kind = kind
        self.pre = "mapor" if kind == "orswot" else "mapmv"
        self.h = handle if handle is not None else getattr(lib(), f"orc_{self.pre}_new")()

    def __del__(self):
        if getattr(self, "h", None):
            getattr(lib(), f"orc_{self.pre}_free")(self.h)
            self.h = None

    def clone(self):
        return OracleMap(self.kind, getattr(lib(), f"orc_{self.pre}_clone")(self.h))

    def apply_up_orswot(self, dot, key, kind, member, rm_pairs=()):
        a, c, n = _clock_arrays(list(rm_pairs))
        lib().orc_mapor_apply_up(self.h, dot[0], dot[1], key, kind, member, a, c, n)

    def apply_up_mvreg(self, dot, key, put_pairs, val):
        a, c, n = _clock_arrays(list(put_pairs))
        lib().orc_mapmv_apply_up(self.h, dot[0], dot[1], key, a, c, n, val)

    def apply_rm(self, key, pairs):
        a, c, n = _clock_arrays(list(pairs))
        getattr(lib(), f"orc_{self.pre}_apply_rm")(self.h, key, a, c, n)

    def merge(self, other):
        getattr(lib(), f"orc_{self.pre}_merge")(self.h, other.h)

    def slab(self, A, caps):
        import crdts_hip

        if self.kind == "orswot":
            S = crdts_hip.MapOrswotSlab.alloc(1, A, **caps)
        else:
            S = crdts_hip.MapSlab.alloc(1, A, caps["kcap"], caps["mcap"], caps["dcap"], caps["scap"])
        st = S.cstruct()
        rc = getattr(lib(), f"orc_{self.pre}_to_slab")(self.h, C.byref(st), 0, A)
        if rc:
            raise ValueError("oracle map to slab: capacity")
        return S
