"""ctypes binding of libcrdts_hip.so (C ABI: include/crdts_hip.h).

The shared library is the product; this module only declares its symbols.
There is no CPU fallback anywhere: if the library is missing, importing the
package raises.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)  # rust-crdt_amd/
LIB_PATH = os.path.join(ROOT, "lib", "libcrdts_hip.so")
# tools/ may select the diagnostic build (make -C rust-crdt_amd diag: kernel
# variants, phase stamps, tuning knobs) with CRDTS_HIP_DIAG=1; never the product.
if os.environ.get("CRDTS_HIP_DIAG") == "1":
    LIB_PATH = os.path.join(ROOT, "lib", "libcrdts_hip_diag.so")
# A/B builds of a compile-time knob (tools/): CRDTS_HIP_AB=<tag> loads
# lib/libcrdts_hip_ab_<tag>.so; never the product.
if os.environ.get("CRDTS_HIP_AB"):
    LIB_PATH = os.path.join(ROOT, "lib", f"libcrdts_hip_ab_{os.environ['CRDTS_HIP_AB']}.so")
DIAG_SYMBOLS = {"crdt_ctx_set_blocks_per_cu", "crdt_ctx_set_variant", "crdt_ctx_debug_read"}

CRDT_OK = 0
CRDT_EINVAL = -1
CRDT_ENONCANON = -2
CRDT_EHIP = -3
CRDT_ECAPACITY = -4
CRDT_ECOMM = -5
CRDT_ENODEV = -6


class CrdtError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = lib.crdt_strerror(code).decode() if lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


class Batch(C.Structure):
    _fields_ = [("base", C.c_void_p), ("off", C.c_void_p), ("n_obj", C.c_size_t), ("bytes", C.c_size_t)]


class GenParams(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("n_actors", "member_universe", "ancestor_adds", "min_div_ops",
                                          "max_div_ops", "pct_add", "pct_future_rm", "pct_deferred_obj",
                                          "pct_shared_actor")]


class RepParams(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("universe", "pool_actors", "own_actors", "member_universe",
                                          "ancestor_adds", "min_div_ops", "max_div_ops", "pct_add",
                                          "pct_future_rm", "pct_deferred_obj")]


SPARSE_CLOCK = 1  # CRDT_ORSWOT_SPARSE_CLOCK

# Every symbol include/crdts_hip.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "crdt_ctx_create", "crdt_ctx_destroy", "crdt_ctx_status", "crdt_strerror", "crdt_abi_version",
    "crdt_vclock_dense_merge", "crdt_gcounter_merge", "crdt_pncounter_merge",
    "crdt_orswot_record_bytes", "crdt_orswot_merge", "crdt_orswot_merge_host", "crdt_orswot_validate",
    "crdt_orswot_compact_scratch_bytes", "crdt_orswot_compact",
    "crdt_orswot_generate", "crdt_orswot_gen_side", "crdt_orswot_gen_free", "crdt_dense_generate",
    "crdt_host_orswot_new", "crdt_host_orswot_clone", "crdt_host_orswot_free",
    "crdt_host_orswot_apply_add", "crdt_host_orswot_apply_rm", "crdt_host_orswot_encode",
    "crdt_host_orswot_decode", "crdt_orswot_record_bytes_ex", "crdt_orswot_merge_ex",
    "crdt_orswot_validate_ex", "crdt_orswot_generate_replicas", "crdt_host_orswot_encode_ex",
    "crdt_orswot_bincode_record_sizes", "crdt_orswot_from_bincode", "crdt_orswot_bincode_sizes",
    "crdt_orswot_to_bincode", "crdt_orswot_apply", "crdt_vclock_partial_cmp", "crdt_mvreg_merge",
    "crdt_map_mvreg_merge", "crdt_map_orswot_merge", "crdt_ctx_set_list_cap", "crdt_orswot_bincode_record_bounds",
    "crdt_comm_unique_id", "crdt_comm_init", "crdt_comm_destroy", "crdt_replica_allreduce_max",
    "crdt_replica_reduce_scatter_max",
    "crdt_orswot_replica_join_bound", "crdt_orswot_replica_join", "crdt_orswot_replica_join_local",
    "crdt_comm_count", "crdt_orswot_replica_join_transport", "crdt_orswot_generate_replicas_subset",
    "crdt_dense_merge_host", "crdt_vclock_csr_merge", "crdt_gcounter_csr_merge", "crdt_pncounter_csr_merge",
    "crdt_orswot_truncate", "crdt_ctx_host_syncs", "crdt_orswot_fold", "crdt_ctx_set_arena_limit",
    "crdt_map_map_merge_scratch_bytes", "crdt_map_map_merge", "crdt_replica_allreduce_max_transport",
    "crdt_replica_reduce_scatter_max_transport",
]

CRDT_COMM_ID_BYTES = 128


def hip_runtime():
    """The HIP runtime library this process already has loaded (torch's), found
    in /proc/self/maps — not a fixed soname, so a ROCm major version change does
    not load a second runtime. Falls back to the unversioned soname."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.split()[-1] if line.strip() else ""
                if os.path.basename(path).startswith("libamdhip64.so"):
                    return C.CDLL(path)
    except OSError:
        pass
    return C.CDLL("libamdhip64.so")


class Ops(C.Structure):
    """crdt_orswot_ops (include/crdts_hip.h)."""
    _fields_ = [("obj_end", C.c_void_p), ("kind", C.c_void_p), ("member", C.c_void_p), ("actor", C.c_void_p),
                ("counter", C.c_void_p), ("clk_end", C.c_void_p), ("clk_act", C.c_void_p),
                ("clk_ctr", C.c_void_p), ("n_ops", C.c_size_t), ("n_clk", C.c_size_t)]


class MapSlabC(C.Structure):
    """crdt_map_mvreg_slab (include/crdts_hip.h)."""
    _fields_ = [(f, C.c_void_p) for f in ("clock", "n_keys", "keys", "eclock", "mv_n", "mv_clock", "mv_val", "n_def",
                                          "dclock", "dset_n", "dset")] + \
               [(f, C.c_uint32) for f in ("kcap", "mcap", "dcap", "scap")]


MAP_MAP_FIELDS = ("clock", "n_keys", "keys", "eclock", "n_def", "dclock", "dset_n", "dset")


class MapMapSlabC(C.Structure):
    """crdt_map_map_slab (include/crdts_hip.h): the outer map and its inner Map<u64, MVReg> slab."""
    _fields_ = [(f, C.c_void_p) for f in MAP_MAP_FIELDS] + [(f, C.c_uint32) for f in ("kcap", "dcap", "scap")] + \
               [("inner", MapSlabC)]


MAP_ORSWOT_FIELDS = ("clock", "n_keys", "keys", "eclock", "vclock", "vn_mem", "vmem", "vmclock", "vn_def", "vdclock",
                     "vdset_n", "vdset", "n_def", "dclock", "dset_n", "dset")
MAP_ORSWOT_CAPS = ("kcap", "mcap", "vdcap", "vscap", "dcap", "scap")


class MapOrswotSlabC(C.Structure):
    """crdt_map_orswot_slab (include/crdts_hip.h)."""
    _fields_ = [(f, C.c_void_p) for f in MAP_ORSWOT_FIELDS] + [(f, C.c_uint32) for f in MAP_ORSWOT_CAPS]


class ClockCsr(C.Structure):
    """crdt_clock_csr (include/crdts_hip.h)."""
    _fields_ = [("off", C.c_void_p), ("len", C.c_void_p), ("act", C.c_void_p), ("ctr", C.c_void_p),
                ("n_obj", C.c_size_t), ("n_entries", C.c_size_t)]


class ClockCsrOut(C.Structure):
    """crdt_clock_csr_out (include/crdts_hip.h)."""
    _fields_ = [("off", C.c_void_p), ("len", C.c_void_p), ("act", C.c_void_p), ("ctr", C.c_void_p),
                ("n_entries", C.c_size_t)]


class Xfer(C.Structure):
    """crdt_xfer (include/crdts_hip.h)."""
    _fields_ = [("peer", C.c_int), ("src", C.c_void_p), ("dst", C.c_void_p), ("bytes", C.c_size_t)]


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_uint64))
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(Xfer), C.c_size_t, C.POINTER(Xfer), C.c_size_t,
                          C.c_void_p)


class TransportC(C.Structure):
    """crdt_transport (include/crdts_hip.h): a caller-provided transport."""
    _fields_ = [("n_ranks", C.c_int), ("rank", C.c_int), ("user", C.c_void_p), ("allgather", ALLGATHER_FN),
                ("exchange", EXCHANGE_FN)]


def _load():
    # One HIP runtime per process: torch ships its own libamdhip64.so.7. Load
    # torch first so this library's libamdhip64.so.7 dependency binds to the
    # already-loaded copy (same SONAME) instead of a second runtime from
    # /opt/rocm, which would fail to open the device next to torch's.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"crdts_hip: native library missing at {LIB_PATH}; build it with "
            "`make -C rust-crdt_amd` or `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    P, I, SZ, U32, U64 = C.c_void_p, C.c_int, C.c_size_t, C.c_uint32, C.c_uint64
    BP = C.POINTER(Batch)
    sig = {
        "crdt_ctx_create": (I, [C.POINTER(P), I]),
        "crdt_ctx_destroy": (I, [P]),
        "crdt_ctx_status": (I, [P, P]),
        "crdt_ctx_set_blocks_per_cu": (I, [P, I]),
        "crdt_ctx_set_list_cap": (I, [P, U32]),
        "crdt_ctx_host_syncs": (U64, [P]),
        "crdt_ctx_set_arena_limit": (I, [P, SZ]),
        "crdt_orswot_fold": (I, [P, BP, U32, U32, U32, P, P, SZ, P]),
        "crdt_ctx_set_variant": (I, [P, I]),
        "crdt_ctx_debug_read": (I, [P, P, SZ, P]),
        "crdt_strerror": (C.c_char_p, [I]),
        "crdt_abi_version": (I, []),
        "crdt_vclock_dense_merge": (I, [P, P, P, SZ, U32, P]),
        "crdt_gcounter_merge": (I, [P, P, P, SZ, U32, P]),
        "crdt_pncounter_merge": (I, [P, P, P, SZ, U32, P]),
        "crdt_orswot_record_bytes": (SZ, [U32] * 6),
        "crdt_orswot_merge": (I, [P, BP, BP, P, P, SZ, U32, P]),
        "crdt_orswot_merge_host": (I, [P, P, P, SZ, P, P, SZ, SZ, U32, P, P, SZ, C.POINTER(SZ)]),
        "crdt_orswot_validate": (I, [P, BP, U32, P]),
        "crdt_orswot_compact_scratch_bytes": (SZ, [SZ]),
        "crdt_orswot_compact": (I, [P, BP, P, P, SZ, P, P]),
        "crdt_orswot_generate": (I, [U64, SZ, SZ, C.POINTER(GenParams), I, C.POINTER(P)]),
        "crdt_orswot_gen_side": (I, [P, I, C.POINTER(P), C.POINTER(P), C.POINTER(SZ)]),
        "crdt_orswot_gen_free": (None, [P]),
        "crdt_dense_generate": (I, [U64, SZ, SZ, U32, U32, U32, I, P]),
        "crdt_host_orswot_new": (P, []),
        "crdt_host_orswot_clone": (P, [P]),
        "crdt_host_orswot_free": (None, [P]),
        "crdt_host_orswot_apply_add": (I, [P, U32, U64, U64]),
        "crdt_host_orswot_apply_rm": (I, [P, U64, P, P, U32]),
        "crdt_host_orswot_encode": (C.c_long, [P, U32, P, SZ]),
        "crdt_host_orswot_decode": (P, [P, SZ]),
        "crdt_orswot_record_bytes_ex": (SZ, [U32] * 7),
        "crdt_orswot_merge_ex": (I, [P, BP, BP, P, P, SZ, U32, U32, P]),
        "crdt_orswot_validate_ex": (I, [P, BP, U32, U32, P]),
        "crdt_orswot_generate_replicas": (I, [U64, SZ, SZ, C.POINTER(RepParams), U32, U32, I, C.POINTER(P)]),
        "crdt_host_orswot_encode_ex": (C.c_long, [P, U32, U32, P, SZ]),
        "crdt_orswot_bincode_record_sizes": (I, [P, P, SZ, P, P, SZ, U32, U32, U32, U32, P, P]),
        "crdt_orswot_bincode_record_bounds": (I, [P, P, SZ, U32, U32, U32, U32, P, P]),
        "crdt_orswot_from_bincode": (I, [P, P, SZ, P, P, SZ, U32, U32, U32, U32, P, P, SZ, P]),
        "crdt_orswot_bincode_sizes": (I, [P, BP, U32, U32, U32, U32, P, P]),
        "crdt_orswot_to_bincode": (I, [P, BP, U32, U32, U32, U32, P, P, SZ, P]),
        "crdt_orswot_apply": (I, [P, BP, C.POINTER(Ops), U32, U32, P, P, SZ, P]),
        "crdt_vclock_partial_cmp": (I, [P, P, P, SZ, U32, P, P]),
        "crdt_mvreg_merge": (I, [P, P, P, P, U32, P, P, P, U32, P, P, P, U32, SZ, U32, P]),
        "crdt_map_mvreg_merge": (I, [P, C.POINTER(MapSlabC), C.POINTER(MapSlabC), C.POINTER(MapSlabC), SZ, U32, P]),
        "crdt_map_orswot_merge": (I, [P, C.POINTER(MapOrswotSlabC), C.POINTER(MapOrswotSlabC),
                                      C.POINTER(MapOrswotSlabC), SZ, U32, P]),
        "crdt_map_map_merge_scratch_bytes": (SZ, [C.POINTER(MapMapSlabC), SZ, U32]),
        "crdt_map_map_merge": (I, [P, C.POINTER(MapMapSlabC), C.POINTER(MapMapSlabC), C.POINTER(MapMapSlabC), SZ,
                                   U32, P, SZ, P]),
        "crdt_comm_unique_id": (I, [P]),
        "crdt_comm_init": (I, [P, P, I, I]),
        "crdt_comm_destroy": (I, [P]),
        "crdt_replica_allreduce_max": (I, [P, P, SZ, P]),
        "crdt_replica_reduce_scatter_max": (I, [P, P, SZ, P, P]),
        "crdt_orswot_replica_join_bound": (I, [P, BP, C.POINTER(SZ), P]),
        "crdt_orswot_replica_join": (I, [P, BP, U32, U32, P, P, SZ, C.POINTER(SZ), P]),
        "crdt_orswot_replica_join_local": (I, [P, BP, U32, U32, U32, P, P, SZ, C.POINTER(SZ), P]),
        "crdt_comm_count": (I, [P, C.POINTER(I)]),
        "crdt_dense_merge_host": (I, [P, P, P, SZ, U32]),
        "crdt_orswot_truncate": (I, [P, BP, C.POINTER(ClockCsr), U32, U32, P, P, SZ, P]),
        "crdt_vclock_csr_merge": (I, [P, C.POINTER(ClockCsr), C.POINTER(ClockCsr), C.POINTER(ClockCsrOut), P]),
        "crdt_gcounter_csr_merge": (I, [P, C.POINTER(ClockCsr), C.POINTER(ClockCsr), C.POINTER(ClockCsrOut), P]),
        "crdt_pncounter_csr_merge": (I, [P] + [C.POINTER(ClockCsr)] * 4 + [C.POINTER(ClockCsrOut)] * 2 + [P]),
        "crdt_orswot_generate_replicas_subset": (I, [U64, SZ, SZ, C.POINTER(RepParams), U32, U32, U32, U32, I,
                                                     C.POINTER(P)]),
        "crdt_orswot_replica_join_transport": (I, [P, C.POINTER(TransportC), BP, U32, U32, P, P, SZ, C.POINTER(SZ),
                                                   P]),
        "crdt_replica_allreduce_max_transport": (I, [P, C.POINTER(TransportC), P, SZ, P]),
        "crdt_replica_reduce_scatter_max_transport": (I, [P, C.POINTER(TransportC), P, SZ, P, P]),
    }
    for name, (res, args) in sig.items():
        if name in DIAG_SYMBOLS and not hasattr(L, name):
            continue  # product build: diagnostic knobs are not exported
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = None
lib = _load()


def check(rc, what=""):
    if rc != CRDT_OK:
        raise CrdtError(rc, what)
    return rc
