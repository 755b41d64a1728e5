"""CPU: the C-ABI library loads and exports every symbol include/*.h declares.

No device work here (there is no GPU in the build container).
"""
import ctypes as C
import glob
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(crdt_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_functions():
    names = declared_functions()
    assert "crdt_orswot_merge" in names and "crdt_gcounter_merge" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol():
    import crdts_hip

    lib = C.CDLL(crdts_hip.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"declared but not exported: {missing}"
    # the Python binding's list is the header's list
    assert sorted(crdts_hip.EXPORTS) == declared_functions()


def exported_functions(path):
    """crdt_* functions in the library's dynamic symbol table (ELF .dynsym)."""
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return sorted({ln.split()[-1] for ln in out.splitlines()
                   if len(ln.split()) == 3 and ln.split()[1] == "T" and ln.split()[-1].startswith("crdt_")})


def test_exported_symbols_equal_declared_symbols():
    """The product library exports exactly the header's functions: no
    undeclared tuning / diagnostic entry points (those live in the
    -DCRDT_DIAG build, lib/libcrdts_hip_diag.so, used by tools/ only)."""
    import crdts_hip

    assert exported_functions(crdts_hip.LIB_PATH) == declared_functions()


def test_abi_version_and_strerror():
    import crdts_hip
    from crdts_hip._lib import lib

    assert lib.crdt_abi_version() == 1
    assert lib.crdt_strerror(-2) == b"non-canonical or inconsistent record"
    assert lib.crdt_strerror(0) == b"ok"


def test_record_bytes_agree(oracle):
    import random

    import crdts_hip
    from crdts_hip._lib import lib

    rng = random.Random(11)
    for _ in range(300):
        args = [rng.randrange(0, 50) for _ in range(6)]
        assert lib.crdt_orswot_record_bytes(*args) == oracle.record_bytes(*args) == crdts_hip.record_bytes(*args)


def test_device_entry_points_fail_cleanly_without_gpu():
    """Argument validation happens before any device call."""
    from crdts_hip._lib import lib

    assert lib.crdt_orswot_merge(None, None, None, None, None, 0, 16, None) == -1
    assert lib.crdt_gcounter_merge(None, None, None, 1, 16, None) == -1
    ctx = C.c_void_p()
    rc = lib.crdt_ctx_create(C.byref(ctx), 0)
    import torch

    if not torch.cuda.is_available():
        assert rc == -6  # CRDT_ENODEV: never a silent CPU fallback


def test_product_has_only_the_product_join_instantiation():
    """The knob variants of the join (orswot_join_kernel's timing-only
    ablations and two-pass modes, the LDS-DMA ring kernel, the join5 memory
    knobs) exist in the -DCRDT_DIAG build only: the product library's code
    objects hold orswot_join5_kernel<MINW, AW, 0> once per actor-mask width —
    the 32-bit form at 6 waves/SIMD and the 64-bit form (dense clocks of
    33-64 actors) at 5 — and no other join kernel."""
    import crdts_hip

    blob = open(crdts_hip.LIB_PATH, "rb").read()
    names = set(re.findall(rb"orswot_join5_kernelILi(\d+)ELi(\d+)ELi(\d+)E", blob))
    assert names == {(b"6", b"32", b"0"), (b"5", b"64", b"0")}, names
    assert b"orswot_join_kernelI" not in blob and b"orswot_ring_kernelI" not in blob
