"""Diagnostics: one config-5 fold step at a given size, mask kernel alone
(variant 203) then the full launch, synchronising after each; prints the
general-path list it leaves behind."""
import os

os.environ.setdefault("CRDTS_HIP_DIAG", "1")  # variants / stamps: diagnostic build (make -C rust-crdt_amd diag)
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, "rust-crdt_amd")
import crdts_hip  # noqa: E402
from crdts_hip._lib import lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
reps = crdts_hip.generate_replicas(n, steps + 1, threads=16)
U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
B = [crdts_hip.OrswotBatch.from_host(b, o, U, flags=SP) for b, o in reps]
eng = crdts_hip.Engine(0)
acc = B[0]
for k in range(1, steps + 1):
    eng.set_variant(203)
    o = eng.orswot_merge(acc, B[k], check_status=False)
    torch.cuda.synchronize()
    eng.status()
    buf = np.zeros(1 << 16, np.uint64)
    lib.crdt_ctx_debug_read(eng.ctx, buf.ctypes.data_as(C.c_void_p), len(buf), None)
    off = o.off.cpu().numpy().view(np.uint64)
    pend = np.nonzero(off >> np.uint64(63))[0]
    print(f"step {k}: mask kernel ok; pending {len(pend)}; list head {buf[:8].tolist()}", flush=True)
    eng.set_variant(0)
    o = eng.orswot_merge(acc, B[k], check_status=False)
    torch.cuda.synchronize()
    eng.status()
    print(f"step {k}: full launch ok", flush=True)
    acc = o
