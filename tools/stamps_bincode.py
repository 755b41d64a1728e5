#!/usr/bin/env python3
"""Per-phase cycle shares of the bincode ingest decode pass (diagnostic
variant 301: s_memtime stamps; read the SHARES)."""
import ctypes as C
import json
import os

os.environ.setdefault("CRDTS_HIP_DIAG", "1")  # variants / stamps: diagnostic build (make -C rust-crdt_amd diag)
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))

PHASES = ["stage + prefetch issue", "walk", "clock", "member ranks + scan", "member writes", "deferred + header",
          "loop tail", "-"]


def main():
    import numpy as np
    import torch

    import crdts_hip
    from crdts_hip._lib import lib

    n = 1_000_000
    (lb, lo), _ = crdts_hip.generate_orswot(n, threads=16)
    eng = crdts_hip.Engine(0)
    B = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    blobs, boff, blen = eng.orswot_to_bincode(B, 1, 8)
    eng.set_variant(301)
    for _ in range(2):
        eng.orswot_from_bincode(blobs, boff, blen, 16, 1, 8, check_status=False)
    torch.cuda.synchronize()
    m = 65536
    buf = np.zeros(m, dtype=np.uint64)
    s = torch.cuda.current_stream()
    assert lib.crdt_ctx_debug_read(eng.ctx, buf.ctypes.data, m, C.c_void_p(s.cuda_stream)) == 0
    per = buf.reshape(-1, 8)
    per = per[per.sum(axis=1) > 0]
    tot = per.sum(axis=0).astype(np.float64)
    print(json.dumps({"waves": int(per.shape[0]),
                      "share": {p: round(float(t / tot.sum()), 4) for p, t in zip(PHASES, tot)},
                      "cycles_per_object": round(float(tot.sum() / n), 1)}))


if __name__ == "__main__":
    main()
