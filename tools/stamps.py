#!/usr/bin/env python3
"""Per-phase cycle shares of the Orswot fast kernel (diagnostic variant 109:
s_memtime stamps; read the SHARES, not the absolute run time)."""
import ctypes as C
import json
import os

os.environ.setdefault("CRDTS_HIP_DIAG", "1")  # variants / stamps: diagnostic build (make -C rust-crdt_amd diag)
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))

PHASES = (["wait+stage", "prefetch issue", "merge path", "count join", "scan+layout(+def count)",
           "member/def writes to LDS", "copy-out", "chunk state"]
          if os.environ.get("STAMP_VARIANT", "109") == "109" else
          ["wait+stage", "prefetch issue", "mask: member join + writes", "mask: same (deferred objs)",
           "mask: dot loads + rank search", "mask: heads + mask atomics", "mask: equal/>= pass", "chunk state"])


def main():
    import numpy as np
    import torch

    import crdts_hip
    from crdts_hip._lib import lib

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(1_000_000, threads=16)
    eng = crdts_hip.Engine(0)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    out = eng.orswot_alloc_out(L, R)
    eng.set_variant(int(os.environ.get("STAMP_VARIANT", "109")))
    for _ in range(3):
        eng.orswot_merge(L, R, out=out, check_status=False)
    n = 65536
    buf = np.zeros(n, dtype=np.uint64)
    s = torch.cuda.current_stream()
    assert lib.crdt_ctx_debug_read(eng.ctx, buf.ctypes.data, n, C.c_void_p(s.cuda_stream)) == 0
    per = buf.reshape(-1, 8)
    per = per[per.sum(axis=1) > 0]
    tot = per.sum(axis=0).astype(np.float64)
    print(json.dumps({"waves": int(per.shape[0]),
                      "share": {p: round(float(t / tot.sum()), 4) for p, t in zip(PHASES, tot)},
                      "cycles_per_object_per_wave": round(float(tot.sum() / 1_000_000 * 1.0), 1)}))


if __name__ == "__main__":
    main()
