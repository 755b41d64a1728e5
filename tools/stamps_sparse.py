#!/usr/bin/env python3
"""Per-phase cycle shares of the sparse (CSR) mask kernel (diagnostic variant
204: s_memtime stamps; read the SHARES, not the absolute run time). Folds
config-5 replicas with the product kernel up to step K-1, then stamps step K."""
import ctypes as C
import json
import os

os.environ.setdefault("CRDTS_HIP_DIAG", "1")  # variants / stamps: diagnostic build (make -C rust-crdt_amd diag)
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))

PHASES = ["wait+stage", "prefetch issue", "clock union", "member ranks + scratch init", "dot masks",
          "equal/>= pass", "member join + layout", "dot/key/clock writes", "deferred pass (count)",
          "deferred pass (write)", "deferred kill (HD)", "-", "-", "-", "-", "-"]


def main():
    import numpy as np
    import torch

    import crdts_hip
    from crdts_hip._lib import lib

    n = 1_000_000
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    reps = crdts_hip.generate_replicas(n, K + 1, threads=16)
    U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
    B = [crdts_hip.OrswotBatch.from_host(b, o, U, flags=SP) for b, o in reps]
    del reps
    eng = crdts_hip.Engine(0)
    acc = B[0]
    for k in range(1, K):
        acc = eng.orswot_merge(acc, B[k])
    out = eng.orswot_alloc_out(acc, B[K])
    eng.set_variant(204)
    for _ in range(3):
        eng.orswot_merge(acc, B[K], out=out, check_status=False)
    m = 65536
    buf = np.zeros(m, dtype=np.uint64)
    s = torch.cuda.current_stream()
    assert lib.crdt_ctx_debug_read(eng.ctx, buf.ctypes.data, m, C.c_void_p(s.cuda_stream)) == 0
    per = buf.reshape(-1, 16)
    per = per[per.sum(axis=1) > 0]
    tot = per.sum(axis=0).astype(np.float64)
    print(json.dumps({"step": K, "waves": int(per.shape[0]),
                      "share": {p: round(float(t / tot.sum()), 4) for p, t in zip(PHASES, tot)},
                      "cycles_per_object": round(float(tot.sum() / n), 1)}))


if __name__ == "__main__":
    main()
