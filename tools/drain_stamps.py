#!/usr/bin/env python3
"""Timeline of the join kernel's drain (diagnostic variant 261: the product
DRN kernel with per-block stamps, s_memrealtime at 100 MHz): when blocks
leave the object loop, how many listed entries each drains, and how long the
last block's leftovers keep the launch alive."""
import ctypes as C
import json
import os
import sys

os.environ.setdefault("CRDTS_HIP_DIAG", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))


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
    eng.set_variant(int(os.environ.get("DRAIN_VARIANT", "261")))
    res = []
    for _ in range(4):
        s = torch.cuda.current_stream()
        buf = np.zeros(65536, dtype=np.uint64)
        eng.orswot_merge(L, R, out=out, check_status=False)
        torch.cuda.synchronize()
        assert lib.crdt_ctx_debug_read(eng.ctx, buf.ctypes.data, 65536, C.c_void_p(s.cuda_stream)) == 0
        st = buf[32768:32768 + 4 * 8000].reshape(-1, 4).astype(np.int64)
        blk = np.nonzero(st[:, 0] > 0)[0]
        st = st[blk]
        t0 = int(buf[32761])  # block 0 wave 0 start
        tin, tout = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0
        nmine, order = st[:, 2] >> 32, st[:, 2] & 0xFFFFFFFF
        last = np.argmax(order)
        v = int(buf[32760])
        n, c0 = v >> 32, v & 0xFFFFFFFF
        busy = nmine > 0
        res.append({"blocks": int(len(blk)), "listed": n, "left_for_last_block": n - c0,
                    "loop_end_us_p0_p10_p50_p90_max": [float(np.percentile(tin, q)) for q in (0, 10, 50, 90, 100)],
                    "drained_by_early_blocks": int(nmine.sum()),
                    "drain_us_per_entry": float(((tout - tin)[busy] / nmine[busy]).mean()) if busy.any() else None,
                    "early_drain_in_out_us": [[float(a), float(b), int(k)] for a, b, k in
                                              zip(tin[busy], tout[busy], nmine[busy])][:20],
                    "last_block_in_done_end_us": [float(tin[last]), float(tout[last]), float((st[last, 3] - t0) / 100.0)]})
    print(json.dumps(res[-1]))


if __name__ == "__main__":
    main()
