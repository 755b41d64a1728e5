#!/usr/bin/env python3
"""Wave start / end times of the headline join kernel (diagnostic variant 143:
s_memrealtime, 100 MHz, per wave). Shows how long the slowest waves keep the
launch alive after the typical wave has finished (a static-split tail)."""
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

    variant = int(os.environ.get("TAIL_VARIANT", "143"))
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(1_000_000, threads=16)
    eng = crdts_hip.Engine(0)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    out = eng.orswot_alloc_out(L, R)
    eng.set_variant(variant)
    res = []
    for _ in range(4):
        eng.orswot_merge(L, R, out=out, check_status=False)
        torch.cuda.synchronize()
        buf = np.zeros(65536, dtype=np.uint64)
        s = torch.cuda.current_stream()
        assert lib.crdt_ctx_debug_read(eng.ctx, buf.ctypes.data, 65536, C.c_void_p(s.cuda_stream)) == 0
        st = buf[32768:32768 + 3 * 10922].reshape(-1, 3)
        wid = np.nonzero(st[:, 0] > 0)[0]
        st = st[wid].astype(np.int64)
        t0 = st[:, 0].min()
        start, end = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0  # us
        dur = end - start
        nj, nhd, nch = st[:, 2] >> 32, (st[:, 2] >> 16) & 0xFFFF, st[:, 2] & 0xFFFF
        xcd = (wid // 4) % 8  # blocks of 4 waves, dispatched round-robin over the 8 XCDs
        slot = wid % 4
        late = end > np.percentile(end, 90)
        res.append({"objects_mean_std": [float(nj.mean()), float(nj.std())], "hd_mean_std": [float(nhd.mean()), float(nhd.std())],
                    "chunks_mean": float(nch.mean()),
                    "corr_dur_objects": float(np.corrcoef(dur, nj)[0, 1]) if nj.std() > 0 else None,
                    "corr_dur_hd": float(np.corrcoef(dur, nhd)[0, 1]) if nhd.std() > 0 else None,
                    "us_per_object_by_xcd": [float((dur[xcd == x] / np.maximum(nj[xcd == x], 1)).mean()) for x in range(8)],
                    "dur_by_slot": [float(dur[slot == k].mean()) for k in range(4)],
                    "late10_objects_hd": [float(nj[late].mean()), float(nhd[late].mean())],
                    "blocks_by_end_decile": [float(np.mean(wid[(end >= np.percentile(end, q)) & (end <= np.percentile(end, q + 10))] // 4)) for q in range(0, 100, 10)],"waves": int(st.shape[0]), "launch_us": float(end.max()),
                    "start_us_p50_max": [float(np.median(start)), float(start.max())],
                    "end_us_p10_p50_p90_p99_max": [float(np.percentile(end, q)) for q in (10, 50, 90, 99, 100)],
                    "dur_us_mean_std": [float(dur.mean()), float(dur.std())]})
    print(json.dumps(res[-1]))


if __name__ == "__main__":
    main()
