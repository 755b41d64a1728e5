#!/usr/bin/env python3
"""Config-3 merge launch times, back-to-back vs synchronised between launches,
in one process (per-launch HIP events, all values printed)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))


def main():
    import numpy as np
    import torch

    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(1_000_000, threads=16)
    eng = crdts_hip.Engine(0)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    out = eng.orswot_alloc_out(L, R)
    s = torch.cuda.Stream()
    res = {}
    for mode in ("b2b", "sync", "b2b", "sleep"):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        s.synchronize()
        t0 = time.perf_counter()
        for a, b in ev:
            a.record(s)
            eng.orswot_merge(L, R, out=out, stream=s, check_status=False)
            b.record(s)
            if mode == "sync":
                s.synchronize()
            if mode == "sleep":
                s.synchronize()
                time.sleep(0.002)
        s.synchronize()
        wall = time.perf_counter() - t0
        t = [a.elapsed_time(b) for a, b in ev]
        res[mode + str(len(res))] = {"mean": float(np.mean(t)), "median": float(np.median(t)),
                                     "max": float(np.max(t)), "wall_ms_per": wall / 20 * 1e3,
                                     "all": [round(x, 3) for x in t]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
