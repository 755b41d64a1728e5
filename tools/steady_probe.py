#!/usr/bin/env python3
"""Per-launch duration of the headline merge over a long back-to-back run
(config 3, 1M objects): HIP events around every launch on the merge stream.
Shows how many launches the part needs to reach its steady clock after the
inputs are generated (bench.py's warmup default is chosen from this).

    python tools/steady_probe.py [--launches 400] [--lib product|diag]
prints one JSON line: per-launch ms, and medians over windows of 10."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=400)
    ap.add_argument("--n-obj", type=int, default=1_000_000)
    ap.add_argument("--window", action="store_true",
                    help="also time the same launches with two events around the whole run (no per-launch events)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import crdts_hip

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(a.n_obj, threads=16)
    eng = crdts_hip.Engine(0)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    out = eng.orswot_alloc_out(L, R)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.launches)]
    for e0, e1 in ev:
        e0.record(s)
        eng.orswot_merge(L, R, out=out, stream=s, check_status=False)
        e1.record(s)
    s.synchronize()
    eng.status(s)
    ms = [e0.elapsed_time(e1) for e0, e1 in ev]
    win = [round(float(np.median(ms[i:i + 10])), 4) for i in range(0, len(ms), 10)]
    res = {"launches": a.launches, "median_by_10": win, "ms": [round(x, 4) for x in ms],
           "per_launch_events_span_ms": ev[0][0].elapsed_time(ev[-1][1]) / a.launches}
    if a.window:  # the same launches again, events only around the whole run
        w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        w0.record(s)
        for _ in range(a.launches):
            eng.orswot_merge(L, R, out=out, stream=s, check_status=False)
        w1.record(s)
        s.synchronize()
        res["window_events_ms_per_launch"] = w0.elapsed_time(w1) / a.launches
    print(json.dumps(res))


if __name__ == "__main__":
    main()
