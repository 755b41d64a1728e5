#!/usr/bin/env python3
"""Interleaved A/B of the config-5 fold (CSR Orswots, 1024-actor universe):
per variant, 7 merge launches fold 8 replicas of n objects; HIP-event time of
the whole fold; every variant's final batch compared byte for byte with the
first variant's. Prints median / min ms per fold as one JSON line."""
import argparse
import json
import os
import sys

os.environ.setdefault("CRDTS_HIP_DIAG", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,205")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--n-obj", type=int, default=1_000_000)
    a = ap.parse_args()
    import numpy as np
    import torch

    import crdts_hip

    reps = crdts_hip.generate_replicas(a.n_obj, 8, threads=16)
    U, SP = crdts_hip.CONFIG5["universe"], crdts_hip.SPARSE_CLOCK
    B = [crdts_hip.OrswotBatch.from_host(b, o, U, flags=SP) for b, o in reps]
    eng = crdts_hip.Engine(0)
    s = torch.cuda.Stream()
    vs = [int(v) for v in a.variants.split(",")]
    res = {v: [] for v in vs}
    ref = None
    for r in range(a.rounds + 1):
        for v in vs:
            eng.set_variant(v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            acc = B[0]
            for k in range(1, 8):
                acc = eng.orswot_merge(acc, B[k], stream=s, check_status=False)
            e1.record(s)
            s.synchronize()
            eng.status(s)
            if r == 0:
                c = eng.orswot_compact(acc, stream=s)
                got = c.base[: c.bytes].cpu().numpy().tobytes(), c.off.cpu().numpy().tobytes()
                if ref is None:
                    ref = got
                elif got != ref:
                    raise AssertionError(f"variant {v}: fold output differs from variant {vs[0]}")
            else:
                res[v].append(e0.elapsed_time(e1))
    print(json.dumps({f"v{v}": {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))} for v, t in res.items()}))


if __name__ == "__main__":
    main()
