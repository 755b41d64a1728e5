#!/usr/bin/env python3
"""Interleaved A/B timing of Orswot merge kernel variants in ONE process
(config 3, 1M objects): N rounds x each variant, HIP-event timing of the
merge launch(es); prints median/min ms per variant as one JSON line."""
import argparse
import json
import os

os.environ.setdefault("CRDTS_HIP_DIAG", "1")  # variants / stamps: diagnostic build (make -C rust-crdt_amd diag)
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--bpc", default="0", help="blocks per CU values to sweep (0: the kernel's occupancy)")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--n-obj", type=int, default=1_000_000)
    ap.add_argument("--check", default="", help="variants >= 100 whose output is also compared byte for byte")
    ap.add_argument("--n-actors", type=int, default=16, help="dense top-clock actors (config 3: 16)")
    ap.add_argument("--tail", action="store_true", help="bench.py's orswot_tail batch (heavy-tailed config 3)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import crdts_hip

    A = a.n_actors
    if a.tail:
        (lb, lo), (rb, ro) = crdts_hip.generate_orswot_tail(a.n_obj, threads=16)
    else:
        (lb, lo), (rb, ro) = crdts_hip.generate_orswot(a.n_obj, threads=16, **({} if A == 16 else {
            "seed": 0xC0FFEE03 + A, "params": {"n_actors": A}}))
    eng = crdts_hip.Engine(0)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, A)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, A)
    out = eng.orswot_alloc_out(L, R)
    s = torch.cuda.Stream()
    configs = [(int(v), int(b)) for v in a.variants.split(",") for b in a.bpc.split(",")]
    res = {c: [] for c in configs}
    ref = None
    seen = set()
    for r in range(a.rounds + 1):
        for c in configs:
            eng.set_variant(c[0])
            eng.set_blocks_per_cu(c[1])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            eng.orswot_merge(L, R, out=out, stream=s, check_status=False)
            e1.record(s)
            s.synchronize()
            eng.status(s)
            if r > 0:
                res[c].append(e0.elapsed_time(e1))
            checked = c[0] < 100 or str(c[0]) in a.check.split(",")
            if r == 0 and checked and c not in seen:  # byte-exact against the first variant
                seen.add(c)
                with torch.cuda.stream(s):  # same stream as the merge
                    out.base.zero_()
                eng.orswot_merge(L, R, out=out, stream=s, check_status=True)
                s.synchronize()
                # compared compacted: variants may place the records differently
                comp = eng.orswot_compact(out, stream=s)
                s.synchronize()
                if ref is None:
                    ref = (comp.base[: comp.bytes].clone(), comp.off.clone())
                elif not (torch.equal(comp.base[: comp.bytes], ref[0]) and torch.equal(comp.off, ref[1])):
                    n = min(comp.bytes, ref[0].numel())
                    bad = (comp.base[:n] != ref[0][:n]).nonzero()
                    bo = (comp.off != ref[1]).nonzero().flatten()
                    raise AssertionError(f"variant {c} output differs: {bad.numel()} bytes, first at {bad[:4].tolist()}; "
                                         f"{bo.numel()} offsets, e.g. {[(int(i), int(comp.off[i]), int(ref[1][i])) for i in bo[:4]]}")
    print(json.dumps({f"v{c[0]}_bpc{c[1]}": {"median_ms": float(np.median(v)), "min_ms": float(np.min(v))}
                      for c, v in res.items()}))


if __name__ == "__main__":
    main()
