#!/usr/bin/env python3
"""Interleaved A/B timing of the batched Map<u64, MVReg> merge
(crdt_map_mvreg_merge, bench.py --workload map's pairs: 250k op-built config-2
replica pairs, A = 16) over diagnostic variants (0: product, 7 waves/SIMD
register bound; 501: unbounded, 5 waves/SIMD); every variant's output slab is
checked against the oracle's merge on a sample and equal to the first
variant's in full. One JSON line."""
import argparse
import json
import os
import sys

os.environ.setdefault("CRDTS_HIP_DIAG", "1")  # variants: diagnostic build (make -C rust-crdt_amd diag)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,501")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--n-obj", type=int, default=250_000)
    a = ap.parse_args()
    import numpy as np
    import torch

    import crdts_hip
    import oracle_ffi

    n, A = a.n_obj, 16
    caps = (8, 4, 8, 8)  # bench.py run_map's
    L, R = oracle_ffi.map_generate(0xC0FFEE07, n, A, 8, 12, caps)
    eng = crdts_hip.Engine(0)
    dL, dR = L.to("cuda"), R.to("cuda")
    s = torch.cuda.Stream()
    m = 2000
    sub = lambda S, k: crdts_hip.MapSlab({f: v[:k] for f, v in S.a.items()}, S.kcap, S.mcap, S.dcap, S.scap)  # noqa: E731
    exp = oracle_ffi.map_merge(sub(L, m), sub(R, m), A).canonical()
    variants = [int(v) for v in a.variants.split(",")]
    res = {v: [] for v in variants}
    ref = None
    outs = {}
    for v in variants:  # each variant's own output slab, zeroed on the default stream before stream s writes it
        outs[v] = eng.map_mvreg_merge(dL, dR, A)
        for t in outs[v].a.values():
            t.zero_()
    torch.cuda.synchronize()
    for r in range(a.rounds + 1):
        for v in variants:
            eng.set_variant(v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            out = eng.map_mvreg_merge(dL, dR, A, stream=s, check_status=False, out=outs[v])
            e1.record(s)
            s.synchronize()
            eng.status(s)
            if r == 0:
                h = out.host().canonical()
                got = sub(out.host(), m).canonical()
                for f in exp.a:
                    assert (got.a[f] == exp.a[f]).all(), f"variant {v}: {f} differs from the oracle"
                if ref is None:
                    ref = h
                for f in ref.a:
                    assert (h.a[f] == ref.a[f]).all(), f"variant {v}: {f} differs from variant {variants[0]}"
            else:
                res[v].append(e0.elapsed_time(e1))
    outj = {"n_obj": n, "A": A, "caps": list(caps)}
    for v, t in res.items():
        outj[f"v{v}"] = {"median_ms": round(float(np.median(t)), 4), "min_ms": round(float(np.min(t)), 4),
                         "M_merges_per_s": round(n / float(np.median(t)) / 1e3, 2)}
    print(json.dumps(outj))


if __name__ == "__main__":
    main()
