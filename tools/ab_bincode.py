#!/usr/bin/env python3
"""Interleaved A/B timing of the bincode decode pass (crdt_orswot_from_bincode
on bound-placed records, config 3, 1M objects, actors u8 / members u64) over
diagnostic variants (0: product, read-once group walk; 306: read once per object; 305: lane walk; 304: read once at 5 waves/SIMD); each variant's
records are compared byte for byte with variant 0's. One JSON line."""
import argparse
import ctypes as C
import json
import os

os.environ.setdefault("CRDTS_HIP_DIAG", "1")  # variants: diagnostic build (make -C rust-crdt_amd diag)
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,302")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--n-obj", type=int, default=1_000_000)
    a = ap.parse_args()
    import numpy as np
    import torch

    import crdts_hip
    from crdts_hip._lib import check, lib

    WA, WM, A, n = 1, 8, 16, a.n_obj
    (lb, lo), _ = crdts_hip.generate_orswot(n, threads=16)
    eng = crdts_hip.Engine(0)
    B = crdts_hip.OrswotBatch.from_host(lb, lo, A)
    blobs, boff, blen = eng.orswot_to_bincode(B, WA, WM)
    s = torch.cuda.Stream()
    st = C.c_void_p(s.cuda_stream)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    sizes = torch.empty(n, dtype=torch.int64, device="cuda")
    check(lib.crdt_orswot_bincode_record_bounds(eng.ctx, p(blen), n, WA, WM, A, 0, p(sizes), st))
    s.synchronize()
    roff = torch.cumsum(sizes, 0) - sizes
    rec = torch.zeros(int(sizes.sum().item()), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the default stream's fill is done before stream s writes
    variants = [int(v) for v in a.variants.split(",")]
    res = {v: [] for v in variants}
    for r in range(a.rounds + 1):
        for v in variants:
            eng.set_variant(v)
            if r == 0:
                with torch.cuda.stream(s):
                    rec.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            check(lib.crdt_orswot_from_bincode(eng.ctx, p(blobs), int(blobs.numel()), p(boff), p(blen), n, WA, WM, A,
                                               0, p(rec), p(roff), int(rec.numel()), st))
            e1.record(s)
            s.synchronize()
            eng.status(s)
            if r == 0:  # compacted, the records are the input batch's (ingest(egest(B)) == B)
                G = crdts_hip.OrswotBatch(rec, roff, A, int(rec.numel()), 0)
                packed = eng.orswot_compact(G, stream=s)
                nb = int(lb.nbytes)
                if not (torch.equal(packed.off, B.off) and torch.equal(packed.base[:nb], B.base[:nb])):
                    bad = (packed.base[:nb] != B.base[:nb]).nonzero().flatten()
                    bo = (packed.off != B.off).nonzero().flatten()
                    raise AssertionError(f"variant {v}: {bad.numel()} bytes, {bo.numel()} offsets differ; first bytes "
                                         f"{bad[:4].tolist()}, offsets {bo[:4].tolist()}")
            else:
                res[v].append(e0.elapsed_time(e1))
    out = {"n_obj": n, "blob_bytes": int(blen.sum().item())}
    for v, t in res.items():
        out[f"v{v}"] = {"median_ms": round(float(np.median(t)), 4), "min_ms": round(float(np.min(t)), 4),
                        "M_obj_per_s": round(n / float(np.median(t)) / 1e3, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
