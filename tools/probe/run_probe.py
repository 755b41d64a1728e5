#!/usr/bin/env python3
"""Times the memory-skeleton probe (stream_probe.hip) on config 3; one JSON line.
    python tools/probe/run_probe.py --variants 11,12,13 --bpc 0,2,4"""
import argparse
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="11,12,13,21,22")
    ap.add_argument("--bpc", default="0")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--n-obj", type=int, default=1_000_000)
    ap.add_argument("--spins", default="0")
    ap.add_argument("--no-extra", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch

    import crdts_hip

    lib = C.CDLL(os.path.join(HERE, "libprobe.so"))
    lib.probe_launch.restype = C.c_int
    lib.probe_launch.argtypes = [C.c_int, C.c_int] + [C.c_void_p] * 6 + [C.c_uint64, C.c_void_p, C.c_void_p]
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(a.n_obj, threads=16)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    ob = torch.zeros(2 * (L.bytes + R.bytes), dtype=torch.uint8, device="cuda")
    oo = torch.zeros(a.n_obj, dtype=torch.int64, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    in_bytes = lb.nbytes + rb.nbytes
    out_bytes = lb.nbytes
    cfgs = [(int(v), int(b), int(sp)) for v in a.variants.split(",") for b in a.bpc.split(",")
            for sp in a.spins.split(",")]
    res = {c: [] for c in cfgs}
    occ = {}
    for r in range(a.rounds + 1):
        for c in cfgs:
            sink[1] = c[2]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            rc = lib.probe_launch(c[0], c[1], L.base.data_ptr(), L.off.data_ptr(), R.base.data_ptr(),
                                  R.off.data_ptr(), ob.data_ptr(), oo.data_ptr(), a.n_obj, sink.data_ptr(),
                                  s.cuda_stream)
            e1.record(s)
            s.synchronize()
            assert rc > 0, rc
            occ[c] = rc
            if r:
                res[c].append(e0.elapsed_time(e1))
    lib.probe_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
    lib.probe_wonly.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
    extra = {}
    for name, fn in () if a.no_extra else (("copy_flat", lambda b: lib.probe_copy(L.base.data_ptr(), ob.data_ptr(), lb.nbytes // 16 * 16, b, s.cuda_stream)),
                     ("write_only", lambda b: lib.probe_wonly(L.base.data_ptr(), L.off.data_ptr(), ob.data_ptr(), a.n_obj, b, s.cuda_stream))):
        for blocks in (1024, 2048, 4096, 8192):
            ts = []
            for r in range(a.rounds + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                assert fn(blocks) == 1
                e1.record(s)
                s.synchronize()
                if r:
                    ts.append(e0.elapsed_time(e1))
            ms = float(np.median(ts))
            nb = 2 * lb.nbytes if name == "copy_flat" else lb.nbytes
            extra[f"{name}_b{blocks}"] = {"ms": round(ms, 4), "GBps": round(nb / ms / 1e6, 1)}
    out = dict(extra)
    for c, v in res.items():
        ms = float(np.median(v))
        out[f"v{c[0]}_bpc{c[1]}_spin{c[2]}"] = {"ms": round(ms, 4), "occ_blocks": occ[c],
                                     "GBps": round((in_bytes + out_bytes) / ms / 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
