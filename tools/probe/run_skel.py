#!/usr/bin/env python3
"""Times the data-flow skeleton (skel_probe.hip) on config 3 next to the
product merge, interleaved in one process; one JSON line (median ms).
    python tools/probe/run_skel.py --variants 0,1,10,11 --spins 0,200"""
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
    ap.add_argument("--variants", default="0,1,10,11")
    ap.add_argument("--spins", default="0")
    ap.add_argument("--rounds", type=int, default=25)
    ap.add_argument("--warm", type=int, default=60)
    ap.add_argument("--n-obj", type=int, default=1_000_000)
    a = ap.parse_args()
    import numpy as np
    import torch

    import crdts_hip

    lib = C.CDLL(os.path.join(HERE, "libskel.so"))
    lib.skel_launch.restype = C.c_int
    lib.skel_launch.argtypes = [C.c_int, C.c_int] + [C.c_void_p] * 8 + [C.c_uint64, C.c_void_p, C.c_void_p]
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(a.n_obj, threads=16)

    def shape(b, o):
        w = b[: b.nbytes // 4 * 4].view(np.uint32)
        i = (o // 4).astype(np.int64)
        return (w[i].astype(np.uint64) | ((w[i + 2] + w[i + 3] + w[i + 4]).astype(np.uint64) << np.uint64(32)))

    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    Ls = torch.from_numpy(shape(lb, lo).view(np.int64)).cuda()
    Rs = torch.from_numpy(shape(rb, ro).view(np.int64)).cuda()
    eng = crdts_hip.Engine(0)
    out = eng.orswot_alloc_out(L, R)
    ob = torch.zeros(L.bytes + R.bytes + 4096, dtype=torch.uint8, device="cuda")
    oo = torch.zeros(a.n_obj, dtype=torch.int64, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    cfgs = [("product", 0)] + [(int(v), int(sp)) for v in a.variants.split(",") for sp in a.spins.split(",")]

    def launch(c):
        if c[0] == "product":
            eng.orswot_merge(L, R, out=out, stream=s, check_status=False)
            return 1
        sink[1] = c[1]
        return lib.skel_launch(c[0], 0, L.base.data_ptr(), L.off.data_ptr(), Ls.data_ptr(), R.base.data_ptr(),
                               R.off.data_ptr(), Rs.data_ptr(), ob.data_ptr(), oo.data_ptr(), a.n_obj,
                               sink.data_ptr(), s.cuda_stream)

    torch.cuda.synchronize()
    for _ in range(a.warm):  # past the part's clock ramp
        launch(cfgs[0])
    s.synchronize()
    res = {c: [] for c in cfgs}
    occ = {}
    for r in range(a.rounds):
        for c in cfgs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            rc = launch(c)
            e1.record(s)
            s.synchronize()
            assert rc > 0, (c, rc)
            occ[c] = rc
            res[c].append(e0.elapsed_time(e1))
    in_b = lb.nbytes + rb.nbytes
    outd = {"n_obj": a.n_obj, "in_bytes": int(in_b), "out_bytes_standin": int(lb.nbytes)}
    for c, v in res.items():
        ms = float(np.median(v))
        outd[f"{c[0]}_spin{c[1]}"] = {"ms": round(ms, 4), "p10": round(float(np.percentile(v, 10)), 4),
                                      "occ": occ[c], "GBps": round((in_b + lb.nbytes) / ms / 1e6, 1)}
    print(json.dumps(outd))


if __name__ == "__main__":
    main()
