#!/usr/bin/env python3
"""Times the LDS-DMA ring skeleton (ring_probe.hip) on config 3 next to the
product merge and the register-prefetch skeleton (skel_probe.hip variant 0),
interleaved in one process; checks that every ring variant copied each
sampled self record to its output place; one JSON line (median ms).
    python tools/probe/run_ring.py --variants 430,640 --spins 0,120"""
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
    ap.add_argument("--variants", default="420,430,530,540,630,640,860,10430,10640,20630,20640,20540,431,641")
    ap.add_argument("--spins", default="0")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--warm", type=int, default=60)
    ap.add_argument("--n-obj", type=int, default=1_000_000)
    ap.add_argument("--skel", action="store_true", help="also time skel_probe variant 0")
    a = ap.parse_args()
    import numpy as np
    import torch

    import crdts_hip

    lib = C.CDLL(os.path.join(HERE, "libring.so"))
    lib.ring_launch.restype = C.c_int
    lib.ring_launch.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
    skel = None
    if a.skel:
        skel = C.CDLL(os.path.join(HERE, "libskel.so"))
        skel.skel_launch.restype = C.c_int
        skel.skel_launch.argtypes = [C.c_int, C.c_int] + [C.c_void_p] * 8 + [C.c_uint64, C.c_void_p, C.c_void_p]
    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(a.n_obj, threads=16)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    eng = crdts_hip.Engine(0)
    out = eng.orswot_alloc_out(L, R)
    ob = torch.zeros(L.bytes + R.bytes + 4096, dtype=torch.uint8, device="cuda")
    oo = torch.zeros(a.n_obj, dtype=torch.int64, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    ctl = torch.zeros(8, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    cfgs = [("product", 0)] + ([("skel0", int(sp)) for sp in a.spins.split(",")] if skel else []) + \
        [(int(v), int(sp)) for v in a.variants.split(",") for sp in a.spins.split(",")]

    def launch(c):
        if c[0] == "product":
            eng.orswot_merge(L, R, out=out, stream=s, check_status=False)
            return 1
        sink[1] = c[1]
        if c[0] == "skel0":
            return skel.skel_launch(0, 0, L.base.data_ptr(), L.off.data_ptr(), None, R.base.data_ptr(),
                                    R.off.data_ptr(), None, ob.data_ptr(), oo.data_ptr(), a.n_obj,
                                    sink.data_ptr(), s.cuda_stream)
        return lib.ring_launch(c[0], L.base.data_ptr(), L.off.data_ptr(), L.bytes, R.base.data_ptr(),
                               R.off.data_ptr(), R.bytes, ob.data_ptr(), oo.data_ptr(), a.n_obj, ctl.data_ptr(),
                               sink.data_ptr(), s.cuda_stream)

    # correctness of every ring variant (spin 0, natural placement only):
    # sampled output places hold the self records
    rng = np.random.default_rng(7)
    samp = np.sort(rng.choice(a.n_obj, 3000, replace=False))
    lo_np, ro_np = np.asarray(lo, dtype=np.int64), np.asarray(ro, dtype=np.int64)
    checks = {}
    for c in cfgs:
        v = c[0]
        if not isinstance(v, int) or c[1] != 0 or v % 10 == 1 or 40000 <= v < 60000 or (60000 <= v < 70000 and v % 10) or (v >= 70000 and v % 100 not in (0, 5)) or (v < 1000 and v % 10 not in (0, 5)) or v % 10 in (7, 8) or v in (441, 442, 70411):
            continue  # (packed, write-ablated variants: nothing to compare)
        ob.zero_()
        assert launch(c) > 0, c
        s.synchronize()
        h = ob.cpu().numpy()
        bad = 0
        for i in samp.tolist():
            sz = int(lb[lo_np[i]:lo_np[i] + 4].view(np.uint32)[0])
            p = lo_np[i] + ro_np[i]
            bad += int(not np.array_equal(h[p:p + sz], lb[lo_np[i]:lo_np[i] + sz]))
        checks[c[0]] = bad
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
    outd = {"n_obj": a.n_obj, "in_bytes": int(in_b), "out_bytes_standin": int(lb.nbytes),
            "copy_check_bad_of_3000": checks}
    for c, v in res.items():
        ms = float(np.median(v))
        outd[f"{c[0]}_spin{c[1]}"] = {"ms": round(ms, 4), "p10": round(float(np.percentile(v, 10)), 4),
                                      "occ": occ[c], "GBps": round((in_b + lb.nbytes) / ms / 1e6, 1)}
    print(json.dumps(outd))


if __name__ == "__main__":
    main()
