#!/usr/bin/env python3
"""Phase cycles of orswot_big_kernel (diag variant 341, ABL 8: wave 0's
s_memtime deltas summed over objects) on bench.py's orswot_tail batch; one
JSON line: per phase the mean cycles per object and the share.
    python tools/big_stamps.py [--n-obj N] [--launches K]"""
import argparse
import ctypes as C
import json
import os
import sys

os.environ["CRDTS_HIP_DIAG"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))

PHASES = ["headers", "staging", "filter+splits", "pass1", "scan", "clock+deferred/pass2", "end barrier",
          "Ooff+barrier", "list walk"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-obj", type=int, default=1_000_000)
    ap.add_argument("--launches", type=int, default=5)
    a = ap.parse_args()
    import torch

    import crdts_hip
    from crdts_hip import _lib

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot_tail(a.n_obj, threads=16)
    L = crdts_hip.OrswotBatch.from_host(lb, lo, 16)
    R = crdts_hip.OrswotBatch.from_host(rb, ro, 16)
    eng = crdts_hip.Engine(0)
    out = eng.orswot_alloc_out(L, R)
    f = _lib.lib.crdt_debug_big_stamps
    f.restype = C.c_int
    f.argtypes = [C.c_void_p]
    buf = (C.c_uint64 * 16)()
    eng.set_variant(341)
    for _ in range(3):
        eng.orswot_merge(L, R, out=out, check_status=False)
    torch.cuda.synchronize()
    assert f(buf) == 0
    for _ in range(a.launches):
        eng.orswot_merge(L, R, out=out, check_status=False)
    torch.cuda.synchronize()
    assert f(buf) == 0
    n = max(1, buf[15])
    cyc = [buf[k] / n for k in range(len(PHASES))]
    tot = sum(cyc)
    print(json.dumps({"objects": int(buf[15]), "cycles_per_object": round(tot, 1),
                      "phases": {p: {"cycles": round(c, 1), "share": round(c / tot, 3)} for p, c in zip(PHASES, cyc)}}))


if __name__ == "__main__":
    main()
