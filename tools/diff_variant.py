#!/usr/bin/env python3
"""Diagnostic: run an Orswot kernel variant on config-3 data and describe how
its records differ from the oracle's (first few objects)."""
import argparse
import os

os.environ.setdefault("CRDTS_HIP_DIAG", "1")  # variants / stamps: diagnostic build (make -C rust-crdt_amd diag)
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "rust-crdt_amd"), os.path.join(REPO, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--show", type=int, default=3)
    a = ap.parse_args()
    import numpy as np

    import crdts_hip
    import oracle_ffi
    import records

    (lb, lo), (rb, ro) = crdts_hip.generate_orswot(a.n, threads=16)
    eng = crdts_hip.Engine(0)
    eng.set_variant(a.variant)
    out = eng.orswot_merge(crdts_hip.OrswotBatch.from_host(lb, lo, 16), crdts_hip.OrswotBatch.from_host(rb, ro, 16))
    got = out.records()
    ob, oo = oracle_ffi.orswot_merge_batch(lb, lo, rb, ro, 16, threads=16)
    exp = records.unpack_batch(ob, oo)
    L = records.unpack_batch(lb, lo)
    R = records.unpack_batch(rb, ro)
    bad = [i for i in range(a.n) if got[i] != exp[i]]
    print(f"variant {a.variant}: {len(bad)} / {a.n} differ")
    for i in bad[: a.show]:
        g, e, l, r = (records.decode(x) for x in (got[i], exp[i], L[i], R[i]))
        print(f"--- object {i}: sizes gpu {g['size']} oracle {e['size']}; nL {len(l['entries'])} nR {len(r['entries'])}"
              f" dL {sum(map(len, l['entries'].values()))} dR {sum(map(len, r['entries'].values()))}")
        if g["clock"] != e["clock"]:
            print("  clock differs", g["clock"], e["clock"])
        ks = sorted(set(g["entries"]) | set(e["entries"]))
        for k in ks:
            if g["entries"].get(k) != e["entries"].get(k):
                print(f"  member {k:#x}: gpu {g['entries'].get(k)} oracle {e['entries'].get(k)} | "
                      f"L {l['entries'].get(k)} R {r['entries'].get(k)}")
        gw = np.frombuffer(got[i], dtype=np.uint32)
        ew = np.frombuffer(exp[i], dtype=np.uint32)
        dif = np.nonzero(gw != ew)[0]
        print("  header", gw[:8].tolist(), "differing u32 words at byte offsets", (4 * dif).tolist()[:40])
        if g["deferred"] != e["deferred"]:
            print("  deferred differ", g["deferred"], e["deferred"])


if __name__ == "__main__":
    main()
