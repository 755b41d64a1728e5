#!/usr/bin/env python3
"""The HBM traffic floor a slab layout sets: for each field of a Map slab, the
distinct G-byte sectors that hold used slots (a reader that touches only used
slots still moves whole sectors), against the used bytes themselves. Prints
one JSON line per workload: used bytes, sector bytes at 32 / 64 / 128 B, and
their ratio — the measured traffic / algorithmic bytes of a kernel that reads
each used sector once and writes the output's used slots cannot go below it.
    python tools/sector_floor.py --workload map_orswot [--n 100000]"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-crdt_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def slab_sectors(slab, gran):
    """(used bytes, bytes of the sectors they touch) over every field; each
    field is its own array (its own allocation, sector-aligned at offset 0)."""
    used = touched = 0
    h = slab.host().a
    for f, m in slab.used_masks().items():
        it = h[f].dtype.itemsize
        flat = np.ascontiguousarray(m).reshape(-1)
        idx = np.nonzero(flat)[0]
        used += idx.size * it
        touched += np.unique((idx * it) // gran).size * gran
    return used, touched


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="map_orswot", choices=["map_orswot", "map"])
    ap.add_argument("--n", type=int, default=100_000)
    a = ap.parse_args()
    import crdts_hip
    import oracle_ffi

    if a.workload == "map_orswot":
        caps = dict(kcap=8, mcap=8, vdcap=4, vscap=4, dcap=8, scap=8)  # bench.py run_map_orswot
        L, R = oracle_ffi.map_orswot_generate(0xC0FFEE08, a.n, 16, 6, 8, 12, 20, caps)
        M = oracle_ffi.map_orswot_merge(L, R, 16)
    else:
        raise SystemExit("map: see bench.py run_map for its generator")
    out = {"workload": a.workload, "n": a.n}
    for g in (32, 64, 128):
        u = t = 0
        for s in (L, R, M):
            x, y = slab_sectors(s, g)
            u += x
            t += y
        out[f"sector{g}"] = {"used_bytes": u, "sector_bytes": t, "ratio": round(t / u, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
