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


class _Outer:
    """The outer arrays of a MapMapSlab as a slab of their own, with the used
    slots of its used_bytes (the nested maps are counted on their own)."""

    def __init__(self, s):
        self.s = s

    def host(self):
        return self.s.host()

    def used_masks(self):
        s = self.s.host()
        a = s.a
        key = np.arange(s.kcap)[None, :] < a["n_keys"][:, None]
        dfr = np.arange(s.dcap)[None, :] < a["n_def"][:, None]
        dset = dfr[..., None] & (np.arange(s.scap)[None, None, :] < a["dset_n"][..., None])
        full = lambda f: np.ones(a[f].shape, bool)  # noqa: E731
        per = {"clock": full("clock"), "n_keys": full("n_keys"), "n_def": full("n_def"), "keys": key,
               "eclock": key[..., None], "dclock": dfr[..., None], "dset_n": dfr, "dset": dset}
        return {f: np.broadcast_to(m, a[f].shape) for f, m in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="map_orswot", choices=["map_orswot", "map", "map_map"])
    ap.add_argument("--n", type=int, default=100_000)
    a = ap.parse_args()
    import crdts_hip
    import oracle_ffi

    if a.workload == "map_orswot":
        caps = dict(kcap=8, mcap=8, vdcap=4, vscap=4, dcap=8, scap=8)  # bench.py run_map_orswot
        L, R = oracle_ffi.map_orswot_generate(0xC0FFEE08, a.n, 16, 6, 8, 12, 20, caps)
        M = oracle_ffi.map_orswot_merge(L, R, 16)
        slabs = (L, R, M)
    elif a.workload == "map":
        L, R = oracle_ffi.map_generate(0xC0FFEE07, a.n, 16, 8, 12, (8, 4, 8, 8))  # bench.py run_map
        M = oracle_ffi.map_merge(L, R, 16)
        slabs = (L, R, M)
    else:  # bench.py run_map_map: 10k op-path pairs (the bench tiles them; the floor ratio is the same)
        import random

        import crdts_hip
        import map_slab
        import nested_gen

        n0 = min(a.n, 10_000)
        rng = random.Random(0xC0FFEE09)
        pairs = [nested_gen.pair(rng, list(range(16))) for _ in range(n0)]
        caps, inner = dict(kcap=4, dcap=8, scap=4), (4, 8, 8, 4)
        L = crdts_hip.MapMapSlab.alloc(n0, 16, inner_caps=inner, **caps)
        R = crdts_hip.MapMapSlab.alloc(n0, 16, inner_caps=inner, **caps)
        for i, (x, y) in enumerate(pairs):
            map_slab.nested_map_to_row(x, L, i, 16)
            map_slab.nested_map_to_row(y, R, i, 16)
        M = oracle_ffi.map_map_merge(L, R, 16)
        slabs = (L, R, M)
    out = {"workload": a.workload, "n": a.n}
    for g in (32, 64, 128):
        u = t = 0
        for s in slabs:
            parts = [s] if not hasattr(s, "inner") else [_Outer(s), s.inner]
            for q in parts:
                x, y = slab_sectors(q, g)
                u += x
                t += y
        out[f"sector{g}"] = {"used_bytes": u, "sector_bytes": t, "ratio": round(t / u, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
