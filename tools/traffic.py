#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/: per-kernel average
duration (rocprofv3 --kernel-trace --stats) and per-launch HBM traffic from
the separate FETCH_SIZE / WRITE_SIZE PMC passes, plus the SQ counters.

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM / rocprofv3
section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports
half the bytes of a wide (16 B/lane) coalesced streaming read, so it is
doubled; WRITE_SIZE reads exactly for 16-B-per-lane streaming stores.

    python tools/traffic.py gpurun_out/prof_r01 profiles/r01 [traffic tag]
writes profiles/r01_kernel_stats.csv, profiles/r01_pmc.json and
profiles/traffic_<tag>.json (default tag r01: the file bench.py reads for
roofline.traffic). The 16-B streaming-read calibration is exact for the
record-streaming kernels; for kernels with other access widths (the slab
kernels' 8-B rows) the absolute is uncalibrated (guide) and the note says so.
"""
import collections
import csv
import json
import os
import shutil
import sys

KERNELS = {"orswot_join_kernel": ("orswot_join_kernel<", "orswot_join5_kernel<"), "orswot_mask_kernel": "orswot_mask_kernel<",
           "orswot_merge_general_kernel": "orswot_merge_general_kernel", "orswot_big_kernel": "orswot_big_kernel<",
           "dense_max_kernel": "dense_max_kernel"}
# every other kernel of the library is summarised under its own name
OTHER = ("orswot_apply_kernel", "orswot_sparse_mask_kernel", "orswot_sparse_general_kernel", "bincode_ingest_kernel",
         "clock_csr_merge_kernel", "orswot_truncate_kernel", "orswot_truncate_fast_kernel", "bincode_decode_big_kernel", "slice_bounds_kernel", "orswot_dense_wide_kernel",
         "bincode_egest_kernel", "bincode_decode_kernel", "bincode_sizes_lane_kernel", "bincode_bounds_kernel", "mvreg_merge_kernel",
         "vclock_cmp_kernel", "map_mvreg_merge_kernel", "map_orswot_merge_kernel", "map_map_outer_kernel", "map_mvreg_truncate_kernel", "validate_kernel", "sizes_kernel", "copy_kernel")


def short(name):
    for k, pat in KERNELS.items():
        if any(p in name for p in ((pat,) if isinstance(pat, str) else pat)):
            return k
    import re
    for k in OTHER:  # whole identifier: mvreg_merge_kernel must not match map_mvreg_merge_kernel
        if re.search(r"(?<![A-Za-z0-9_])" + k + r"(?![A-Za-z0-9_])", name):
            # instantiations told apart by their last template argument
            # (apply: workspace tier 0 / 1 / 2; egest: two passes)
            t = re.search(k + r"<(?:.*[, ])?\(?(\w+)\)?>\(", name)
            return k + ("_" + t.group(1) if t else "")
    return None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(dst)
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), dst + "_kernel_stats.csv")
    # the stats average every launch, the clock ramp of the first ~30 included;
    # the timed steps are the trace's last launches: their mean per kernel
    # (STEADY_LAUNCHES, default 10 = profile.sh's --steps) is what the bench's
    # HIP-event time is compared with
    n_last = int(os.environ.get("STEADY_LAUNCHES", "10"))
    tr = os.path.join(src, "kt", "run_kernel_trace.csv")
    if os.path.exists(tr):
        rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
        durs = collections.defaultdict(list)
        for r in rows:
            k = short(r["Kernel_Name"])
            if k:
                durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        json.dump({k: {"launches": len(v), "mean_ms_all": sum(v) / len(v), "last": min(n_last, len(v)),
                       "mean_ms_last": sum(v[-n_last:]) / len(v[-n_last:])} for k, v in durs.items()},
                  open(dst + "_kernel_steady.json", "w"), indent=1)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(os.listdir(src)):
        f = os.path.join(src, d, "run_counter_collection.csv")
        if not d.startswith("pmc_") or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    pmc = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    traffic = {}
    for k, cs in pmc.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            rd = 2.0 * cs["FETCH_SIZE"] * 1024.0
            wr = cs["WRITE_SIZE"] * 1024.0
            note = "per launch; FETCH_SIZE x2 (gfx950 16-B streaming-read correction), KiB->B"
            if k.startswith(("mvreg_merge_kernel", "map_", "vclock_cmp_kernel", "orswot_apply_kernel")):
                note += ("; partial-line 8-B / 4-B accesses: x2 FETCH_SIZE is the 128-B line traffic "
                         "(calibrated, profiles/r05_fetch_calib_partial_lines.json)")
            traffic[k] = {"read_bytes": rd, "write_bytes": wr, "total_bytes": rd + wr, "note": note}
    json.dump({"pmc_avg_per_launch": pmc, "source": src}, open(dst + "_pmc.json", "w"), indent=1)
    tdir = os.path.dirname(dst) or "."
    json.dump({k: v["total_bytes"] for k, v in traffic.items()} | {"detail": traffic},
              open(os.path.join(tdir, f"traffic_{tag}.json"), "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
