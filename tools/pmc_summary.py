#!/usr/bin/env python3
"""Per-kernel averages of the counters collected by tools/pmc_variants.sh:
    python tools/pmc_summary.py gpurun_out/pmcv_<tag>"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
for vdir in sorted({os.path.basename(p).split("_")[0] for p in glob.glob(os.path.join(root, "v*_*"))}):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, vdir + "_*", "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "orswot" not in k:
                continue
            k = k.replace("void ", "").replace("crdts_hip::(anonymous namespace)::", "").split("(")[0]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {vdir}")
    for k, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"  {k}: " + ", ".join(f"{c}={v:.4g}" for c, v in sorted(avg.items())))
