#!/usr/bin/env python3
"""Per-kernel averages of every counter under a tools/pmc_ab.sh output dir
(kernels told apart by their full template name):
    python tools/pmc_ab_summary.py gpurun_out/pmcab_<tag> [--json out.json]"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "orswot" not in k:
            continue
        k = k.replace("void ", "").replace("crdts_hip::(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
for k, avg in out.items():
    print(f"{k}:\n  " + ", ".join(f"{c}={v:.4g}" for c, v in sorted(avg.items())))
if "--json" in sys.argv:
    with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
        json.dump(out, fh, indent=1)
