#!/usr/bin/env python3
"""Reads the FETCH_SIZE / WRITE_SIZE passes of fetch_probe (rocprofv3 csv
dirs) and prints, per kernel, counter bytes / the kernel's true byte count."""
import csv
import json
import sys

N = 1 << 30
res = {}
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        res.setdefault(name, {})[r["Counter_Name"]] = float(r["Counter_Value"]) * 1024.0 / N
print(json.dumps(res, indent=1))
