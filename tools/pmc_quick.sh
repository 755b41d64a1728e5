#!/bin/bash
# Quick PMC passes over a short bench run (one counter group per pass).
# Usage (on the box): bash tools/pmc_quick.sh <tag> [bench args]
set -euo pipefail
TAG=${1:-q}; shift || true
ARGS=${@:---steps 5 --warmup 1 --no-cpu-baseline}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$name -o run -- python3 bench.py $ARGS > $OUT/pmc_$name.log 2>&1
done
python3 - $OUT <<'PY'
import csv, collections, os, sys, json
d = sys.argv[1]; agg = collections.defaultdict(list)
for sub in os.listdir(d):
    f = os.path.join(d, sub, "run_counter_collection.csv")
    if os.path.exists(f):
        for r in csv.DictReader(open(f)):
            if ("orswot_merge_kernel<" in r["Kernel_Name"] or "orswot_mask_kernel<" in r["Kernel_Name"]):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: sum(v) / len(v) for k, v in agg.items()}
json.dump(res, open(os.path.join(d, "summary.json"), "w"), indent=1)
print(json.dumps({k: round(v / 1e6, 3) for k, v in sorted(res.items())}))
PY
