#!/bin/bash
# TA / TD / LDS busy counters of diagnostic variants (tools/ab_bench.py, one
# variant per rocprofv3 pass). Usage (on the box): bash tools/pmc_variants_td.sh "0 136 137"
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_td
mkdir -p $OUT
for v in ${1:-0 136 137}; do
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/v$v -o run -- python3 tools/ab_bench.py --variants $v --rounds 3 > $OUT/v$v.log 2>&1 || { echo "variant $v failed rc=$?"; tail -5 $OUT/v$v.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, collections, os, sys, json
d = sys.argv[1]; out = {}
for sub in sorted(os.listdir(d)):
    f = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "orswot_join_kernel<" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out[sub] = {k: round(sum(v) / len(v) / 1e6, 3) for k, v in agg.items()}
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
print(json.dumps(out))
PY
