#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lds
mkdir -p $OUT
i=0
for grp in "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" "TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, collections, os, sys, json
d = sys.argv[1]; agg = collections.defaultdict(list)
for sub in sorted(os.listdir(d)):
    f = os.path.join(d, sub, "run_counter_collection.csv")
    if os.path.exists(f):
        for r in csv.DictReader(open(f)):
            if "orswot_join_kernel<" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: sum(v) / len(v) for k, v in agg.items()}
json.dump(res, open(os.path.join(d, "summary.json"), "w"), indent=1)
print(json.dumps({k: round(v / 1e6, 3) for k, v in sorted(res.items())}))
PY
