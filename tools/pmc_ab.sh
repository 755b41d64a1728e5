#!/bin/bash
# PMC passes (one counter group per run, no tracing domains) over
# tools/ab_bench.py variants (diag build).
# Usage: bash tools/pmc_ab.sh <tag> <variants> [rounds] [short]
#   short: only the instruction-mix group and FETCH / WRITE
set -euo pipefail
TAG=$1; VARS=$2; ROUNDS=${3:-3}; MODE=${4:-full}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcab_$TAG
mkdir -p $OUT
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
G2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
G3="SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"
if [ "$MODE" = short ]; then PMCG=("$G1" "FETCH_SIZE" "WRITE_SIZE"); else PMCG=("$G1" "$G2" "$G3" "FETCH_SIZE" "WRITE_SIZE"); fi
i=0
for grp in "${PMCG[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/ab_bench.py --variants $VARS --rounds $ROUNDS > $OUT/p$i.log 2>&1
done
python3 tools/pmc_ab_summary.py $OUT --json $OUT/summary.json > $OUT/summary.txt 2>&1 || true
cut -c1-600 $OUT/summary.txt
