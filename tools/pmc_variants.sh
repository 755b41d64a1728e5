#!/bin/bash
# SQ / TA counter passes of Orswot kernel variants (diagnostic build) on the box:
#   bash tools/pmc_variants.sh <tag> <variant> [<variant> ...]
# one rocprofv3 --pmc run per counter group per variant (never mixed with tracing)
set -uo pipefail
TAG=$1; shift
export TMPDIR=/tmp
for v in "$@"; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS" \
             "TA_TA_BUSY TA_BUFFER_WAVEFRONTS" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    OUT=gpurun_out/pmcv_$TAG/v${v}_$i
    mkdir -p $OUT
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT -o run -- python3 tools/ab_bench.py --variants $v --rounds 3 > $OUT/log 2>&1 || { echo "pass $i of v$v failed"; tail -5 $OUT/log; exit 1; }
  done
done
echo PMC_DONE
