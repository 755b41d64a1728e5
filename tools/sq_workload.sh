#!/bin/bash
# One SQ counter pass per workload (instruction mix and wait split per wave),
# counters never mixed with tracing. Usage (repo root, on the box):
#   bash tools/sq_workload.sh <tag> <workload> [<workload> ...]
set -euo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for WL in "$@"; do
  OUT=gpurun_out/sq_${TAG}_$WL
  mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc -o run -- python3 bench.py --workload $WL --steps 2 --warmup 0 --no-cpu-baseline > $OUT/pmc.log 2>&1
done
