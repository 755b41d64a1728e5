#!/bin/bash
# Per-workload rocprofv3 evidence on the GPU box: kernel trace + stats, then one
# FETCH_SIZE and one WRITE_SIZE PMC pass (counters never mixed with tracing).
# Usage (repo root, on the box): bash tools/profile_workload.sh <tag> <workload> [bench args...]
set -euo pipefail
TAG=$1; WL=$2; shift 2
ARGS="--workload $WL --steps 5 --warmup 20 --no-cpu-baseline $*"
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}_$WL
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python3 bench.py $ARGS > $OUT/pmc_$c.log 2>&1
done
echo done > $OUT/DONE
