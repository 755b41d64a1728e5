#!/bin/bash
# Kernel trace + stats of tools/ab_bench.py variants (diag build) on the GPU box.
# Usage: bash tools/prof_ab.sh <tag> <variants> [rounds]
set -euo pipefail
TAG=$1; VARS=$2; ROUNDS=${3:-6}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/profab_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/ab_bench.py --variants $VARS --rounds $ROUNDS > $OUT/ab.json 2> $OUT/ab.err
cat $OUT/ab.json
find $OUT/kt -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-220
