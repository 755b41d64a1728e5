#!/bin/bash
# Round-6 A/B of Orswot join variants (diag build): interleaved timing in one
# process, then the same under a kernel trace for the per-kernel split.
# Usage: bash tools/gpu_r06_ab.sh <tag> <variants> [check-variants] [extra ab_bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
TAG=$1; V=$2; C=${3:-$2}; shift 3 || true
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_bench.py --variants $V --check $C --rounds 10 "$@" > $OUT/ab.json 2> $OUT/ab.err || { echo AB_FAILED; tail -30 $OUT/ab.err; exit 1; }
cat $OUT/ab.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/ab_bench.py --variants $V --check "" --rounds 5 "$@" > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -30 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | cut -c1-220 | head -12

if [ -n "${PMC:-}" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d $OUT/pmc -o run -- python3 tools/ab_bench.py --variants $V --check "" --rounds 1 "$@" > $OUT/pmc.log 2>&1 || { echo PMC_FAILED; tail -20 $OUT/pmc.log; exit 1; }
  echo PMC_OK
fi
echo AB_OK
