#!/bin/bash
# Profiles the headline bench on the GPU box: kernel trace + stats, then PMC
# passes (one counter group per pass, never mixed with tracing domains).
# Usage (on the box, from the repo root): bash tools/profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}; shift || true
ARGS=${@:---steps 10 --warmup 50 --no-cpu-baseline}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/kt.log 2>&1
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$name -o run -- python3 bench.py $ARGS > $OUT/pmc_$name.log 2>&1
done
echo done > $OUT/DONE
