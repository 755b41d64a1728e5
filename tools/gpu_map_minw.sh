#!/bin/bash
# Map<MVReg> merge register bound A/B (diag 0: 7 waves/SIMD, 501: unbounded,
# 502: 6 waves/SIMD): interleaved timing, then FETCH_SIZE / WRITE_SIZE passes.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/map_minw
mkdir -p $OUT
timeout -k 10 300 python3 tools/ab_map.py --variants 0,501,502 --rounds 15 > $OUT/ab.json 2> $OUT/ab.err
cat $OUT/ab.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python3 tools/ab_map.py --variants 0,501,502 --rounds 2 > $OUT/pmc_$c.log 2>&1
done
python3 tools/pmc_ab_summary.py $OUT --json $OUT/summary.json > $OUT/summary.txt 2>&1 || true
cut -c1-1500 $OUT/summary.txt
