#!/bin/bash
# Kernel shares at 100 / 128 dense actors, and the N=2 rehearsal test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/a128
mkdir -p $OUT
for a in 128 100; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$a -o run -- python3 bench.py --n-actors $a --steps 10 --warmup 20 --no-cpu-baseline > $OUT/kt$a.log 2>&1 || { echo KT_FAILED $a; tail -20 $OUT/kt$a.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kt$a/run_kernel_stats.csv')):
    if 'crdts' in r['Name']: print($a, r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_rehearse.py -x -q --timeout 300 --timeout-method thread > $OUT/reh.log 2>&1 || { echo REH_FAILED; tail -30 $OUT/reh.log; exit 1; }
tail -1 $OUT/reh.log
