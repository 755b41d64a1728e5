#!/bin/bash
# General-kernel grid check: headline, 64 / 128 actors, tail, with kernel traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/gen_${1:-a}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_orswot.py -x -q --timeout 170 --timeout-method thread > $OUT/t.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for a in "" "--n-actors 64" "--n-actors 128" "--workload orswot_tail"; do
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED $a; tail -20 $OUT/b.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); r=d['roofline']; print('$a', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), 'ms', round(r['frac'],4))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --n-actors 64 --steps 10 --warmup 20 --no-cpu-baseline > $OUT/kt.log 2>&1
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kt/run_kernel_stats.csv')):
    if 'crdts' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
