#!/bin/bash
# Config-5 check: the sparse GPU tests, the orswot_csr bench line with a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/csr_${1:-a}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_replica.py -x -q --timeout 170 --timeout-method thread > $OUT/t.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 400 python bench.py --workload orswot_csr > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED; tail -20 $OUT/b.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); r=d['roofline']; print('csr', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), 'ms', round(r['frac'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --workload orswot_csr --steps 3 --warmup 2 --no-cpu-baseline > $OUT/kt.log 2>&1
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kt/run_kernel_stats.csv')):
    if 'crdts' in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
