#!/bin/bash
# Dense-wide (DN) check: the wide-actor tests, then bench lines at 100 / 128 / 700 actors.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/dn_${1:-a}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_orswot.py -k "wide or dense" -x -q --timeout 170 --timeout-method thread > $OUT/t.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for a in 128 100 256; do
  timeout -k 10 300 python bench.py --n-actors $a --no-cpu-baseline > $OUT/b$a.json 2> $OUT/b$a.err || { echo BENCH_FAILED $a; tail -20 $OUT/b$a.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b$a.json').read().strip().split(chr(10))[-1]); r=d['roofline']; print($a, round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), 'ms', round(r['frac'],4))"
done
