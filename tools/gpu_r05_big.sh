#!/bin/bash
# Big-object kernel check: its GPU tests, the phase stamps, the tail bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/big_${1:-a}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_orswot.py tests/test_gpu_big_objects.py -k "big or tail or wide" -x -q --timeout 170 --timeout-method thread > $OUT/t.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 300 python3 tools/big_stamps.py > $OUT/st.json 2> $OUT/st.err || { echo STAMPS_FAILED; tail -10 $OUT/st.err; exit 1; }
cat $OUT/st.json
timeout -k 10 300 python bench.py --workload orswot_tail --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED; tail -20 $OUT/b.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]); r=d['roofline']; print('tail', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), 'ms', round(r['frac'],4))"
