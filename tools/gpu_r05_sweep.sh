#!/bin/bash
# Every bench.py workload once on the final tree (one JSON line each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/sweep_${1:-a}
mkdir -p $OUT
for wl in vclock gcounter pncounter orswot_csr gcounter_ae clock_csr bincode apply truncate mvreg map map_orswot map_map; do
  timeout -k 10 400 python bench.py --workload $wl > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { echo BENCH_FAILED $wl; tail -10 $OUT/bench_$wl.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$wl.json').read().strip().split(chr(10))[-1]); r=d.get('roofline') or {}; print('$wl', round(d['value']/1e6,2), d['unit'], round(d['ms_per_step'],4), 'ms', r.get('frac'))"
done
echo SWEEP_OK
