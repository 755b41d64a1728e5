#!/bin/bash
# Round-6 GPU-box pass. Usage (repo root, under gpurun):
#   [SKIP_TESTS=1] [WL="w1 w2"] [PROF="w1"] [PMC="w1"] bash tools/gpu_r06.sh <tag> [pytest -k expr]
# -m gpu tests (or a -k subset), then one bench.py line per workload in WL,
# then a kernel trace (--stats) of each workload in PROF and a traffic pass
# (FETCH_SIZE / WRITE_SIZE) plus an instruction-count pass of each in PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${1:-r06}; K=${2:-}
OUT=gpurun_out/r06_$TAG
mkdir -p $OUT
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread "${KARG[@]}" > $OUT/gputests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/gputests.log; exit 1; }
  tail -2 $OUT/gputests.log
fi
for wl in ${WL:-}; do
  timeout -k 10 400 python bench.py --workload $wl ${BENCH_ARGS:-} > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { echo BENCH_FAILED $wl; tail -20 $OUT/bench_$wl.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$wl.json').read().strip().split(chr(10))[-1]); r=d.get('roofline') or {}; print('$wl', round(d['value']/1e6,2), d['unit'], round(d['ms_per_step'],4), 'ms', 'frac', r.get('frac'), 'kernel_ms', r.get('kernel_ms'))"
done
for wl in ${PROF:-}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$wl -o run -- python3 bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_$wl.log 2>&1 || { echo PROF_FAILED $wl; tail -20 $OUT/prof_$wl.log; exit 1; }
  f=$(find $OUT/prof_$wl -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv, re
for r in list(csv.DictReader(open('$f')))[:6]:
    m = re.search(r'(\w+_kernel(<[^()]*>)?)', r['Name'])
    print('  ', m.group(1) if m else r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')"
done
for wl in ${PMC:-}; do
  for c in FETCH_SIZE WRITE_SIZE; do  # one TCC counter per pass (FETCH_SIZE takes 3 of the 4)
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_${wl}_$c -o run -- python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/pmc_${wl}_$c.log 2>&1 || { echo TRAFFIC_FAILED $wl $c; tail -20 $OUT/pmc_${wl}_$c.log; exit 1; }
  done
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d $OUT/pmc_$wl -o run -- python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/pmc_$wl.log 2>&1 || { echo PMC_FAILED $wl; tail -20 $OUT/pmc_$wl.log; exit 1; }
  echo "  pmc $wl ok"
done
echo R06_OK
