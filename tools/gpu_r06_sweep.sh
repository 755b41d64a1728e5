#!/bin/bash
# Round-6 final evidence on one box: (1) every bench.py workload once (one
# JSON line each, default sizes), (2) the headline's kernel trace + PMC passes
# (tools/profile.sh), (3) traffic passes of the workloads this round changed
# (tools/profile_workload.sh), (4) the N = 2 rehearsal and the driver-shaped
# headline (--warmup 5 --steps 20). Usage: bash tools/gpu_r06_sweep.sh <tag> <part: bench|prof|tail>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=${1:-r06z}; PART=${2:-bench}
OUT=gpurun_out/sweep_$TAG
mkdir -p $OUT
if [ "$PART" = bench ]; then
  for wl in orswot vclock gcounter pncounter orswot_csr gcounter_ae clock_csr bincode apply truncate mvreg map map_orswot map_map orswot_tail orswot_csr_tail; do
    timeout -k 10 400 python bench.py --workload $wl > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { echo BENCH_FAILED $wl; tail -10 $OUT/bench_$wl.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/bench_$wl.json').read().strip().split(chr(10))[-1]); r=d.get('roofline') or {}; print('$wl', round(d['value']/1e6,2), d['unit'], round(d['ms_per_step'],4), 'ms', r.get('frac'))"
  done
  timeout -k 10 300 python bench.py --n-actors 64 > $OUT/bench_orswot_a64.json 2> $OUT/bench_orswot_a64.err || { echo BENCH_FAILED a64; exit 1; }
  timeout -k 10 300 python bench.py --n-actors 128 > $OUT/bench_orswot_a128.json 2> $OUT/bench_orswot_a128.err || { echo BENCH_FAILED a128; exit 1; }
  timeout -k 10 300 python bench.py --n-actors 128 --gen-params '{"ancestor_adds": 96, "member_universe": 32, "pct_add": 45, "max_div_ops": 20}' > $OUT/bench_orswot_wide.json 2> $OUT/bench_orswot_wide.err || { echo BENCH_FAILED wide; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_orswot_wide.json').read().strip().split(chr(10))[-1]); print('wide', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['roofline']['frac'])"
  python3 -c "import json; d=json.loads(open('$OUT/bench_orswot_a128.json').read().strip().split(chr(10))[-1]); print('a128', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['roofline']['frac'])"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_orswot_w5.json 2> $OUT/bench_orswot_w5.err || { echo BENCH_FAILED w5; exit 1; }
  cut -c1-400 $OUT/bench_orswot_w5.json
  timeout -k 10 300 python bench.py --gpus 2 --rehearse --n-obj 200000 --ae-n-obj 100000 --steps 3 --warmup 1 > $OUT/bench_rehearse2.json 2> $OUT/bench_rehearse2.err || { echo REHEARSE_FAILED; tail -20 $OUT/bench_rehearse2.err; exit 1; }
  cut -c1-300 $OUT/bench_rehearse2.json
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
elif [ "$PART" = prof ]; then
  bash tools/profile.sh $TAG || { echo PROFILE_FAILED; exit 1; }
  for wl in truncate orswot_tail orswot_csr_tail orswot_csr; do
    bash tools/profile_workload.sh $TAG $wl || { echo PROFILE_WL_FAILED $wl; exit 1; }
  done
  bash tools/profile_workload.sh ${TAG}_a128 orswot --n-actors 128 || { echo PROFILE_WL_FAILED a128; exit 1; }
  bash tools/profile_workload.sh ${TAG}_wide orswot --n-actors 128 \
    --gen-params '{"ancestor_adds":96,"member_universe":32,"pct_add":45,"max_div_ops":20}' || { echo PROFILE_WL_FAILED wide; exit 1; }
fi
echo SWEEP_OK
