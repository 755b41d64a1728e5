#!/bin/bash
# Round-5 Map pass on the GPU box: the Map GPU tests, then per Map workload a
# bench line and tools/profile_workload.sh's trace + FETCH / WRITE passes.
# Usage (repo root, on the box): bash tools/gpu_r05_maps.sh <tag>
set -o pipefail
TAG=${1:-r05}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/maps_$TAG
mkdir -p $OUT
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_map_nested.py tests/test_gpu_map_orswot.py tests/test_map_mvreg.py -m gpu -x -q --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
[ -n "${SKIP_TESTS:-}" ] || tail -2 $OUT/tests.log
for wl in ${WLS:-map_map map map_orswot}; do
  timeout -k 10 400 python bench.py --workload $wl > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { echo BENCH_FAILED $wl; tail -20 $OUT/bench_$wl.err; exit 1; }
  echo "$wl $(cut -c1-600 $OUT/bench_$wl.json)"
  bash tools/profile_workload.sh $TAG $wl || { echo PROF_FAILED $wl; exit 1; }
done
echo ALL_OK
