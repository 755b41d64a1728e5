# Map<MVReg> / nested-map kernels on the GPU box: their parity tests and bench
# lines. Usage: bash tools/gpu_map_check.sh <tag>
set -o pipefail
TAG=${1:-r04}
O=gpurun_out/map_$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "map" > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for wl in map map_map; do
  timeout -k 10 300 python bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo BENCH_FAILED $wl; tail -20 $O/bench_$wl.err; exit 1; }
  echo "$wl $(cut -c1-300 $O/bench_$wl.json)"
done
echo ALL_OK
