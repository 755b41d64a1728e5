# The -m gpu tests selected by a pytest -k expression, then optionally one
# bench workload. Usage (under gpurun): bash tools/gpu_tests_k.sh <tag> "<k expr>" [workload]
set -o pipefail
TAG=$1; K=$2; WL=${3:-}
O=gpurun_out/t_$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert|^E " $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
if [ -n "$WL" ]; then
  timeout -k 10 300 python bench.py --workload $WL > $O/bench_$WL.json 2> $O/bench_$WL.err || { echo BENCH_FAILED; tail -20 $O/bench_$WL.err; exit 1; }
  cut -c1-400 $O/bench_$WL.json
fi
echo ALL_OK
