# One GPU-box pass: the -m gpu suite, smoke, headline bench (+ extra workloads),
# then the headline profile (kernel trace + separate PMC passes).
# Usage (from the repo root, under gpurun): bash tools/gpu_check.sh <tag> [workload ...]
set -o pipefail
TAG=${1:-r02}; shift || true
OUT=gpurun_out/chk_$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for wl in orswot "$@"; do
  timeout -k 10 300 python bench.py --workload $wl > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { echo BENCH_FAILED $wl; tail -20 $OUT/bench_$wl.err; exit 1; }
  echo "$wl $(cut -c1-400 $OUT/bench_$wl.json)"
done
bash tools/profile.sh $TAG || { echo PROF_FAILED; exit 1; }
echo ALL_OK
