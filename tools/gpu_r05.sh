# Round-5 GPU-box pass: the -m gpu suite (or a subset), smoke, the one-GPU
# rehearsal of bench.py's N > 1 paths (2 ranks on cuda:0 over gloo), the headline.
# Usage (from the repo root, under gpurun): bash tools/gpu_r05.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-r05}; K=${2:-}
OUT=gpurun_out/chk_$TAG
mkdir -p $OUT
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread "${KARG[@]}" > $OUT/gputests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/gputests.log; exit 1; }
[ -n "${SKIP_TESTS:-}" ] || tail -2 $OUT/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 2 --rehearse --n-obj 200000 --ae-n-obj 100000 --steps 3 --warmup 1 > $OUT/bench_rehearse2.json 2> $OUT/bench_rehearse2.err || { echo REHEARSE_FAILED; tail -30 $OUT/bench_rehearse2.err; exit 1; }
cut -c1-1500 $OUT/bench_rehearse2.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_orswot_w5.json 2> $OUT/bench_orswot_w5.err || { echo BENCH_W5_FAILED; tail -20 $OUT/bench_orswot_w5.err; exit 1; }
cut -c1-800 $OUT/bench_orswot_w5.json
timeout -k 10 300 python bench.py > $OUT/bench_orswot.json 2> $OUT/bench_orswot.err || { echo BENCH_FAILED; tail -20 $OUT/bench_orswot.err; exit 1; }
cut -c1-800 $OUT/bench_orswot.json
for wl in ${EXTRA_WL:-}; do
  timeout -k 10 300 python bench.py --workload $wl > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { echo BENCH_FAILED $wl; tail -20 $OUT/bench_$wl.err; exit 1; }
  echo "$wl $(cut -c1-700 $OUT/bench_$wl.json)"
done
echo ALL_OK
