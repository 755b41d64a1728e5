set -o pipefail
mkdir -p gpurun_out/fin
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin/gputests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/fin/gputests.log; exit 1; }
tail -2 gpurun_out/fin/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
tail -1 gpurun_out/fin/smoke.log
for wl in orswot apply mvreg map; do
  timeout -k 10 240 python bench.py --workload $wl > gpurun_out/fin/bench_$wl.json 2> gpurun_out/fin/bench_$wl.err || { echo BENCH_FAILED $wl; exit 1; }
  echo "$wl $(cut -c1-160 gpurun_out/fin/bench_$wl.json)"
done
for wl in apply mvreg map; do bash tools/profile_workload.sh r01e $wl || { echo PROF_FAILED $wl; exit 1; }; done
echo ALL_OK
