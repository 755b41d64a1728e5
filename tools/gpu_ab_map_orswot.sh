# Map<Orswot> merge on the GPU box: its parity tests, the A/B of the LDS
# staging variants (diagnostic build) and the bench line.
# Usage: bash tools/gpu_ab_map_orswot.sh <tag>
set -o pipefail
TAG=${1:-r04}
O=gpurun_out/abmo_$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "map_orswot or orswot_map or MapOrswot" > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/ab_map_orswot.py --variants ${AB_VARIANTS:-0,401} > $O/ab.json 2> $O/ab.err || { echo AB_FAILED; tail -30 $O/ab.err; exit 1; }
cat $O/ab.json
timeout -k 10 300 python bench.py --workload map_orswot > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -20 $O/bench.err; exit 1; }
cut -c1-700 $O/bench.json
echo ALL_OK
