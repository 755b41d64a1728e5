# Bincode decode on the GPU box: parity tests, the A/B of the decode variants
# (diagnostic build), the bincode bench line and its rocprof kernel trace +
# FETCH_SIZE / WRITE_SIZE passes. Usage: bash tools/gpu_ab_bincode.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04}
O=gpurun_out/abbc_$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "bincode or big_objects" > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/ab_bincode.py --variants ${AB_VARIANTS:-305,306,0} > $O/ab.json 2> $O/ab.err || { echo AB_FAILED; tail -30 $O/ab.err; exit 1; }
cat $O/ab.json
timeout -k 10 300 python bench.py --workload bincode > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
timeout -k 10 600 bash tools/profile_workload.sh $TAG bincode > $O/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $O/prof.log; exit 1; }
echo ALL_OK
