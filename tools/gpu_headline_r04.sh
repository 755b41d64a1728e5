# Headline on the GPU box: the driver's invocation (--steps 20 --warmup 5),
# the default one, the N = 2 rehearsal, then tools/profile.sh (kernel trace
# + PMC passes). Usage: bash tools/gpu_headline_r04.sh <tag>
set -o pipefail
TAG=${1:-r04}
O=gpurun_out/hl_$TAG
mkdir -p $O
if [ -n "${SKEL:-}" ]; then
  timeout -k 10 300 python tools/probe/run_skel.py --variants 0,3,200,201,202 --spins 0,120 > $O/skel.json 2> $O/skel.err || { echo SKEL_FAILED; tail -20 $O/skel.err; exit 1; }
  cat $O/skel.json
fi
if [ -n "${AB:-}" ]; then
  timeout -k 10 400 python tools/ab_bench.py --variants $AB --rounds 12 --check ${AB_CHECK:-} > $O/ab.json 2> $O/ab.err || { echo AB_FAILED; tail -20 $O/ab.err; exit 1; }
  cat $O/ab.json
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_w5.json 2> $O/bench_w5.err || { echo BENCH_W5_FAILED; tail -20 $O/bench_w5.err; exit 1; }
cut -c1-400 $O/bench_w5.json
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 300 python bench.py --gpus 2 --rehearse --n-obj 200000 --ae-n-obj 100000 --steps 3 --warmup 1 > $O/rehearse2.json 2> $O/rehearse2.err || { echo REHEARSE_FAILED; tail -30 $O/rehearse2.err; exit 1; }
cut -c1-300 $O/rehearse2.json
timeout -k 10 900 bash tools/profile.sh $TAG > $O/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $O/prof.log; exit 1; }
echo ALL_OK
