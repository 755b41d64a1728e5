set -o pipefail
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python tools/probe/run_ring.py --spins 0,120 --skel > $O/ring1.json 2> $O/ring1.err || { echo RING_FAILED; tail -5 $O/ring1.err; exit 1; }
cat $O/ring1.json
timeout -k 10 400 python tools/ab_bench.py --variants 0,300,301,302,303,304,305,306 --rounds 15 --check 300,301,302,303,304,305,306 > $O/ab1.json 2> $O/ab1.err || { echo AB_FAILED; tail -20 $O/ab1.err; exit 1; }
cat $O/ab1.json
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_replica_procs.py tests/test_gpu_map_nested.py tests/test_gpu_bench_rehearse.py > $O/t1.log 2>&1; echo trc=$?; tail -15 $O/t1.log
