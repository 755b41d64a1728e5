# codec: GPU tests + bench + kernel trace (on the GPU box)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bincode.py > gpurun_out/bc.log 2>&1 && \
timeout -k 10 300 python bench.py --workload bincode --steps 5 --warmup 2 > gpurun_out/bc_bench.json 2>gpurun_out/bc_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bc -o run -- python3 bench.py --workload bincode --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bc_prof.log 2>&1
rc=$?
tail -2 gpurun_out/bc.log
cut -c1-200 gpurun_out/bc_bench.json
python3 - <<'PY'
import csv
try:
    for r in csv.DictReader(open('gpurun_out/prof_bc/run_kernel_stats.csv')):
        if 'bincode' in r['Name']:
            print(r['Name'][40:80], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
except OSError:
    pass
PY
exit $rc
