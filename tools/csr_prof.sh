# kernel trace of the config-5 bench (sparse kernels), summary to stdout
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_csr -o run -- python3 bench.py --workload orswot_csr --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/csr_prof.log 2>&1
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_csr/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us', r['Percentage'])
PY
grep metric gpurun_out/csr_prof.log | cut -c1-250
