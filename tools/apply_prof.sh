#!/bin/bash
# apply workload: kernel-trace stats, then one SQ counter pass (instruction mix / wait split)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_apply -o run -- python3 bench.py --workload apply --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/apply_prof.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_apply -o run -- python3 bench.py --workload apply --steps 1 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/apply_pmc.log 2>&1 &&
python3 - <<'PY'
import csv, collections, glob
for r in csv.DictReader(open('gpurun_out/prof_apply/run_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us', r['Percentage'])
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob('gpurun_out/pmc_apply/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'apply' not in r['Kernel_Name']: continue
        k = r['Kernel_Name'][:60]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in acc.items():
    print(k); [print('  ', c, f"{v:.4g}") for c, v in sorted(d.items())]
PY
grep metric gpurun_out/apply_prof.log | cut -c1-200
