#!/bin/bash
# The wide-union dense distribution: 128 dense actors, ~72
# present per object pair (union > 64 for 98 %), <= 64 members, ~80 dots.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/wide_${1:-a}
mkdir -p $OUT
GP='{"ancestor_adds": 96, "member_universe": 32, "pct_add": 45, "max_div_ops": 20}'
# AB="tag1 tag2": also time lib/libcrdts_hip_ab_<tag>.so (CRDTS_HIP_AB) on the same box
for tag in "" ${AB:-}; do
  timeout -k 10 300 env CRDTS_HIP_AB=$tag python bench.py --n-actors 128 --gen-params "$GP" ${BENCH_ARGS:-} > $OUT/bench$tag.json 2> $OUT/bench$tag.err || { echo BENCH_FAILED $tag; tail -20 $OUT/bench$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench$tag.json').read().strip().split(chr(10))[-1]); print('wide${tag:+ ab }$tag', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --n-actors 128 --gen-params "$GP" --no-cpu-baseline --steps 5 --warmup 2 > $OUT/prof.log 2>&1 || { echo PROF_FAILED; exit 1; }
python3 -c "
import csv, re
for r in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:4]:
    m = re.search(r'(\w+_kernel(<[^()]*>)?)', r['Name'])
    print('  ', m.group(1) if m else r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')"
echo WIDE_OK
