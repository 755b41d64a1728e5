#!/bin/bash
# A/B of the DN kernel's in-kernel wide join (lib/libcrdts_hip_ab_<tag>.so via
# CRDTS_HIP_AB) on the 128-actor line and the wide-union line, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/abw
mkdir -p $OUT
GP='{"ancestor_adds": 96, "member_universe": 32, "pct_add": 45, "max_div_ops": 20}'
for rep in 1 2; do
  for tag in "" ${AB:-}; do
    timeout -k 10 200 env CRDTS_HIP_AB=$tag python bench.py --n-actors 128 --no-cpu-baseline > $OUT/a128_$tag$rep.json 2> $OUT/err || { echo FAIL a128 $tag; tail -5 $OUT/err; exit 1; }
    timeout -k 10 200 env CRDTS_HIP_AB=$tag python bench.py --n-actors 128 --gen-params "$GP" --no-cpu-baseline > $OUT/wide_$tag$rep.json 2> $OUT/err || { echo FAIL wide $tag; tail -5 $OUT/err; exit 1; }
    python3 -c "
import json
f=lambda p: json.loads(open(p).read().strip().split(chr(10))[-1])
a=f('$OUT/a128_$tag$rep.json'); w=f('$OUT/wide_$tag$rep.json')
print('rep $rep tag=${tag:-prod}', 'a128', round(a['ms_per_step'],4), round(a['roofline']['frac'],4), 'wide', round(w['ms_per_step'],4), round(w['roofline']['frac'],4))"
  done
done
echo ABW_OK
