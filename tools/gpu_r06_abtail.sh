#!/bin/bash
# A/B of big-kernel builds (lib/libcrdts_hip_ab_<tag>.so via CRDTS_HIP_AB) on
# the dense heavy tail: parity tests under the variant, then the bench,
# interleaved with the product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/abtail
mkdir -p $OUT
for tag in ${AB:-}; do
  CRDTS_HIP_AB=$tag timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orswot.py -k "heavy_tail or big_kernel" > $OUT/t_$tag.log 2>&1 || { echo TESTS_FAILED $tag; tail -30 $OUT/t_$tag.log; exit 1; }
  echo "tests $tag: $(tail -1 $OUT/t_$tag.log)"
done
for rep in 1 2; do
  for tag in "" ${AB:-}; do
    timeout -k 10 200 env CRDTS_HIP_AB=$tag python bench.py --workload ${WL:-orswot_tail} --no-cpu-baseline > $OUT/b_$tag$rep.json 2> $OUT/err || { echo FAIL $tag; tail -5 $OUT/err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/b_$tag$rep.json').read().strip().split(chr(10))[-1])
print('rep $rep tag=${tag:-prod}', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
  done
done
echo ABTAIL_OK
