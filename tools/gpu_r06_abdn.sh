#!/bin/bash
# A/B of dense-wide builds (lib/libcrdts_hip_ab_<tag>.so via CRDTS_HIP_AB):
# 100 / 128 / 256 actors and the wide-union batch, parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
OUT=gpurun_out/abdn
mkdir -p $OUT
GP='{"ancestor_adds": 96, "member_universe": 32, "pct_add": 45, "max_div_ops": 20}'
for tag in ${AB:-}; do
  CRDTS_HIP_AB=$tag timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orswot.py -k "dense_wide" > $OUT/t_$tag.log 2>&1 || { echo TESTS_FAILED $tag; tail -30 $OUT/t_$tag.log; exit 1; }
  echo "tests $tag: $(tail -1 $OUT/t_$tag.log)"
done
for tag in "" ${AB:-}; do
  line="tag=${tag:-prod}"
  for A in 100 128 256; do
    timeout -k 10 200 env CRDTS_HIP_AB=$tag python bench.py --n-actors $A --no-cpu-baseline > $OUT/a${A}_$tag.json 2> $OUT/err || { echo FAIL $tag $A; tail -5 $OUT/err; exit 1; }
    line="$line a$A $(python3 -c "import json; d=json.loads(open('$OUT/a${A}_$tag.json').read().strip().split(chr(10))[-1]); print(round(d['ms_per_step'],4), round(d['roofline']['frac'],4))")"
  done
  timeout -k 10 200 env CRDTS_HIP_AB=$tag python bench.py --n-actors 128 --gen-params "$GP" --no-cpu-baseline > $OUT/wide_$tag.json 2> $OUT/err || { echo FAIL wide $tag; exit 1; }
  line="$line wide $(python3 -c "import json; d=json.loads(open('$OUT/wide_$tag.json').read().strip().split(chr(10))[-1]); print(round(d['ms_per_step'],4), round(d['roofline']['frac'],4))")"
  echo "$line"
done
echo ABDN_OK
