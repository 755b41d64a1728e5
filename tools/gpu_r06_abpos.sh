set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/abpos
for wl in orswot_tail orswot_csr_tail; do
  for tag in "" 256 640; do
    CRDTS_HIP_AB=$tag timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/abpos/${wl}_$tag.json 2> gpurun_out/abpos/${wl}_$tag.err || { echo FAIL $wl $tag; tail -5 gpurun_out/abpos/${wl}_$tag.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abpos/${wl}_$tag.json').read().strip().split(chr(10))[-1]); print('$wl', '$tag', round(d['ms_per_step'],4), d['roofline']['frac'])"
  done
done
