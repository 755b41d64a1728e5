# Round-3 probes on the GPU box: VALU issue rates, FETCH/WRITE_SIZE calibration
# per access width, and the truncate bench. Usage (repo root): bash tools/gpu_probe_r03.sh
set -o pipefail
OUT=gpurun_out/probe_r03
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/probe/valu_probe > $OUT/valu_probe.txt 2>&1 || { echo VALU_FAILED; tail $OUT/valu_probe.txt; exit 1; }
cat $OUT/valu_probe.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/fp_$c -o run -- ./tools/probe/fetch_probe > $OUT/fp_$c.log 2>&1 || { echo FP_FAILED $c; tail $OUT/fp_$c.log; exit 1; }
done
python3 tools/probe/fetch_calib.py $OUT/fp_FETCH_SIZE $OUT/fp_WRITE_SIZE | tee $OUT/fetch_calib.json
timeout -k 10 300 python bench.py --workload truncate > $OUT/bench_truncate.json 2> $OUT/bench_truncate.err || { echo TRUNC_FAILED; tail -20 $OUT/bench_truncate.err; exit 1; }
cut -c1-1500 $OUT/bench_truncate.json
echo ALL_OK
