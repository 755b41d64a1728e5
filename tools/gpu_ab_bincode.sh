set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/abbc6
mkdir -p $O
timeout -k 10 300 python tools/ab_bincode.py --variants 0,302,304 > $O/ab.json 2> $O/ab.err || { echo AB_FAILED; tail -30 $O/ab.err; exit 1; }
cat $O/ab.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 tools/ab_bincode.py --variants 0,304 --rounds 2 > $O/pmc_$c.log 2>&1 || { echo PMC_FAILED $c; tail -20 $O/pmc_$c.log; exit 1; }
done

if [ -n "${PROF_MAP:-}" ]; then
  timeout -k 10 600 bash tools/profile_workload.sh r04 map > $O/prof_map.log 2>&1 || { echo PROF_MAP_FAILED; tail -20 $O/prof_map.log; exit 1; }
  echo PROF_MAP_OK
fi
echo ALL_OK
