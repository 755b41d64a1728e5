# rocprof kernel trace + FETCH_SIZE / WRITE_SIZE passes for several workloads (tools/profile_workload.sh).
set -o pipefail
for wl in ${WLS:-orswot_csr truncate mvreg map_orswot map_map}; do
  timeout -k 10 600 bash tools/profile_workload.sh r04 $wl > gpurun_out/prof_r04_$wl.log 2>&1 || { echo PROF_FAILED $wl; tail -20 gpurun_out/prof_r04_$wl.log; exit 1; }
  echo "$wl done"
done
echo ALL_OK
