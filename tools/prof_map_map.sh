export TMPDIR=/tmp
mkdir -p gpurun_out/prof_mm
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mm/kt -o run -- python3 bench.py --workload map_map --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_mm/kt.log 2>&1 && head -8 gpurun_out/prof_mm/kt/run_kernel_stats.csv | cut -c1-220
