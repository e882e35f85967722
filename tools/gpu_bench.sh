# Default bench line + rocprofv3 kernel stats of the C1 r=15 rollout (headline).
set -e
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o c1 -- python bench.py --no-extras --cpu-steps 0 --steps 20 --warmup 5 > gpurun_out/prof_c1.log 2>&1 || { tail -20 gpurun_out/prof_c1.log; exit 1; }
find gpurun_out/prof_c1 -name "*kernel_stats.csv" | head -3
