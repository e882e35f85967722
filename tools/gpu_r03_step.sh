# Round 3: one-launch step tests + C1 headline timing + kernel stats.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_parity.py > gpurun_out/t_step.log 2>&1 || { tail -40 gpurun_out/t_step.log; exit 1; }
tail -3 gpurun_out/t_step.log
timeout -k 10 240 python bench.py --no-extras --cpu-steps 0 > gpurun_out/b_step.json 2> gpurun_out/b_step.err || { tail -20 gpurun_out/b_step.err; exit 1; }
cat gpurun_out/b_step.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_c1 -o run -- python3 bench.py --mode rollout --workload c1_r15 --steps 20 --warmup 2 --cpu-steps 0 > /dev/null 2> gpurun_out/st.err || { tail -20 gpurun_out/st.err; exit 1; }
find gpurun_out/st_c1 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -20
