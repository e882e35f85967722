# Round 3: step-kernel correctness (golden + oracle + 20-step headline), headline timing, phase probe.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_step.py > gpurun_out/t_step.log 2>&1 || { tail -60 gpurun_out/t_step.log; exit 1; }
tail -2 gpurun_out/t_step.log
timeout -k 10 200 python bench.py --no-extras --cpu-steps 0 > gpurun_out/b_step.json 2> gpurun_out/b_step.err || { tail -20 gpurun_out/b_step.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_step.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
timeout -k 10 120 python tools/exp_probe_step16.py c1_r15 > gpurun_out/probe_c1.txt 2>&1 && cat gpurun_out/probe_c1.txt || { tail -20 gpurun_out/probe_c1.txt; exit 1; }
timeout -k 10 400 $T tests/test_gpu_modules.py tests/test_gpu_dp.py > gpurun_out/t_mod.log 2>&1 || { tail -60 gpurun_out/t_mod.log; exit 1; }
tail -2 gpurun_out/t_mod.log
