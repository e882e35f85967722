# Round 3: H = 128 backward changes -- gradient tests at H = 128 (single- and multi-scale), then C5 / C4-shape timing.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_multi_scale_training.py tests/test_gpu_configs.py -k "wide_and_deep or multi_scale or c5_shapes or c4_shapes or many_particle" > gpurun_out/t_h128.log 2>&1 || { tail -40 gpurun_out/t_h128.log; exit 1; }
tail -2 gpurun_out/t_h128.log
timeout -k 10 400 python -u bench.py --mode ms-train --workload c5 --steps 3 --warmup 1 --cpu-steps 0 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c5.json')); print('C5', d['ms_per_step'], 'ms/step', d['hbm_peak_gib'], 'GiB', d['kernel_avg_us'])"
timeout -k 10 120 python -u tools/exp_probe_step16.py c1_r15 > gpurun_out/probe16.txt 2>&1; grep -v amdgpu.ids gpurun_out/probe16.txt
