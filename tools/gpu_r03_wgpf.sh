# Round 3: register-prefetched H = 128 weight-gradient GEMMs, clean build -- the H = 128 single-scale gradient test
# first (the case that faulted with a build made while the source was being edited), then the H = 128 tests, then C5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_gpu_training.py::test_wide_and_deep_mlp_gradients_against_oracle" > gpurun_out/t_wgpf1.log 2>&1 || { tail -30 gpurun_out/t_wgpf1.log; exit 1; }
tail -1 gpurun_out/t_wgpf1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multi_scale_training.py tests/test_gpu_configs.py tests/test_gpu_training.py -k "multi_scale or c5_shapes or c4_shapes or many_particle" > gpurun_out/t_wgpf2.log 2>&1 || { tail -30 gpurun_out/t_wgpf2.log; exit 1; }
tail -1 gpurun_out/t_wgpf2.log
timeout -k 10 400 python -u bench.py --mode ms-train --workload c5 --steps 3 --warmup 1 --cpu-steps 0 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c5.json')); print('C5', d['ms_per_step'], 'ms/step', d['hbm_peak_gib'], 'GiB', d['kernel_avg_us'])"
