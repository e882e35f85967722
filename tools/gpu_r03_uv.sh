# Round 3: uv backward gather change -- training tests, then the C2 step (twice) with the call ablation.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_dp.py tests/test_gpu_configs.py tests/test_gpu_multi_scale_training.py -k "not c4_full and not c5_full" > gpurun_out/t_uv.log 2>&1 || { tail -40 gpurun_out/t_uv.log; exit 1; }
tail -1 gpurun_out/t_uv.log
timeout -k 10 300 python -u tools/exp_train_ablate.py sgnn_uv_bwd sgnn_reduce_slabs > gpurun_out/ablate_uv.txt 2>&1
grep -v amdgpu.ids gpurun_out/ablate_uv.txt
