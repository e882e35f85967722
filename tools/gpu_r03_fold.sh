# Round 3: in-kernel slab fold -- training parity / determinism / DP tests (H = 64 and 128), then the C2 step with and without the fold.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_dp.py tests/test_gpu_configs.py tests/test_gpu_harness.py -k "not c4_full and not c5_full" > gpurun_out/t_fold.log 2>&1 || { tail -40 gpurun_out/t_fold.log; exit 1; }
tail -2 gpurun_out/t_fold.log
timeout -k 10 300 python -u tools/exp_train_ablate.py flag:SLAB_FOLD=0 flag:SLAB_FOLD=1 > gpurun_out/ablate_fold.txt 2>&1
grep -v amdgpu.ids gpurun_out/ablate_fold.txt
