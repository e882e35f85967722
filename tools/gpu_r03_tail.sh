# Round 3: training tail overlap -- training parity / determinism / DP tests, then the C2 step with and without it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_dp.py tests/test_gpu_configs.py -k "not c4_full and not c5_full" > gpurun_out/t_tail.log 2>&1 || { tail -40 gpurun_out/t_tail.log; exit 1; }
tail -2 gpurun_out/t_tail.log
timeout -k 10 300 python -u tools/exp_train_ablate.py flag:TAIL_OVERLAP=0 flag:TAIL_OVERLAP=1 flag:TAIL_OVERLAP=0 > gpurun_out/ablate_tail.txt 2>&1
grep -v amdgpu.ids gpurun_out/ablate_tail.txt
