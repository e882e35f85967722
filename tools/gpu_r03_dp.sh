# Round 3: multi-rank GPU training test (incl. the overlapped per-layer buckets), then the C5 profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dp.py tests/test_gpu_training.py > gpurun_out/t_dp.log 2>&1 || { tail -40 gpurun_out/t_dp.log; exit 1; }
tail -2 gpurun_out/t_dp.log
bash tools/gpu_r03_prof_c5.sh > gpurun_out/prof_c5.log 2>&1 || { tail -20 gpurun_out/prof_c5.log; exit 1; }
tail -1 gpurun_out/prof_c5.log
