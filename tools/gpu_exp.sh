set -e
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_harness.py tests/test_gpu_training.py -q -x -m gpu > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -3 gpurun_out/t.log
