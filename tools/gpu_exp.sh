set -e
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_noise.py tests/test_gpu_training.py tests/test_gpu_harness.py -q -x -m gpu > gpurun_out/t.log 2>&1 || { grep -E "Error|assert" gpurun_out/t.log | head; tail -3 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-rollout-extras > gpurun_out/b.json 2>gpurun_out/b.err
python -c "import json;d=json.load(open('gpurun_out/b.json'));print(d['ms_per_step'], d['value'])"
