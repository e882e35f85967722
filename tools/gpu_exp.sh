set -e
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_training.py -q -x -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_t -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-steps 0 --no-rollout-extras > gpurun_out/b.json 2>/dev/null
python -c "import json;d=json.load(open('gpurun_out/b.json'));print(d['ms_per_step'])"
