set -e
export TMPDIR=/tmp
SGNN_SPLIT_H64=1 timeout -k 10 300 python -m pytest tests/test_gpu_training.py -q -x -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-steps 0 --no-rollout-extras > gpurun_out/a.json
SGNN_SPLIT_H64=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-steps 0 --no-rollout-extras > gpurun_out/b.json
python - <<'PY'
import json
for f in ['a','b']:
    d=json.load(open(f'gpurun_out/{f}.json'))
    print(f, round(d['ms_per_step'],4), {k: round(v,1) for k,v in d['kernel_avg_us'].items()})
PY
SGNN_SPLIT_H64=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_split -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-steps 0 --no-rollout-extras > /dev/null 2>&1
