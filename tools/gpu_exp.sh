set -e
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-steps 0 --no-rollout-extras > gpurun_out/a.json
SGNN_EXP_GW=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-steps 0 --no-rollout-extras > gpurun_out/b.json
SGNN_EXP_GW=1 timeout -k 10 300 python -m pytest tests/test_gpu_training.py -q -x -m gpu 2>&1 | tail -2
python - <<'PY'
import json
for f in ['a','b']:
    d=json.load(open(f'gpurun_out/{f}.json'))
    print(f, d['ms_per_step'], d['kernel_avg_us'])
PY
