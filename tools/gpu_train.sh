set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-steps 0 --no-rollout-extras > gpurun_out/b.json 2>gpurun_out/b.err
python -c "import json;d=json.load(open('gpurun_out/b.json'));print('train', round(d['ms_per_step'],4), d['roofline']['frac'])"
done
