set -e
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-steps 0 --no-rollout-extras > gpurun_out/b.json
python - <<'PY'
import json
d=json.load(open('gpurun_out/b.json'))
print('train', round(d['ms_per_step'],4), {k: round(v,1) for k,v in d['kernel_avg_us'].items()})
PY
for wl in c2 c1_r15 c4; do
timeout -k 10 300 python bench.py --mode rollout --workload $wl --steps 20 --warmup 3 --cpu-steps 0 > gpurun_out/r_$wl.json
python -c "import json;d=json.load(open('gpurun_out/r_$wl.json'));print('$wl', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', round(d['roofline']['avg_launch_us'],1), 'us', round(d['roofline']['frac'],3))"
done
timeout -k 10 300 python bench.py --mode ms-train --workload c5_small --steps 5 --warmup 2 --cpu-steps 0 > gpurun_out/ms.json
python -c "import json;d=json.load(open('gpurun_out/ms.json'));print('c5s', round(d['ms_per_step'],2), d['kernel_avg_us'])"
