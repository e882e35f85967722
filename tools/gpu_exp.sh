set -e
export TMPDIR=/tmp
for wl in c2 c1_r06 c4; do
timeout -k 10 300 python bench.py --mode rollout --workload $wl --steps 20 --warmup 3 --cpu-steps 0 > gpurun_out/r_$wl.json
python -c "import json;d=json.load(open('gpurun_out/r_$wl.json'));print('$wl', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d['config']['edges'], round(d['roofline']['avg_launch_us'],1), 'us', round(d['roofline']['frac'],3))"
done
