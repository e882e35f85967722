set -e
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -x -m gpu > gpurun_out/t.log 2>&1 || { grep -E "Error|assert" gpurun_out/t.log | head; tail -3 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --mode rollout --workload c4 --steps 10 --warmup 2 --cpu-steps 0 > gpurun_out/c4.json 2>gpurun_out/c4.err
python -c "import json;d=json.load(open('gpurun_out/c4.json'));print(d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
timeout -k 10 600 python bench.py --mode ms-train --workload c5_small --steps 5 --warmup 2 --cpu-steps 0 > gpurun_out/c5s.json 2>gpurun_out/c5s.err
python -c "import json;d=json.load(open('gpurun_out/c5s.json'));print(d['ms_per_step'], d['value'])"
