set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 300 python bench.py --mode ms-train --workload c5_small --steps 5 --warmup 2 --cpu-steps 0 > gpurun_out/ms_small.json 2> gpurun_out/ms_small.err
timeout -k 10 300 python bench.py --mode rollout --workload c4 --steps 10 --warmup 2 --cpu-steps 0 > gpurun_out/c4.json 2> gpurun_out/c4.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-steps 0 --no-rollout-extras > gpurun_out/c2.json 2> gpurun_out/c2.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ms_small -o run -- python bench.py --mode ms-train --workload c5_small --steps 3 --warmup 1 --cpu-steps 0 > /dev/null 2> gpurun_out/prof.err
cat gpurun_out/ms_small.json gpurun_out/c4.json gpurun_out/c2.json
