set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --mode ms-train --workload c5 --steps 3 --warmup 1 --cpu-steps 3 > gpurun_out/c5_train.json 2> gpurun_out/c5_train.err
cat gpurun_out/c5_train.json
timeout -k 10 300 python bench.py --mode ms-rollout --workload c5 --steps 5 --warmup 1 --cpu-steps 0 > gpurun_out/c5_roll.json 2> gpurun_out/c5_roll.err
cat gpurun_out/c5_roll.json
