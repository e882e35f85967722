set -e
export TMPDIR=/tmp
SGNN_NO_GRAPH=1 timeout -k 10 300 python bench.py --mode rollout --workload c1_r15 --steps 40 --warmup 3 --cpu-steps 0 > gpurun_out/r_nog.json 2> gpurun_out/r_nog.err
echo "no-graph ok"; cat gpurun_out/r_nog.json | cut -c1-200
AMD_LOG_LEVEL=1 timeout -k 10 300 python bench.py --mode rollout --workload c1_r15 --steps 40 --warmup 3 --cpu-steps 0 > gpurun_out/r_g.json 2> gpurun_out/r_g.err
echo "graph ok"; cat gpurun_out/r_g.json | cut -c1-200
