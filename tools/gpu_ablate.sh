set -e
export TMPDIR=/tmp
for ab in 0 1 2 4 8 16 32 64 68 3 63 127; do
SGNN_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abb_$ab -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-steps 0 --no-rollout-extras > /dev/null 2> gpurun_out/ab.err
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/abb_$ab/run_kernel_stats.csv')):
    if 'k_edge_bwd' in r['Name']: print('ablate $ab', round(float(r['AverageNs'])/1e3,2), 'us')
"
done
