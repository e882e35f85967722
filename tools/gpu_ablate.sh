set -e
export TMPDIR=/tmp
for wv in 4 8; do for st in 0 5 10 20; do
SGNN_EDGE_WAVES=$wv SGNN_STAGGER=$st timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_${wv}_$st -o run -- python3 bench.py --mode rollout --workload c2 --steps 10 --warmup 2 --cpu-steps 0 > /dev/null 2> gpurun_out/ab.err
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/ab_${wv}_$st/run_kernel_stats.csv')):
    if 'k_edge_layer' in r['Name']: print('waves $wv stagger $st', round(float(r['AverageNs'])/1e3,2), 'us')
"
done; done
