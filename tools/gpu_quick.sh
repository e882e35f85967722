# Quick GPU iteration: selected tests (-k expression $1), then the C1 headline
# bench without extras, then (optional $2 = rocprof) its kernel stats.
set -e
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$1" > gpurun_out/tq.log 2>&1 || { tail -40 gpurun_out/tq.log; exit 1; }
tail -2 gpurun_out/tq.log
timeout -k 10 200 python bench.py --no-extras --cpu-steps 0 > gpurun_out/bq.json 2> gpurun_out/bq.err || { tail -20 gpurun_out/bq.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bq.json'));print('C1 ms/step',d['ms_per_step'],'edge us',d['roofline']['avg_launch_us'])"
if [ "$2" = "rocprof" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pq -o run -- python3 bench.py --no-extras --cpu-steps 0 > /dev/null 2> gpurun_out/pq.err || { tail -20 gpurun_out/pq.err; exit 1; }
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/pq/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:25]: print(r['Name'][:90].ljust(90), r['Calls'].rjust(6), '%.2f'%(float(r['AverageNs'])/1e3), r['Percentage'])
"
fi
