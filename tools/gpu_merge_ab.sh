# Parity of the predict/rollout paths, then A/B of the merged radius + node-encoder
# launch (SGNN_NO_RADIUS_ENC_MERGE=1 restores the two separate launches) on the small graphs.
set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_par.log 2>&1 || { tail -30 gpurun_out/t_par.log; exit 1; }
tail -1 gpurun_out/t_par.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep smoke
for wl in c1_r15 c1_r06 t4800 t8000; do
  for v in merged split merged split; do
    if [ $v = split ]; then export SGNN_NO_RADIUS_ENC_MERGE=1; else unset SGNN_NO_RADIUS_ENC_MERGE; fi
    timeout -k 10 120 python bench.py --mode rollout --workload $wl --steps 40 --warmup 5 --cpu-steps 0 > gpurun_out/ab_$wl.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/ab_$wl.json'));r=d['roofline'];print('$wl', '$v', round(d['ms_per_step'],4), 'ms', r['kernel'], round(r['avg_launch_us'],2), 'us', round(r['frac'],3))"
  done
done
unset SGNN_NO_RADIUS_ENC_MERGE
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_c1m -o run -- python3 bench.py --mode rollout --workload c1_r15 --steps 20 --warmup 2 --cpu-steps 0 > /dev/null 2> gpurun_out/st.err
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/st_c1m/**/*kernel_stats.csv',recursive=True)+glob.glob('gpurun_out/st_c1m/*kernel_stats.csv')
for r in csv.DictReader(open(f[0])): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))
"
