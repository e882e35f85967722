# A/B of a build switch read from SGNN_AB_OLD (set = the previous behaviour) on rollout workloads:
#   bash tools/gpu_ab_env.sh <workload> [<workload> ...]
set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_par.log 2>&1 || { tail -30 gpurun_out/t_par.log; exit 1; }
tail -1 gpurun_out/t_par.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep smoke
for wl in "$@"; do
  for v in new old new old; do
    if [ $v = old ]; then export SGNN_AB_OLD=1; else unset SGNN_AB_OLD; fi
    timeout -k 10 120 python bench.py --mode rollout --workload $wl --steps 40 --warmup 5 --cpu-steps 0 --no-extras > gpurun_out/ab_$wl.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/ab_$wl.json'));r=d['roofline'];print('$wl', '$v', round(d['ms_per_step'],4), 'ms', r['kernel'], round(r['avg_launch_us'],2), 'us', round(r['frac'],3))"
  done
done
unset SGNN_AB_OLD
