# Round 3: step-kernel correctness (golden + oracle + 20-step headline + graph replay), headline timing,
# phase probes (C1 r = 15 and r = 0.6).  DBG=1: also the bounds-checked debug build on every path.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_step.py tests/test_gpu_graph.py > gpurun_out/t_step.log 2>&1 || { tail -60 gpurun_out/t_step.log; exit 1; }
tail -2 gpurun_out/t_step.log
timeout -k 10 200 python bench.py --no-extras --cpu-steps 0 > gpurun_out/b_step.json 2> gpurun_out/b_step.err || { tail -20 gpurun_out/b_step.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_step.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['executed_frac'])"
timeout -k 10 200 python bench.py --workload c1_r06 --no-extras --cpu-steps 0 > gpurun_out/b_r06.json 2> gpurun_out/b_step.err || { tail -20 gpurun_out/b_step.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_r06.json')); print('r06', d['ms_per_step'], d['roofline']['avg_launch_us'])"
for w in c1_r15 c1_r06; do
  timeout -k 10 120 python tools/exp_probe_step16.py $w > gpurun_out/probe_$w.txt 2>&1 && grep -v amdgpu.ids gpurun_out/probe_$w.txt || { tail -20 gpurun_out/probe_$w.txt; exit 1; }
done
if [ "${DBG:-0}" = 1 ]; then
  timeout -k 10 300 python tools/exp_debug_bounds.py > gpurun_out/debug_bounds.txt 2>&1 || { tail -30 gpurun_out/debug_bounds.txt; exit 1; }
  grep -c SGNN-BOUNDS gpurun_out/debug_bounds.txt || true
  grep -v amdgpu.ids gpurun_out/debug_bounds.txt | tail -12
fi
