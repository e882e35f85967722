# Round 3 close: C5 profile (the weight-gradient kernels changed), every -m gpu test + smoke, default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_r03_prof_c5.sh > gpurun_out/prof_c5.log 2>&1 || { tail -20 gpurun_out/prof_c5.log; exit 1; }
tail -1 gpurun_out/prof_c5.log
cp profiles/r03_c5_train_summary.json profiles/r03_c5_train_kernel_stats.csv gpurun_out/
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
