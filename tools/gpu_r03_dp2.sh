# Round 3: multi-rank GPU training test after the bucket-range cache, plus smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dp.py > gpurun_out/t_dp2.log 2>&1 || { tail -30 gpurun_out/t_dp2.log; exit 1; }
tail -1 gpurun_out/t_dp2.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
