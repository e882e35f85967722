# Round 3: every -m gpu test + smoke, then the C2 training call ablation and the default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u tools/exp_train_ablate.py sgnn_reduce_slabs sgnn_edge_latent_grad@dw sgnn_edge_latent_grad@de0 sgnn_encode_edges_bwd sgnn_uv_bwd sgnn_node_layer_bwd sgnn_edge_layer_bwd > gpurun_out/ablate.txt 2>&1
grep -v amdgpu.ids gpurun_out/ablate.txt
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
