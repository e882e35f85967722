# Round 3: the whole -m gpu suite + smoke, then the C2 training ablation timings.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 1000 $T tests -m gpu > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python tools/exp_train_ablate.py sgnn_reduce_slabs sgnn_edge_latent_grad sgnn_encode_nodes_bwd sgnn_encode_edges_bwd sgnn_uv_bwd sgnn_edge_layer_bwd sgnn_node_layer_bwd > gpurun_out/ablate.txt 2>&1; cat gpurun_out/ablate.txt | grep -v amdgpu.ids
