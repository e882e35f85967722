# Round 3: new tests, training ablation / A-B, then the default bench line (progress on stderr into gpurun_out/).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_training.py -k "caps_above or bruteforce or many_particle or particle_types or against_oracle_autograd or deterministic or trainer_step" > gpurun_out/t_cap.log 2>&1 || { tail -30 gpurun_out/t_cap.log; exit 1; }
tail -2 gpurun_out/t_cap.log
timeout -k 10 400 python -u tools/exp_train_ablate.py flag:DW1E_IN_LAYER=0 sgnn_reduce_slabs sgnn_edge_latent_grad@de0 sgnn_encode_nodes_bwd sgnn_encode_edges_bwd sgnn_uv_bwd sgnn_edge_layer_bwd sgnn_node_layer_bwd sgnn_transpose_csr sgnn_adam_step > gpurun_out/ablate.txt 2>&1
grep -v amdgpu.ids gpurun_out/ablate.txt
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
