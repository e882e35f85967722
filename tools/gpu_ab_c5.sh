# Same-box A/B of two library builds (_ab/old, _ab/new) on C5 multi-scale training, after the H = 128 gradient tests (new).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
cp _ab/new/libsgnn_hip.so sgnn_amd/_lib/libsgnn_hip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multi_scale_training.py tests/test_gpu_configs.py tests/test_gpu_training.py -k "multi_scale or c5_shapes or c4_shapes or wide_and_deep or many_particle" > gpurun_out/t_ab_c5.log 2>&1 || { tail -30 gpurun_out/t_ab_c5.log; exit 1; }
tail -1 gpurun_out/t_ab_c5.log
for v in old new old new; do
  cp _ab/$v/libsgnn_hip.so sgnn_amd/_lib/libsgnn_hip.so
  timeout -k 10 300 python bench.py --mode ms-train --workload c5 --steps 3 --warmup 1 --cpu-steps 0 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print(sys.argv[1], 'ms', round(d['ms_per_step'],2), {k: round(v,1) for k, v in d['kernel_avg_us'].items()})" "$v"
done
cp _ab/new/libsgnn_hip.so sgnn_amd/_lib/libsgnn_hip.so
