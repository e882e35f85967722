# Same-box A/B of two library builds (_ab/old, _ab/new) on the C2 training step (bench.py --mode train).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in old new old new old new; do
  cp _ab/$v/libsgnn_hip.so sgnn_amd/_lib/libsgnn_hip.so
  timeout -k 10 200 python bench.py --mode train --steps 20 --warmup 5 --cpu-steps 0 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print(sys.argv[1], 'ms', round(d['ms_per_step'],4), {k: round(v,1) for k, v in d['kernel_avg_us'].items()})" "$v"
done
cp _ab/new/libsgnn_hip.so sgnn_amd/_lib/libsgnn_hip.so
