# A/B of two library builds (_ab/old, _ab/new) on the same bench commands:
#   bash tools/gpu_ab.sh "<bench args>" ["<bench args>" ...]
set -e
export TMPDIR=/tmp
for args in "$@"; do
  for v in old new old new; do
    cp _ab/$v/libsgnn_hip.so sgnn_amd/_lib/libsgnn_hip.so
    timeout -k 10 200 python bench.py $args --no-extras --cpu-steps 0 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print(sys.argv[1], sys.argv[2], 'ms', round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['avg_launch_us'],2), round(d['roofline']['frac'],3))" "$v" "$args"
  done
done
cp _ab/new/libsgnn_hip.so sgnn_amd/_lib/libsgnn_hip.so
