# A/B of the in-tree library against _ab/libsgnn_hip_old.so (same box, alternating)
set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
cp sgnn_amd/_lib/libsgnn_hip.so _ab/libsgnn_hip_new.so
for i in 1 2; do
for v in new old; do
cp _ab/libsgnn_hip_$v.so sgnn_amd/_lib/libsgnn_hip.so
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-steps 0 --no-rollout-extras > gpurun_out/b.json 2>gpurun_out/b.err
python -c "import json;d=json.load(open('gpurun_out/b.json'));print('$v train', round(d['ms_per_step'],4))"
for wl in c1_r15 c2; do
timeout -k 10 300 python bench.py --mode rollout --workload $wl --steps 40 --warmup 3 --cpu-steps 0 > gpurun_out/r.json 2>gpurun_out/r.err
python -c "import json;d=json.load(open('gpurun_out/r.json'));print('$v $wl', round(d['ms_per_step'],4))"
done
done
done
cp _ab/libsgnn_hip_new.so sgnn_amd/_lib/libsgnn_hip.so
