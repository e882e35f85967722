# Round 3 experiment (timing only): every layer's dW1e in the dE0 pass vs per layer on the side stream.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/exp_train_ablate.py flag:DEFER_DW1E=1 flag:DEFER_DW1E=0 flag:DEFER_DW1E=1 flag:DEFER_DW1E=0 > gpurun_out/ablate_defer.txt 2>&1
grep -v amdgpu.ids gpurun_out/ablate_defer.txt
