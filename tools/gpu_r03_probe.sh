# Round 3: the step kernel's phase probe only (experiment library).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/exp_probe_step16.py c1_r15 > gpurun_out/probe_c1.txt 2>&1 && cat gpurun_out/probe_c1.txt || { tail -20 gpurun_out/probe_c1.txt; exit 1; }
