# Full default bench line + round-2 profiles (kernel stats + FETCH/WRITE passes)
# of the headline (C1 r=15 rollout), the C2 rollout and C2 training.
set -e
export TMPDIR=/tmp
bash tools/profile_round.sh r02_c1r15_rollout c1_r15 rollout -- --workload c1_r15 --no-extras --cpu-steps 0 --steps 20 --warmup 5
bash tools/profile_round.sh r02_c2_rollout c2 rollout -- --workload c2 --no-extras --cpu-steps 0 --steps 20 --warmup 5
bash tools/profile_round.sh r02_c2_train c2 train -- --mode train --workload c2 --no-extras --cpu-steps 0 --steps 10 --warmup 3
timeout -k 10 800 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json | head -c 600
