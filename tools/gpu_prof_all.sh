set -e
bash tools/profile_round.sh r01_c2_train c2 train -- --steps 10 --warmup 3 --cpu-steps 0 --no-rollout-extras
bash tools/profile_round.sh r01_c2_rollout c2 rollout -- --mode rollout --workload c2 --steps 20 --warmup 3 --cpu-steps 0
bash tools/profile_round.sh r01_c1r15_rollout c1_r15 rollout -- --mode rollout --workload c1_r15 --steps 20 --warmup 3 --cpu-steps 0
bash tools/profile_round.sh r01_c4_rollout c4 rollout -- --mode rollout --workload c4 --steps 5 --warmup 1 --cpu-steps 0
timeout -k 10 900 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
ls gpurun_out/prof_*/
