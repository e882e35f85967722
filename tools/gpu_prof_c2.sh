set -e
bash tools/profile_round.sh r01_c2_train c2 train -- --steps 10 --warmup 3 --cpu-steps 0 --no-rollout-extras
bash tools/profile_round.sh r01_c2_rollout c2 rollout -- --mode rollout --workload c2 --steps 20 --warmup 3 --cpu-steps 0
ls gpurun_out/prof_*/
