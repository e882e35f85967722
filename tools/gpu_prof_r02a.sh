# Round-2 profiles (kernel stats + FETCH/WRITE passes): C1 r=15 rollout (headline), C2 rollout, C2 training.
set -e
bash tools/profile_round.sh r02_c1r15_rollout c1_r15 rollout -- --no-extras --cpu-steps 0 --steps 20 --warmup 5
bash tools/profile_round.sh r02_c2_rollout c2 rollout -- --mode rollout --workload c2 --no-extras --cpu-steps 0 --steps 20 --warmup 5
bash tools/profile_round.sh r02_c2_train c2 train -- --mode train --no-extras --cpu-steps 0 --steps 10 --warmup 3
ls profiles
