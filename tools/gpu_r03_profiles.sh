# Round 3 profiles: rocprofv3 kernel stats + FETCH_SIZE + WRITE_SIZE passes (tools/profile_round.sh)
# of every workload the default bench line reports.  Usage: bash tools/gpu_r03_profiles.sh rollout|train
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date > gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
R="--no-extras --cpu-steps 0"
if [ "$1" = rollout ]; then
  bash tools/profile_round.sh r03_c1r15_rollout c1_r15 rollout -- --workload c1_r15 $R --steps 20 --warmup 5
  bash tools/profile_round.sh r03_c1r06_rollout c1_r06 rollout -- --workload c1_r06 $R --steps 20 --warmup 5
  bash tools/profile_round.sh r03_t4800_rollout t4800 rollout -- --workload t4800 $R --steps 20 --warmup 3
  bash tools/profile_round.sh r03_t6400_rollout t6400 rollout -- --workload t6400 $R --steps 20 --warmup 3
  bash tools/profile_round.sh r03_t8000_rollout t8000 rollout -- --workload t8000 $R --steps 20 --warmup 3
  bash tools/profile_round.sh r03_c2_rollout c2 rollout -- --workload c2 $R --steps 20 --warmup 3
  bash tools/profile_round.sh r03_c4_rollout c4 rollout -- --workload c4 $R --steps 10 --warmup 3
else
  bash tools/profile_round.sh r03_c2_train c2 train -- --mode train --workload c2 $R --steps 10 --warmup 3
  bash tools/profile_round.sh r03_c3_train c3 train -- --mode train-c3 $R --steps 10 --warmup 3
  bash tools/profile_round.sh r03_c5_train c5 train -- --mode ms-train --workload c5 $R --steps 3 --warmup 1
fi
ls profiles/r03_*
