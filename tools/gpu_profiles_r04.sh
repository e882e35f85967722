# Round-4 profiles of every workload the default bench line reports (tools/gpu.sh profile: trace-mode
# durations + FETCH_SIZE / WRITE_SIZE passes).  Usage: bash tools/gpu_profiles_r04.sh rollout|train
set -e
R="--no-extras --cpu-steps 0"
if [ "$1" = rollout ]; then
  bash tools/gpu.sh profile r04_c1r15_rollout c1_r15 rollout --workload c1_r15 $R --steps 20 --warmup 5
  bash tools/gpu.sh profile r04_c1r06_rollout c1_r06 rollout --workload c1_r06 $R --steps 20 --warmup 5
  bash tools/gpu.sh profile r04_t4800_rollout t4800 rollout --workload t4800 $R --steps 20 --warmup 3
  bash tools/gpu.sh profile r04_t6400_rollout t6400 rollout --workload t6400 $R --steps 20 --warmup 3
  bash tools/gpu.sh profile r04_t8000_rollout t8000 rollout --workload t8000 $R --steps 20 --warmup 3
  bash tools/gpu.sh profile r04_c2_rollout c2 rollout --workload c2 $R --steps 20 --warmup 3
  bash tools/gpu.sh profile r04_c4_rollout c4 rollout --workload c4 $R --steps 10 --warmup 3
else
  bash tools/gpu.sh profile r04_c2_train c2 train --mode train --workload c2 $R --steps 10 --warmup 3
  bash tools/gpu.sh profile r04_c3_train c3 train --mode train-c3 $R --steps 10 --warmup 3
  bash tools/gpu.sh profile r04_c5_train c5 train --mode ms-train --workload c5 $R --steps 3 --warmup 1
fi
