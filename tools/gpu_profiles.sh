# Profiles of every workload the default bench line reports (tools/gpu.sh profile: trace-mode durations +
# FETCH_SIZE / WRITE_SIZE passes), named per round.  Usage: bash tools/gpu_profiles.sh ROUND rollout|train [workload ...]
set -e
RD=$1
MODE=$2
shift 2
R="--no-extras --cpu-steps 0"
if [ "$MODE" = rollout ]; then
  for wl in ${@:-c1_r15 c1_r06 t4800 t6400 t8000 c2 c4}; do
    case $wl in c1_r15) tag=c1r15;; c1_r06) tag=c1r06;; *) tag=$wl;; esac
    case $wl in c1_*) w=5;; *) w=3;; esac
    case $wl in c4) st=10;; *) st=20;; esac
    bash tools/gpu.sh profile ${RD}_${tag}_rollout $wl rollout --workload $wl $R --steps $st --warmup $w
  done
else
  for wl in ${@:-c2 c3 c5}; do
    case $wl in
      c2) bash tools/gpu.sh profile ${RD}_c2_train c2 train --mode train --workload c2 $R --steps 10 --warmup 3;;
      c3) bash tools/gpu.sh profile ${RD}_c3_train c3 train --mode train-c3 $R --steps 10 --warmup 3;;
      c5) bash tools/gpu.sh profile ${RD}_c5_train c5 train --mode ms-train --workload c5 $R --steps 3 --warmup 1;;
    esac
  done
fi
