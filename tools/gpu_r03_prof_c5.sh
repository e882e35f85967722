# Round 3: C5 multi-scale training profile (kernel stats + FETCH_SIZE + WRITE_SIZE passes).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date > gpurun_out/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
bash tools/profile_round.sh r03_c5_train c5 train -- --mode ms-train --workload c5 --no-extras --cpu-steps 0 --steps 3 --warmup 1
