# Full default bench line + round-2 profile of the headline (kernel stats + FETCH/WRITE passes).
set -e
export TMPDIR=/tmp
timeout -k 10 700 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
bash tools/profile_round.sh r02_c1r15_rollout c1_r15 rollout -- --no-extras --cpu-steps 0 --steps 20 --warmup 5
