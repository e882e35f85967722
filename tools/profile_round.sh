# Usage (on the GPU box): bash tools/profile_round.sh TAG WORKLOAD MODE -- <bench.py args>
# Three rocprofv3 passes (kernel-trace --stats, then FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes) of the same bench command, summarised into
# profiles/TAG_summary.json + profiles/TAG_kernel_stats.csv.
set -e
TAG=$1; WL=$2; MODE=$3; shift 4
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT profiles
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py "$@" > $OUT/stats.json 2> $OUT/stats.err
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py "$@" > /dev/null 2> $OUT/fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py "$@" > /dev/null 2> $OUT/write.err
K=$(dirname $(find $OUT/stats -name run_kernel_stats.csv | head -1))
F=$(dirname $(find $OUT/fetch -name run_counter_collection.csv | head -1))
W=$(dirname $(find $OUT/write -name run_counter_collection.csv | head -1))
python3 profiles/summarize.py $TAG $WL $K $F $W $MODE
cp $K/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
cp profiles/${TAG}_summary.json $OUT/
cp profiles/${TAG}_kernel_stats.csv $OUT/
