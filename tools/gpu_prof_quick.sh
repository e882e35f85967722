# Kernel stats (rocprofv3 --kernel-trace --stats) of one bench configuration:
#   bash tools/gpu_prof_quick.sh TAG <bench.py args...>
set -e
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pq_$TAG -o run -- python3 bench.py "$@" > gpurun_out/pq_$TAG.json 2> gpurun_out/pq_$TAG.err || { tail -20 gpurun_out/pq_$TAG.err; exit 1; }
python3 - "$TAG" <<'PY'
import csv, glob, json, sys
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/pq_{tag}/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:22]:
    print(r["Name"].replace("(anonymous namespace)::", "")[:64].ljust(64), r["Calls"].rjust(5),
          "%8.2f" % (float(r["AverageNs"]) / 1e3), r["Percentage"][:5])
d = json.load(open(f"gpurun_out/pq_{tag}.json"))
print("ms_per_step", d.get("ms_per_step"))
PY
