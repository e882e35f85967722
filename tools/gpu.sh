# GPU-box steps, one parameterised script (run through gpurun; every GPU step has its own time limit and
# the first failing step ends the script).
#
#   bash tools/gpu.sh tests [pytest -k expr]     every -m gpu test (or a -k subset)   -> gpurun_out/t.log
#   bash tools/gpu.sh smoke                      __graft_entry__.smoke()               -> gpurun_out/smoke.log
#   bash tools/gpu.sh bench [bench.py args]      one bench line                        -> gpurun_out/bench.json
#   bash tools/gpu.sh handoff VARIANT [SKEW]    the step's hand-off check build (base: the shipping kernel)
#   bash tools/gpu.sh bounds128                  H = 128 gradient tests on the bounds-checked library
#   bash tools/gpu.sh profile TAG WORKLOAD MODE [bench.py args]
#        rocprofv3 kernel trace (--stats, durations) + separate FETCH_SIZE / WRITE_SIZE passes of the same
#        bench command -> profiles/TAG_summary.json (+ TAG_kernel_stats.csv)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
step=$1
shift
case "$step" in
  tests)
    K=()
    [ -n "$1" ] && K=(-k "$1")
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
      > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
    tail -3 gpurun_out/t.log ;;
  smoke)
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 \
      || { tail -20 gpurun_out/smoke.log; exit 1; }
    tail -2 gpurun_out/smoke.log ;;
  bench)
    timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err \
      || { tail -20 gpurun_out/bench.err; exit 1; }
    python -c "import json; d = json.load(open('gpurun_out/bench.json')); print(len(open('gpurun_out/bench.json').read()), 'bytes;', d['metric'], d['value'], d['ms_per_step'], d.get('roofline', {}).get('frac'))" ;;
  handoff)
    # the one-launch step's hand-off check build (tools/exp_handoff.py): VARIANT [SKEW]
    V=$1 S=${2:-0}
    timeout -k 10 400 python -u tools/exp_handoff.py run "$V" "$S" > "gpurun_out/handoff_${V}_s${S}.log" 2>&1 \
      || { tail -30 "gpurun_out/handoff_${V}_s${S}.log"; exit 1; }
    mkdir -p gpurun_out/profiles && cp "gpurun_out/handoff_${V}_s${S}.log" gpurun_out/profiles/
    tail -1 "gpurun_out/handoff_${V}_s${S}.log" ;;
  bounds128)
    timeout -k 10 600 python -u tools/exp_debug_bounds.py train128 > gpurun_out/bounds128.log 2>&1 \
      || { tail -30 gpurun_out/bounds128.log; exit 1; }
    echo "SGNN-BOUNDS lines: $(grep -c SGNN-BOUNDS gpurun_out/bounds128.log)"
    tail -3 gpurun_out/bounds128.log ;;
  profile)
    TAG=$1 WL=$2 MODE=$3
    shift 3
    D=gpurun_out/prof_$TAG
    rm -rf "$D"
    mkdir -p "$D"
    # trace mode first (the durations the roofline quotes), then one counter pass each
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/k" -o run -- \
      python3 bench.py "$@" > "$D/k.log" 2>&1 || { tail -20 "$D/k.log"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/f" -o run -- \
      python3 bench.py "$@" > "$D/f.log" 2>&1 || { tail -20 "$D/f.log"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/w" -o run -- \
      python3 bench.py "$@" > "$D/w.log" 2>&1 || { tail -20 "$D/w.log"; exit 1; }
    k=$(dirname "$(find "$D/k" -name run_kernel_stats.csv | head -1)")
    f=$(dirname "$(find "$D/f" -name run_counter_collection.csv | head -1)")
    w=$(dirname "$(find "$D/w" -name run_counter_collection.csv | head -1)")
    python3 profiles/summarize.py "$TAG" "$WL" "$k" "$f" "$w" "$MODE" && cp "$k/run_kernel_stats.csv" "profiles/${TAG}_kernel_stats.csv"
    mkdir -p gpurun_out/profiles && cp "profiles/${TAG}_summary.json" "profiles/${TAG}_kernel_stats.csv" gpurun_out/profiles/
    python3 - "$TAG" <<'PY'
import json, sys
d = json.load(open(f"profiles/{sys.argv[1]}_summary.json"))
rows = sorted(d["kernels"].items(), key=lambda kv: -kv[1].get("pct_time", 0))[:12]
for k, v in rows:
    print(k[:60].ljust(60), str(v.get("calls", "")).rjust(5), "%9.2f us" % v.get("avg_us", 0),
          "%7.1f%%" % v.get("pct_time", 0), "%10.3f MB" % (v.get("hbm_bytes", 0) / 1e6))
PY
    ;;
  *)
    echo "unknown step $step"; exit 2 ;;
esac
