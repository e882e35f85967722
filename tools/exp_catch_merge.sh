# Round-5 experiment: how often the merged two-sub-tile node phase fails the 3D two-example case
# (tools/exp_localize.py, 10 launches per process, the e0 region NaN-filled between launches unless
# FILL=none), libraries alternated over ROUNDS rounds; one line per process: the launches that failed.
ROUNDS=${ROUNDS:-3}
for r in $(seq $ROUNDS); do
  for lib in "$@"; do
    FILL=${FILL:-e0} SGNN_LIB=$PWD/sgnn_amd/_lib/libsgnn_hip_$lib.so timeout -k 10 300 python -u tools/exp_localize.py 3 16,16,12 0.75 2 3 20 10 > gpurun_out/loc_$lib.log 2>&1 || exit 1
    echo "round $r $lib: failing launches [$(grep '^rep [0-9]*:' gpurun_out/loc_$lib.log | grep -v 'bad particles 0 ' | awk '{print $2}' | tr -d ':' | tr '\n' ' ')]"
  done
done
