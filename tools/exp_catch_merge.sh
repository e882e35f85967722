# Round-5 experiment: how often the merged two-sub-tile node phase fails the 3D two-example case
# (tools/exp_localize.py, 10 launches each, e0 region NaN-filled between launches), per library.
for lib in "$@"; do
  FILL=e0 SGNN_LIB=$PWD/sgnn_amd/_lib/libsgnn_hip_$lib.so timeout -k 10 300 python -u tools/exp_localize.py 3 16,16,12 0.75 2 3 20 10 > gpurun_out/loc_$lib.log 2>&1 || exit 1
  echo "== $lib: $(grep -c 'bad particles 0 ' gpurun_out/loc_$lib.log) of 10 launches clean"
done
