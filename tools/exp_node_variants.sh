# Round-6 record: the node-phase / layer-transition variants of k_step16, each built
# from temporary defines (SGNN_AB_*; removed from step16.hip again) as sgnn_amd/_lib/libsgnn_hip_<variant>.so.
# Results: profiles/r06_node_phase_variants.txt.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/loc5
run() {  # lib case proc
  L=$PWD/sgnn_amd/_lib/libsgnn_hip_$1.so
  tag=$1_$(echo $2 | tr ' ,' '__')_p$3
  FILL=none SGNN_LIB=$L timeout -k 10 200 python -u tools/exp_localize.py $2 > gpurun_out/loc5/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/loc5/$tag.log; return 1; }
  echo "== $tag: $(grep '^rep [0-9]*:' gpurun_out/loc5/$tag.log | awk '{printf "%s ", $13}')"
}
C2="2 60,40 1.1 3 1 20 4"
for p in 1 2; do
  for lib in xz0 xzp xhalf; do
    run $lib "$C2" $p || exit 1
  done
done
timeout -k 10 900 python -u tools/exp_ab.py run xhalf,xrel,xacq,xbar,nob2,oldstage c1_r15,c1_r06,t4800 2 > gpurun_out/ab_fix.txt 2>&1; echo "ab rc $?"
