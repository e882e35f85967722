# The shipping one-launch step on a cold GPU: the first processes of a gpurun call run the two-sub-tile
# oracle cases of tests/test_gpu_step.py (tools/exp_localize.py, 10 launches each, e0 / node-half regions
# NaN-filled between launches), one line per process with the launches that failed.
for fill in e0 uv; do
  for case in "3 16,16,12 0.75 2 3 20" "2 90,40 15.0 2 1 20" "2 120,40 0.6 1 1 20" "2 200,40 0.6 1 1 20"; do
    FILL=$fill timeout -k 10 300 python -u tools/exp_localize.py $case 10 > gpurun_out/cold.log 2>&1 || exit 1
    echo "FILL=$fill case [$case]: failing launches [$(grep '^rep [0-9]*:' gpurun_out/cold.log | grep -v 'bad particles 0 ' | awk '{print $2}' | tr -d ':' | tr '\n' ' ')]"
  done
done
