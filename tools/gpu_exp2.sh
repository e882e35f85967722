set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-rollout-extras > gpurun_out/b.json 2>gpurun_out/b.err
python -c "import json;d=json.load(open('gpurun_out/b.json'));print('train', d['ms_per_step'], d['value'], d['kernel_avg_us'])"
for wl in c1_r15 c2 c4; do
timeout -k 10 300 python bench.py --mode rollout --workload $wl --steps 40 --warmup 3 --cpu-steps 0 > gpurun_out/r_$wl.json
python -c "import json;d=json.load(open('gpurun_out/r_$wl.json'));print('$wl', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d['roofline']['frac'])"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_c2r -o run -- python3 bench.py --mode rollout --workload c2 --steps 10 --warmup 2 --cpu-steps 0 > /dev/null 2> gpurun_out/st.err
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_c2t -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-steps 0 --no-rollout-extras > /dev/null 2> gpurun_out/st.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_c2 -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-steps 0 --no-rollout-extras > /dev/null 2> gpurun_out/pmc.err
python tools/pmc_summary.py gpurun_out/pmc_c2 k_ > gpurun_out/pmc_c2.txt
echo pmc done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_c1r -o run -- python3 bench.py --mode rollout --workload c1_r15 --steps 20 --warmup 2 --cpu-steps 0 > /dev/null 2> gpurun_out/st.err
