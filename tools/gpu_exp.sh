set -e
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_c2 -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-steps 0 --no-rollout-extras > /dev/null 2> gpurun_out/pmc.err
echo pmc done
