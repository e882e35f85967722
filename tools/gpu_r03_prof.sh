# Round 3: SQ counters of the step kernel (one pass per counter group) + the phase probe.
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 5 90 rocprofv3 --list-avail > $R/gpurun_out/avail.txt 2>&1 || true
cd $R
P="python bench.py --no-extras --cpu-steps 0 --steps 20 --warmup 5"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/pmc/p1 -o p1 --output-format csv -- $P > gpurun_out/pmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT -d gpurun_out/pmc/p2 -o p2 --output-format csv -- $P > gpurun_out/pmc/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_LDS -d gpurun_out/pmc/p3 -o p3 --output-format csv -- $P > gpurun_out/pmc/p3.log 2>&1
echo "pmc rc $?"
tail -3 gpurun_out/pmc/p1.log gpurun_out/pmc/p2.log gpurun_out/pmc/p3.log
