cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && \
for w in cfg2; do \
AIRS_DBG=2 timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/prof2_pmc1 -o p1 -- python3 scripts/kbench.py $w > gpurun_out/prof2_pmc1.log 2>&1 && \
AIRS_DBG=2 timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/prof2_pmc2 -o p2 -- python3 scripts/kbench.py $w > gpurun_out/prof2_pmc2.log 2>&1 ; done
