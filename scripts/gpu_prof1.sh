cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 ; \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt -- python3 scripts/kbench.py cfg2 > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/prof_pmc1 -o p1 -- python3 scripts/kbench.py cfg2 > gpurun_out/prof_pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d gpurun_out/prof_pmc2 -o p2 -- python3 scripts/kbench.py cfg2 > gpurun_out/prof_pmc2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_pmc3 -o p3 -- python3 scripts/kbench.py cfg2 > gpurun_out/prof_pmc3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_pmc4 -o p4 -- python3 scripts/kbench.py cfg2 > gpurun_out/prof_pmc4.log 2>&1
