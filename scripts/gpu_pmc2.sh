# two PMC passes per exp variant on one workload: VARIANTS="A B" WL=cfg2 bash gpu_pmc2.sh
O=gpurun_out/pmc2
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && \
for v in ${VARIANTS:-A B}; do \
  AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $O/${v}_1 -o p -- python3 scripts/kbench.py ${WL:-cfg2} > $O/${v}_1.log 2>&1 || exit 1; \
  AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC -d $O/${v}_2 -o p -- python3 scripts/kbench.py ${WL:-cfg2} > $O/${v}_2.log 2>&1 || exit 1; \
done
