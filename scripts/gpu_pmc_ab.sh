# PMC comparison of exp variants on one workload: usage VARIANTS="a b" WL=cfg4 bash gpu_pmc_ab.sh
O=gpurun_out/pmcab
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && \
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 ; \
for v in ${VARIANTS:-r1 lean}; do \
  AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d $O/$v -o p -- python3 scripts/kbench.py ${WL:-cfg4} > $O/$v.log 2>&1 || exit 1; \
done
