# VALU/SALU/LDS instruction counts per AIRS_DBG ablation mode: V=variant MODES="0 32768" WL=cfg2
O=gpurun_out/pmcm
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && \
for m in ${MODES:-0 32768 32 2048 2}; do \
  AIRS_DBG=$m AIRS_LIB=exp/${V:-K1abl}/libairscmp.so timeout -k 10 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $O/m$m -o p -- python3 scripts/kbench.py ${WL:-cfg2} > $O/m$m.log 2>&1 || exit 1; \
done
