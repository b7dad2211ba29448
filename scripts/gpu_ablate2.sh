# time + instruction counts per ablation mode (AIRS_DBG bits) of exp/abl
# (build: bash scripts/build_exp.sh abl "-DAIRS_ABLATE=1 -DAIRS_EXP_ONLY"); output is garbage
O=gpurun_out/abl2
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && export AIRS_LIB=exp/abl/libairscmp.so && : > $O/t.jsonl && \
for m in ${MODES:-0 32768 32 2048 2 8 4096}; do \
  AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py ${WL:-cfg2} >> $O/t.jsonl 2>> $O/err || exit 1; \
  AIRS_DBG=$m timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -d $O/m$m -o p -- python3 scripts/kbench.py ${WL:-cfg2} > $O/m$m.log 2>&1 || exit 1; \
done
