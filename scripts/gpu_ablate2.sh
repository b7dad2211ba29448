# time + VALU count per ablation mode (AIRS_DBG bits; output is garbage for bits 8..64)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abl2 && export TMPDIR=/tmp && : > gpurun_out/abl2/t.jsonl && \
for m in ${MODES:-2 10 18 34 66 50 122}; do \
  AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py cfg2 >> gpurun_out/abl2/t.jsonl 2>> gpurun_out/abl2/err || exit 1; \
  AIRS_DBG=$m timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES -d gpurun_out/abl2/m$m -o p -- python3 scripts/kbench.py cfg2 > gpurun_out/abl2/m$m.log 2>&1 || exit 1; \
done
