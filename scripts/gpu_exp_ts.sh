# kernel timings of exp variants (VARIANTS) then debug timelines of ablation builds (TSV)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ts && export TMPDIR=/tmp && : > gpurun_out/exp.jsonl && \
for v in ${VARIANTS}; do for w in ${WLS:-cfg2 cfg4}; do \
  echo "{\"variant\": \"$v\"}" >> gpurun_out/exp.jsonl; \
  AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/exp.jsonl 2>> gpurun_out/exp.err || exit 1; \
done; done && \
for v in ${TSV}; do for w in ${WLS:-cfg2 cfg4}; do \
  AIRS_LIB=exp/$v/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=gpurun_out/ts/${v}_$w.bin timeout -k 10 120 python scripts/kbench.py $w > gpurun_out/ts/${v}_$w.log 2>&1 || exit 1; \
done; done
