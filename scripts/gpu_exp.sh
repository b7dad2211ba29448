# kernel timings for alternative builds exp/<V>/libairscmp.so (AIRS_LIB override)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/exp.jsonl && \
for v in ${VARIANTS:-A B C}; do for m in ${MODES:-0 2}; do for w in ${WLS:-cfg2 cfg4}; do \
  echo "{\"variant\": \"$v\"}" >> gpurun_out/exp.jsonl; \
  AIRS_LIB=exp/$v/libairscmp.so AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/exp.jsonl 2>> gpurun_out/exp.err || exit 1; \
done; done; done
