# cold (rotated buffers) vs warm kernel timings of exp variants and ablation modes
# VARIANTS="A" MODES="0 2 32768" WLS="cfg2 cfg4" ROTS="1 4" bash scripts/gpu_cold.sh
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/exp.jsonl && \
for v in ${VARIANTS:-A}; do for m in ${MODES:-0}; do for w in ${WLS:-cfg2 cfg4}; do for r in ${ROTS:-1 4}; do \
  echo "{\"variant\": \"$v\"}" >> gpurun_out/exp.jsonl; \
  AIRS_KB_ROT=$r AIRS_LIB=exp/$v/libairscmp.so AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/exp.jsonl 2>> gpurun_out/exp.err || exit 1; \
done; done; done; done
