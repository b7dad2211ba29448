# GPU tests + kernel timings (modes: AIRS_DBG values) on cfg2 and cfg4
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/quick.jsonl && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
for m in ${MODES:-0 2}; do for w in ${WLS:-cfg2 cfg4}; do \
  AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/quick.jsonl 2>> gpurun_out/quick.err || exit 1; \
done; done
