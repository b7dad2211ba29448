cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && : > gpurun_out/ablate.jsonl && \
for m in 0 4 2 6; do for w in cfg2 cfg4; do \
  AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/ablate.jsonl 2>> gpurun_out/ablate.err || exit 1; \
done; done
