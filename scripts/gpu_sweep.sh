# Timing sweep over AIRS_DBG ablation modes (kbench; output is garbage for
# most modes) plus PMC passes for mode 0.  usage: gpu_sweep.sh TAG [WORKLOAD]
TAG=${1:-sw}; W=${2:-cfg2}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && : > $O/t.jsonl && \
for m in ${MODES:-0 2 32 512 1024 32768 16384 64 2048 544 1536}; do \
  AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $W >> $O/t.jsonl 2>> $O/err || exit 1; \
done && \
bash scripts/gpu_prof2.sh $TAG/pmc 0 $W
