# Final-tree check of the round: scripts/gpu_r03_round.sh (GPU suite, smoke,
# bench line of every workload, kernel traces, traffic), then the N > 1 bench
# path rehearsed with 2 gloo ranks on the one GPU (not a measurement).
#   bash scripts/gpu_r03_final.sh TAG
TAG=${1:-r03_final}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r03_round.sh $TAG || exit 1
AIRS_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-gather \
  > $O/rehearsal_n2.json 2> $O/rehearsal_n2.err || { tail -5 $O/rehearsal_n2.err; exit 1; }
cut -c1-300 $O/rehearsal_n2.json
