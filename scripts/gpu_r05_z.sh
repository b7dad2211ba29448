# Round 5: rehearse the N > 1 bench path (two ranks on the box's one GPU, gloo), with the gather
TAG=${1:-r05z}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
AIRS_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
cat $O/n2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['n_gpus'], d['value'], d['ms_per_step'], d['bitexact_vs_reference'], d.get('scaling_reference'), d.get('gather', {}).get('bitexact_vs_reference'))"
