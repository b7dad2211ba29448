# Round 5: where cfg5fbs8's step goes (kernel + copy trace)
TAG=${1:-r05m}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o run -- python3 bench.py --workload cfg5fbs8 --no-cpu-baseline --no-warm --steps 10 --warmup 2 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
ls -R $O/prof | head -20
