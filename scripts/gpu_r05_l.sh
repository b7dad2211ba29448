# Round 5: the speculative segment walk for fallback batches: tests, then cfg5s8 / cfg5fbs8 benches
TAG=${1:-r05l}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for w in cfg5s8 cfg5fbs8; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-warm --steps 20 --warmup 5 > $O/bench_$w.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done
