# Round 4: walk-fb read-back through page-locked memory (one copy, no final sync)
TAG=${1:-r04h}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_walk.py tests/test_gpu_cli.py -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2; do for w in cfg5fb cfg5; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_$w.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'], r.get('frac_samples_only'))"
done; done
