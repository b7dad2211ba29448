# Round 4: histogram bin with a full-rate shift: AUTO tests and cfg3 bench (3 reps)
TAG=${1:-r04r}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_autorice.py tests/test_gpu_arena.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for w in cfg3 cfg4; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done
