# Round 4: context walk identifier draws deferred (product) against the previous build (exp/prev)
TAG=${1:-r04ae}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_batch.py tests/test_gpu_autorice.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for w in cfg5fb; do for lib in "" exp/prev/libairscmp.so; do
  AIRS_LIB=$lib timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w ${lib:-defer}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
