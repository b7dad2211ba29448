# context walk: walk parity tests, cfg5 bench + kernel trace
O=gpurun_out/r03_b5
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_walk.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_walk.log | cut -c1-200 | tail -16
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print('cfg5', d['ms_per_step'], d['value'], d['bitexact_vs_reference'], d['roofline']['avg_launch_ms_hip_events'], d.get('warm'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --workload cfg5 --no-cpu-baseline --no-warm > $O/kt.json 2> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" | xargs cat | cut -c1-220
