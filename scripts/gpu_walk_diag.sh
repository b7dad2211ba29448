# walk kernel diagnosis: all walk/drop-in tests (no -x), the differing frames
# of the failing trials, then the cfg5 bench + kernel trace
O=gpurun_out/${1:-walkdiag}
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_dropin.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_walk.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_walk.log | cut -c1-200
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -u scripts/walk_diag.py 3 9 > $O/diag.jsonl 2> $O/diag.err || { tail -20 $O/diag.err; exit 1; }
cut -c1-1500 $O/diag.jsonl
timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
cut -c1-600 $O/bench_cfg5.json
