# walk kernel: its parity tests, then cfg5 bench (cold) + kernel trace
O=gpurun_out/${1:-walk}
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_walk.log 2>&1; rc=$?
tail -15 $O/pytest_walk.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
cut -c1-600 $O/bench_cfg5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cfg5 -o kt -- python3 bench.py --workload cfg5 --no-cpu-baseline --no-warm > $O/kt_cfg5.json 2> $O/kt_cfg5.err || { tail -20 $O/kt_cfg5.err; exit 1; }
find $O -name "*kernel_stats.csv" | xargs cat | cut -c1-200
