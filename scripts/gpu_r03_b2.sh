# drop-in probe (HIP log), walk parity after the two-piece escape fix,
# AUTO_RICE tests, then the KEEP_Q=0 / NIMG=2 occupancy A/B on cfg2, cfg4
O=gpurun_out/r03_b2
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
AMD_LOG_LEVEL=2 timeout -k 10 60 tests/dropin/host_probe > $O/probe.out 2> $O/probe.err; echo "probe rc=$?"; cat $O/probe.out; tail -c 3000 $O/probe.err
AMD_LOG_LEVEL=2 timeout -k 10 60 tests/dropin/simple_compression > $O/simple.out 2> $O/simple.err; echo "simple rc=$?"; head -c 600 $O/simple.out; tail -c 2000 $O/simple.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_autorice.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | cut -c1-200
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
VARIANTS="base kq0 kq0n2" WLS="cfg2 cfg4" REPS=2 bash scripts/gpu_ab.sh r03_b2/ab > /dev/null 2>&1 || { echo "A/B failed"; tail -5 $O/ab/ab.err; exit 1; }
cat $O/ab/ab.jsonl | cut -c1-220
