# decoder: GPU tests, then throughput and kernel profile
O=gpurun_out/dec
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && \
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
cd "$GRAFT_REPO_ROOT" && for w in cfg2 cfg4; do \
  timeout -k 10 300 python scripts/dec_bench.py $w > $O/bench_$w.json 2> $O/bench_$w.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$w -o d -- python3 scripts/dec_bench.py $w > $O/kt_$w.log 2>&1 || exit 1; \
done
