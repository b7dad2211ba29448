# fused auto-Rice + payload streams: parity tests, digests, bench cfg3 / cfg2s / cfg2 (cold), kernel stats
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/auto2 && export TMPDIR=/tmp || exit 1
O=gpurun_out/auto2
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_autorice.py tests/test_gpu_stream.py "tests/test_gpu_parity.py::test_config_digest_gpu" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -15 $O/pytest.log; exit 1; }
for w in ${WLS:-cfg3 cfg2s cfg2}; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['roofline']['avg_launch_ms_hip_events'], d['roofline']['frac'], d['bitexact_vs_reference'], d.get('warm',{}).get('avg_step_gpu_ms'), (d.get('cpu_baseline') or {}).get('value'))"
done
for w in cfg3 cfg2s; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$w -o kt -- python3 bench.py --workload $w --no-cpu-baseline --no-warm > $O/kt_$w.json 2> $O/kt_$w.err || exit 1
grep encode_kernel $O/kt_$w/kt_kernel_stats.csv | cut -c1-160
done
