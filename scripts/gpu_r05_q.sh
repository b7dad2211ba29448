# Round 5: Rice kernel A/B against the committed tree (exp/head): parity (rice + stream tests), cfg2 cfg4 cfg2s
TAG=${1:-r05q}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_rice.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for w in cfg2 cfg4 cfg2s; do for lib in exp/head airs-compression_amd/lib; do
  AIRS_LIB=$lib/libairscmp.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-warm --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w $lib', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
