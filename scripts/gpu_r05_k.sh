# Round 5: 512-thread rice workgroups (32 Ki-sample segments): parity, then A/B cfg2/cfg4 against the product
TAG=${1:-r05k}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
AIRS_LIB=exp/w512/libairscmp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_rice.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_w512.log 2>&1
rc=$?; tail -2 $O/pytest_w512.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for w in cfg2 cfg4; do for lib in exp/old airs-compression_amd/lib exp/w512; do
  AIRS_LIB=$lib/libairscmp.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-warm --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w $lib', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
