# Round 4: encode kernel header in three stores (product) against the five-store build (exp/prev) and no header (exp/nohdr)
TAG=${1:-r04ai}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for w in cfg4 cfg3 cfg2; do for lib in "" exp/nohdr/libairscmp.so exp/prev/libairscmp.so; do
  AIRS_LIB=$lib timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w ${lib:-prod}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
