# Round 4: frame walk for AUTO (cfg3) and the segment walk after the
# prefetch fix: tests, cfg5s8 timeline (ablation build), A/B benches.
TAG=${1:-r04f}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_autorice.py tests/test_gpu_walk.py tests/test_gpu_batch.py -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AIRS_TS_SEG=2048 AIRS_LIB=exp/abl/libairscmp.so AIRS_WL=cfg5s8 timeout -k 10 200 python scripts/walk_ts.py $O/ts_cfg5s8_seg2048.json > $O/ts.log 2>&1 || { tail -5 $O/ts.log; exit 1; }
cat $O/ts_cfg5s8_seg2048.json | tr -d ' \n' | cut -c1-700; echo
for rep in 1 2; do for v in cfg3:AIRS_FAUTO=1 cfg3:AIRS_FAUTO=0 cfg5s8:AIRS_WALK_SEG=2048 cfg5s8:AIRS_WALK_SEG=4096; do
  w=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w $e', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done
