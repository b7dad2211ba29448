# Round 4: segment walk tests, timelines (ablation build) and benches per segment size and ticket mode
TAG=${1:-r04i}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_batch.py -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
for seg in 4096 2048; do
  AIRS_WALK_SEG=$seg AIRS_TS_SEG=$seg AIRS_LIB=exp/abl/libairscmp.so AIRS_WL=cfg5s8 timeout -k 10 200 python scripts/walk_ts.py $O/ts_cfg5s8_seg$seg.json > $O/ts.log 2>&1 || { tail -5 $O/ts.log; exit 1; }
  cat $O/ts_cfg5s8_seg$seg.json | tr -d ' \n' | cut -c1-500; echo
done
for rep in 1 2; do for v in cfg5s8:AIRS_WALK_SEG=4096 cfg5s8:AIRS_WALK_SEG=2048 cfg5s8:AIRS_WALK_SEG=4096,AIRS_WALK_TICKET=1; do
  w=${v%%:*}; e=$(echo ${v#*:} | tr ',' ' ')
  env $e timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w $e', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'], r.get('frac_samples_only'))"
done; done
