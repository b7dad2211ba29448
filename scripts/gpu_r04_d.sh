# Round 4: segment walk with 2048-sample segments (8 samples per lane) against
# 4096 (AIRS_WALK_SEG=4096): walk tests, timelines (ablation build), benches.
TAG=${1:-r04d}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_batch.py -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
AIRS_TS_SEG=2048 AIRS_LIB=exp/abl/libairscmp.so AIRS_WL=cfg5s8 timeout -k 10 200 python scripts/walk_ts.py $O/ts_cfg5s8_seg2048.json > $O/ts.log 2>&1 || { tail -5 $O/ts.log; exit 1; }
cat $O/ts_cfg5s8_seg2048.json | tr -d ' \n' | cut -c1-900; echo
AIRS_WALK_SEG=4096 AIRS_LIB=exp/abl/libairscmp.so AIRS_WL=cfg5s8 timeout -k 10 200 python scripts/walk_ts.py $O/ts_cfg5s8_seg4096.json > $O/ts2.log 2>&1 || { tail -5 $O/ts2.log; exit 1; }
cat $O/ts_cfg5s8_seg4096.json | tr -d ' \n' | cut -c1-900; echo
for rep in 1 2; do for v in 2048:: 4096::; do
  seg=${v%%:*}; lib=${v#*:}; lib=${lib%:}
  AIRS_LIB=$lib AIRS_WALK_SEG=$seg timeout -k 10 300 python bench.py --workload cfg5s8 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('cfg5s8 seg $seg lib ${lib:-product}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done
