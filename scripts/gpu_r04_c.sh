# Round 4: after the store-hazard fix: the walk-fallback diagnostic, the
# walk/arena/AUTO GPU tests, the segment-walk timeline of cfg5s8 (ablation
# build exp/abl), bench lines.
TAG=${1:-r04c}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 250 python exp/diag_walkfb.py u16 > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
grep -E "^bad|state" $O/diag.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_walk.py tests/test_gpu_arena.py \
  tests/test_gpu_autorice.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AIRS_LIB=exp/abl/libairscmp.so AIRS_WL=cfg5s8 timeout -k 10 200 python scripts/walk_ts.py $O/ts_cfg5s8.json > $O/ts.log 2>&1 || { tail -5 $O/ts.log; exit 1; }
cat $O/ts_cfg5s8.json | tr -d ' \n' | cut -c1-1500; echo
AIRS_TS_SEG=2048 AIRS_LIB=exp/abl2/libairscmp.so AIRS_WL=cfg5s8 timeout -k 10 200 python scripts/walk_ts.py $O/ts_cfg5s8_dw2.json > $O/ts2.log 2>&1 || { tail -5 $O/ts2.log; exit 1; }
cat $O/ts_cfg5s8_dw2.json | tr -d ' \n' | cut -c1-1500; echo
for w in ${BENCH_WLS:-cfg5s8 cfg2 cfg3}; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['value'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'], r.get('frac_samples_only'))"
done
AIRS_LIB=exp/dw2/libairscmp.so timeout -k 10 300 python bench.py --workload cfg5s8 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_cfg5s8_dw2.json 2> $O/bench_cfg5s8_dw2.err || { tail -5 $O/bench_cfg5s8_dw2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5s8_dw2.json')); r=d['roofline']; print('cfg5s8-dw2', d['ms_per_step'], d['value'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
