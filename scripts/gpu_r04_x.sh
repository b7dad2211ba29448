# Round 4: segment walk look-back loads before the frame epilogue (product) against the previous build (exp/prev)
TAG=${1:-r04x}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_batch.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
AIRS_TS_SEG=2048 AIRS_LIB=exp/abl/libairscmp.so AIRS_WL=cfg5s8 timeout -k 10 200 python scripts/walk_ts.py $O/ts.json > $O/ts.log 2>&1 || { tail -5 $O/ts.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/ts.json')); [print(k, d[k]) for k in ('kernel_span_us','block_start_us','block_life_us','life_by_segment_us','end_by_stream_us')]"
for rep in 1 2 3; do for lib in "" exp/prev/libairscmp.so; do
  AIRS_LIB=$lib timeout -k 10 300 python bench.py --workload cfg5s8 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('cfg5s8 ${lib:-epi}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done
