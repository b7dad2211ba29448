# full GPU suite on the product library (model update rework, checksum fix),
# the cfg5 bench, then the walk timeline on the ablation build
O=gpurun_out/r03_b4
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | cut -c1-200 | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print('cfg5', d['ms_per_step'], d['value'], d['bitexact_vs_reference'], d['roofline']['avg_launch_ms_hip_events'])"
AIRS_LIB=exp/abl/libairscmp.so timeout -k 10 300 python3 -u scripts/walk_ts.py $O/walk_ts.json > $O/walk_ts.log 2>&1 || { tail -20 $O/walk_ts.log; exit 1; }
cat $O/walk_ts.json
