# Round deliverable run: full GPU suite, smoke, bench line of every workload,
# rocprofv3 kernel trace + stats (cfg2, cfg5), FETCH_SIZE / WRITE_SIZE passes
# -> traffic (cfg2, cfg5).  usage: bash scripts/gpu_r03_round.sh TAG
TAG=${1:-r03}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log | cut -c1-200
[ $rc -eq 0 ] || { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail $O/bench_cfg2.err; exit 1; }
for w in cfg2s cfg3 cfg4 cfg5 cfg5fb; do
  timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail $O/bench_$w.err; exit 1; }
done
for w in cfg2 cfg2s cfg3 cfg4 cfg5 cfg5fb; do
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['value'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'], r.get('frac_samples_only'))"
done
for w in cfg2 cfg5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$w -o kt -- python3 bench.py --workload $w --no-cpu-baseline --no-warm > $O/kt_$w.log 2>&1 || { tail $O/kt_$w.log; exit 1; }
done
K2=encode_kernel; K5=walk_ctx_kernel
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf2 -o pf -- python3 bench.py --workload cfg2 --steps 5 --warmup 1 --no-cpu-baseline --no-warm > $O/pf2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pw2 -o pw -- python3 bench.py --workload cfg2 --steps 5 --warmup 1 --no-cpu-baseline --no-warm > $O/pw2.log 2>&1 && \
python3 scripts/traffic.py $O/pf2/pf_results.db $O/pw2/pw_results.db cfg2 $O/traffic_cfg2.json --kernel $K2 > $O/traffic2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf5 -o pf -- python3 bench.py --workload cfg5 --steps 5 --warmup 1 --no-cpu-baseline --no-warm > $O/pf5.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pw5 -o pw -- python3 bench.py --workload cfg5 --steps 5 --warmup 1 --no-cpu-baseline --no-warm > $O/pw5.log 2>&1 && \
python3 scripts/traffic.py $O/pf5/pf_results.db $O/pw5/pw_results.db cfg5 $O/traffic_cfg5.json --kernel $K5 > $O/traffic5.log 2>&1 || { echo "traffic failed"; tail -3 $O/traffic*.log; exit 1; }
cat $O/traffic_cfg2.json $O/traffic_cfg5.json | cut -c1-400
find $O -name "*.db" -delete
