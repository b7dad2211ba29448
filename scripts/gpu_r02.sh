# Round deliverable on the GPU box, every BASELINE workload:
#   smoke, pytest -m gpu, bench.py per workload (cold rotated inputs + warm),
#   rocprofv3 --kernel-trace --stats per workload, FETCH_SIZE / WRITE_SIZE
#   passes per workload -> traffic json.
# usage: bash scripts/gpu_r02.sh TAG [workloads...]   (SKIP_TESTS=1 to skip pytest)
TAG=${1:-r02}; shift
WLS=${@:-cfg2 cfg2s cfg3 cfg4 cfg5 cfg5fb}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
for w in $WLS; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  cut -c1-400 $O/bench_$w.json
done
for w in $WLS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$w -o kt -- python3 bench.py --workload $w --no-cpu-baseline --no-warm > $O/kt_$w.json 2> $O/kt_$w.err || { tail -20 $O/kt_$w.err; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$w -o pf -- python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-warm > $O/pf_$w.log 2>&1 || { tail -20 $O/pf_$w.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw_$w -o pw -- python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-warm > $O/pw_$w.log 2>&1 || { tail -20 $O/pw_$w.log; exit 1; }
  python3 scripts/traffic.py $O/pf_$w/pf_results.db $O/pw_$w/pw_results.db $w $O/traffic_$w.json > $O/traffic_$w.log 2>&1 || cat $O/traffic_$w.log
done
find $O -name "*kernel_stats.csv"
