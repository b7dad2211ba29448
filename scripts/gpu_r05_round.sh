# Round 5 deliverable run: GPU suite, smoke, the bench line of every workload,
# then per workload a rocprofv3 kernel trace + stats and the FETCH_SIZE /
# WRITE_SIZE passes (separate runs) -> traffic of the dominant kernel.
#   bash scripts/gpu_r05_round.sh TAG [WORKLOADS...]
TAG=${1:-r05}
shift
WLS=${*:-cfg2 cfg2s cfg3 cfg4 cfg5 cfg5fb cfg5s8 cfg5fbs8}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
  tail -3 $O/pytest_gpu.log | cut -c1-200
  [ $rc -eq 0 ] || { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
kern() {
  case $1 in
    cfg2|cfg2s|cfg4) echo rice_kernel ;;
    cfg3) echo encode_kernel ;;
    cfg5|cfg5fb) echo walk_ctx_kernel ;;
    cfg5s8|cfg5fbs8) echo walk_kernel ;;
  esac
}
[ -n "$SKIP_BENCH" ] || for w in $WLS; do
  cpu=--no-cpu-baseline; [ "$w" = cfg2 ] && cpu=
  timeout -k 10 400 python bench.py --workload $w $cpu > $O/bench_$w.json 2> $O/bench_$w.err || { tail $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], d['value'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'], r.get('frac_samples_only'))"
done
[ -n "$SKIP_PROF" ] || for w in $WLS; do
  K=$(kern $w)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$w -o kt -- python3 bench.py --workload $w --no-cpu-baseline --no-warm > $O/kt_$w.log 2>&1 || { tail $O/kt_$w.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$w -o pf -- python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-warm > $O/pf_$w.log 2>&1 || { tail -3 $O/pf_$w.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pw_$w -o pw -- python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-warm > $O/pw_$w.log 2>&1 || { tail -3 $O/pw_$w.log; exit 1; }
  python3 scripts/traffic.py $O/pf_$w/pf_results.db $O/pw_$w/pw_results.db $w $O/traffic_$w.json --kernel $K > $O/traffic_$w.log 2>&1 || { tail -3 $O/traffic_$w.log; exit 1; }
  cut -c1-300 $O/traffic_$w.json
done
if [ -n "$AUTO_TRACE" ]; then
  # CMP_GPU_AUTO_RICE on cfg2-shaped frames (4 Mi samples, above the fused limit): the sliced selection's
  # grid (select_rice_hist_kernel: one workgroup per 32 Ki-sample slice, 2048 > 16 frames)
  AIRS_KB_AUTO=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_auto4mi -o kt -- python3 scripts/kbench.py cfg2 > $O/kt_auto4mi.log 2>&1 || { tail $O/kt_auto4mi.log; exit 1; }
  tail -1 $O/kt_auto4mi.log
fi
find $O -name "*.db" -delete
