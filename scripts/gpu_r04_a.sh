# Round 4: GPU suite on the current tree, then an env A/B (scripts/gpu_envab.sh)
#   VARIANTS=... WLS=... bash scripts/gpu_r04_a.sh TAG
TAG=${1:-r04a}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log
# a failed test (rc 1) still lets the measurements run; anything else (a fault,
# an abort, a time limit) ends the call here
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head; [ $rc -eq 1 ]; } || exit $rc
bash scripts/gpu_envab.sh $TAG
for w in ${BENCH_WLS:-}; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  cut -c1-400 $O/bench_$w.json
done
