#!/bin/bash
# usage: scripts/gpu_benchall.sh TAG [workloads...]
# pytest -m gpu, then bench.py for each workload (JSON under gpurun_out/),
# then one rocprofv3 --kernel-trace --stats pass per workload.
set -o pipefail
TAG=${1:-r02}; shift
WLS=${@:-cfg2 cfg3 cfg4 cfg5}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
for w in $WLS; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  cat $OUT/bench_$w.json
done
for w in $WLS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o run -- python3 bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-warm > $OUT/prof_$w.json 2> $OUT/prof_$w.err || { tail -20 $OUT/prof_$w.err; exit 1; }
done
find $OUT -name "*kernel_stats.csv" | head -20
