# GPU suite + cfg5/cfg5fb benches
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/q5 && export TMPDIR=/tmp || exit 1
O=gpurun_out/q5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for w in ${WLS:-cfg5 cfg5fb}; do
timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d['bitexact_vs_reference'], d.get('warm',{}).get('avg_step_gpu_ms'))"
done
