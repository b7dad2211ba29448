# full GPU suite, then cfg5 with the fallback enabled: device state machine vs the host-stepped path
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/fb2 && export TMPDIR=/tmp || exit 1
O=gpurun_out/fb2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --workload cfg5fb --steps 10 --warmup 2 > $O/bench_cfg5fb.json 2> $O/bench_cfg5fb.err || { tail -20 $O/bench_cfg5fb.err; exit 1; }
AIRS_HOST_EXACT=1 timeout -k 10 300 python -u bench.py --workload cfg5fb --steps 3 --warmup 1 --no-cpu-baseline --no-warm > $O/bench_cfg5fb_host.json 2> $O/bench_cfg5fb_host.err || { tail -20 $O/bench_cfg5fb_host.err; exit 1; }
for f in bench_cfg5fb bench_cfg5fb_host; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['bitexact_vs_reference'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cfg5fb -o kt -- python3 bench.py --workload cfg5fb --steps 10 --warmup 2 --no-cpu-baseline --no-warm > $O/kt.json 2> $O/kt.err || exit 1
cut -d, -f1-4 $O/kt_cfg5fb/kt_kernel_stats.csv | cut -c1-150
