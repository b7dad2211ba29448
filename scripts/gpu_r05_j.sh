# Round 5: A/B timing of cfg2/cfg4 (exp/old, product, exp/pipe), then the default bench line
TAG=${1:-r05j}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2; do for w in cfg2 cfg4; do for lib in exp/old airs-compression_amd/lib exp/pipe; do
  AIRS_LIB=$lib/libairscmp.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-warm --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w $lib', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_def.json 2> $O/bench_def.err || { tail -5 $O/bench_def.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_def.json')); print('default', d['ms_per_step'], d['bitexact_vs_reference'], d.get('scaling_reference'))"
