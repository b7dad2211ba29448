# Round 4: encode kernel without the frame header writes (ablation exp/nohdr, output incomplete) against the product
TAG=${1:-r04ah}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2; do for w in cfg4 cfg3 cfg2; do for lib in "" exp/nohdr/libairscmp.so; do
  AIRS_LIB=$lib timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w ${lib:-prod}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
