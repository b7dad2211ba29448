# Round 4: which part of the segment walk's frame epilogue costs: product, no final bytes (exp/ne1), no header words (exp/ne2)
TAG=${1:-r04ab}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2 3; do for lib in "" exp/ne1/libairscmp.so exp/ne2/libairscmp.so; do
  AIRS_LIB=$lib timeout -k 10 300 python bench.py --workload cfg5s8 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('cfg5s8 ${lib:-prod}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done
