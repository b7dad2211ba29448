# Round 4: cfg5 on the context walk against the segment walk (AIRS_WALK_CTX=0, per segment size)
TAG=${1:-r04k}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2; do for v in X=1 AIRS_WALK_CTX=0,AIRS_WALK_SEG=4096 AIRS_WALK_CTX=0,AIRS_WALK_SEG=2048; do
  e=$(echo $v | tr ',' ' ')
  env $e timeout -k 10 300 python bench.py --workload cfg5 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('cfg5 $v', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'], r.get('frac_samples_only'))"
done; done
