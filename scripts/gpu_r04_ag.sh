# Round 4: cfg5s8 segment size after the deferred epilogues: default (2048 samples, 8 per lane) against AIRS_WALK_SEG=4096
TAG=${1:-r04ag}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2 3; do for seg in "" 4096; do
  AIRS_WALK_SEG=$seg timeout -k 10 300 python bench.py --workload cfg5s8 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('cfg5s8 seg=${seg:-default}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done
