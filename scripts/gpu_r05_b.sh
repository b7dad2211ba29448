# Round 5: enc_rice variants (look-back point, scalar round size, occupancy) against encode_kernel (exp/old)
TAG=${1:-r05b}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2; do for w in cfg2 cfg4; do for lib in "" exp/old exp/lbc2 exp/lbc0 exp/slb32 exp/wpe4 exp/lbc2wpe4; do
  L=${lib:+$lib/libairscmp.so}
  AIRS_LIB=$L timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w ${lib:-prod}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
