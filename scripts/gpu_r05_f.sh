# Round 5: enc_rice workgroup geometry (256 x 4 / 5 per CU, 512 x 2 / 3 per CU) against encode_kernel (exp/old)
TAG=${1:-r05f}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2 3; do for w in cfg2 cfg4; do for lib in exp/old exp/w256x4 exp/w256x5 exp/w512x2 exp/w512x3; do
  AIRS_LIB=$lib/libairscmp.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w $lib', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
