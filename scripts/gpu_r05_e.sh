# Round 5: enc_rice with the early look-back window: A/B (5 and 4 workgroups per CU), timeline
TAG=${1:-r05e}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2 3; do for w in cfg2 cfg4; do for lib in "" exp/old exp/wpe4 exp/noearly; do
  L=${lib:+$lib/libairscmp.so}
  AIRS_LIB=$L timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w ${lib:-prod}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
AIRS_KB_ROT=4 AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=$O/ts_abl_cfg2.bin timeout -k 10 120 python scripts/kbench.py cfg2 > $O/ts.log 2>&1 || exit 1
