# Round 5: enc_rice at five workgroups per CU: A/B, ablation matrix, timeline, rocprof kernel stats
TAG=${1:-r05d}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for rep in 1 2; do for w in cfg2 cfg4; do for lib in "" exp/old exp/wpe4; do
  L=${lib:+$lib/libairscmp.so}
  AIRS_LIB=$L timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('$w ${lib:-prod}', d['ms_per_step'], d['bitexact_vs_reference'], r['avg_launch_ms_hip_events'], r['frac'])"
done; done; done
for m in 0 2 32 34 2048 32768; do
  AIRS_KB_ROT=4 AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py cfg2 >> $O/abl.jsonl 2>> $O/abl.err || { tail -3 $O/abl.err; exit 1; }
done
cat $O/abl.jsonl
AIRS_KB_ROT=4 AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=$O/ts_abl_cfg2.bin timeout -k 10 120 python scripts/kbench.py cfg2 > $O/ts.log 2>&1 || exit 1
for lib in prod old; do
  L=$([ $lib = old ] && echo exp/old/libairscmp.so)
  AIRS_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$lib -o run -- python bench.py --workload cfg2 --no-cpu-baseline --steps 20 --warmup 5 > $O/prof_$lib.log 2>&1 || { tail -5 $O/prof_$lib.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | head
