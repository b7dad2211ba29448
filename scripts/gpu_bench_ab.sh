# Interleaved A/B of experiment builds through bench.py (cold rotation):
#   VARIANTS="a b" WLS="cfg2 cfg4" REPS=2 bash scripts/gpu_bench_ab.sh TAG
# one JSON line per run: variant, workload, kernel ms per step (HIP events), bit-exactness
TAG=${1:-bab}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && : > $O/ab.jsonl || exit 1
for rep in $(seq ${REPS:-2}); do for w in ${WLS:-cfg2}; do for v in ${VARIANTS:-base}; do
  AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --no-warm --steps 20 > $O/one.json 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/one.json')); print(json.dumps(dict(variant='$v', rep=$rep, workload='$w', kernel_ms=d['roofline']['avg_launch_ms_hip_events'], frac=d['roofline']['frac'], bitexact=d['bitexact_vs_reference'])))" >> $O/ab.jsonl
done; done; done
cat $O/ab.jsonl
