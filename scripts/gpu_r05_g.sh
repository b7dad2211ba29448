# Round 5: enc_rice ablations (ablation builds, 5 and 4 workgroups per CU): cfg2 / cfg4 cold,
# modes 0 kernel, 2 no look-back, 512 no HBM reads, 514 neither, 32768 phase 1 only, 2048 no stores
TAG=${1:-r05g}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && : > $O/abl.jsonl || exit 1
for lib in abl abl4; do for w in cfg2 cfg4; do for m in 0 2 512 514 32768 2048; do
  AIRS_KB_ROT=4 AIRS_LIB=exp/$lib/libairscmp.so AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w > $O/one.json 2>> $O/abl.err || { tail -3 $O/abl.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/one.json')); print('$lib', d['workload'], d['dbg'], round(d['median_ms']*1e3,1), round(d['min_ms']*1e3,1))" | tee -a $O/abl.jsonl
done; done; done
