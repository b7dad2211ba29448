# Round 5: per-segment timelines (ablation builds) of enc_rice (exp/abl) and encode_kernel (exp/ablold), cold
TAG=${1:-r05c}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for lib in abl ablold; do for w in cfg2 cfg4; do
  AIRS_KB_ROT=4 AIRS_LIB=exp/$lib/libairscmp.so AIRS_DBG=0 timeout -k 10 120 python scripts/kbench.py $w >> $O/kb.jsonl 2>> $O/kb.err || { tail -3 $O/kb.err; exit 1; }
  AIRS_KB_ROT=4 AIRS_LIB=exp/$lib/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=$O/ts_${lib}_$w.bin timeout -k 10 120 python scripts/kbench.py $w > $O/ts_${lib}_$w.log 2>&1 || { tail -3 $O/ts_${lib}_$w.log; exit 1; }
done; done
cat $O/kb.jsonl
