# Round 5: timelines of the persistent Rice kernel (ablation build exp/ablp, exclusive engine) and the
# one-segment-per-workgroup kernel (exp/abl), cold, cfg2 and cfg4
TAG=${1:-r05u}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for w in cfg2 cfg4; do
  AIRS_KB_EXCL=1 AIRS_KB_ROT=4 AIRS_LIB=exp/ablp/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=$O/tsp_$w.bin timeout -k 10 120 python scripts/kbench.py $w > $O/kbp_$w.json 2> $O/kbp_$w.err || { tail -3 $O/kbp_$w.err; exit 1; }
  cat $O/kbp_$w.json
done
