# Round 5: per-segment timelines of the Rice kernel (ablation build, AIRS_DBG 65536), cold, cfg2 and cfg4
TAG=${1:-r05s}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp || exit 1
for w in cfg2 cfg4; do
  AIRS_KB_ROT=4 AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=$O/ts_$w.bin timeout -k 10 120 python scripts/kbench.py $w > $O/kb_$w.json 2> $O/kb_$w.err || { tail -3 $O/kb_$w.err; exit 1; }
  cat $O/kb_$w.json
done
