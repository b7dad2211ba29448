# Round-3 ablation matrix of the exp/abl build (-DAIRS_ABLATE=1, enc_common.h DBG bits):
# cold (R=4) and warm (R=1) kbench of each mode, then per-segment timelines.
#   MODES="0 2 ..." WLS="cfg2" bash scripts/gpu_abl_r03.sh TAG
TAG=${1:-abl3}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && : > $O/abl.jsonl || exit 1
for w in ${WLS:-cfg2}; do for r in ${ROTS:-4 1}; do for m in ${MODES:-0 2}; do
  AIRS_KB_ROT=$r AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w >> $O/abl.jsonl 2>> $O/abl.err || { echo "mode $m failed"; tail -3 $O/abl.err; exit 1; }
done; done; done
for w in ${TSWLS:-}; do
  AIRS_KB_ROT=4 AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=$O/ts_$w.bin timeout -k 10 120 python scripts/kbench.py $w > $O/ts_$w.log 2>&1 || exit 1
done
cat $O/abl.jsonl
