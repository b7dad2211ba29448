# Ablation matrix of the encode kernel (exp/abl build, -DAIRS_ABLATE=1): cold
# (AIRS_KB_ROT=4) and warm (1) kernel time per AIRS_DBG mode (enc_common.h DBG):
#   2 no look-back, 8 no tail rebuild, 32 no packing puts, 512 no HBM reads,
#   1024 no HBM writes, 2048 no image store-out, 4096 no image clears,
#   16384 empty kernel, 32768 stop after phase 1
# usage: LIB=exp/abl/libairscmp.so WLS="cfg2" MODES="0 2" bash scripts/gpu_ablate.sh TAG
TAG=${1:-abl}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && : > $O/abl.jsonl || exit 1
for w in ${WLS:-cfg2}; do for r in ${ROTS:-4 1}; do for m in ${MODES:-0 2 8 32 512 1024 2048 4096 16384 32768}; do
  AIRS_KB_ROT=$r AIRS_LIB=${LIB:-exp/abl/libairscmp.so} AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w >> $O/abl.jsonl 2>> $O/abl.err || exit 1
done; done; done
cat $O/abl.jsonl
