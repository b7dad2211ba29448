# cold/warm ablation modes and debug timelines of the exp/abl build (-DAIRS_ABLATE=1)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ts && export TMPDIR=/tmp && : > gpurun_out/abl.jsonl || exit 1
for w in ${WLS:-cfg2 cfg4}; do for r in 1 4; do for m in ${MODES:-0 2 1024 32768 512 3}; do
  AIRS_KB_ROT=$r AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=$m timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/abl.jsonl 2>> gpurun_out/abl.err || exit 1
done; done; done
for w in ${WLS:-cfg2 cfg4}; do for r in 1 4; do
  AIRS_KB_ROT=$r AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=gpurun_out/ts/abl_${w}_r$r.bin timeout -k 10 120 python scripts/kbench.py $w > gpurun_out/ts/abl_${w}_r$r.log 2>&1 || exit 1
done; done
cat gpurun_out/abl.jsonl
