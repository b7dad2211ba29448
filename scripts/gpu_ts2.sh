# debug timelines (AIRS_DBG=65536) of exp variants, cfg2 warm
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ts && export TMPDIR=/tmp || exit 1
for v in ${VARIANTS}; do for w in ${WLS:-cfg2}; do
  AIRS_LIB=exp/$v/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=gpurun_out/ts/${v}_$w.bin AIRS_KB_ROT=${ROT:-1} timeout -k 10 120 python scripts/kbench.py $w > gpurun_out/ts/${v}_$w.log 2>&1 || exit 1
  cat gpurun_out/ts/${v}_$w.log
done; done
