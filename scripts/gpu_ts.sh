# debug timelines of exp variants built with -DAIRS_ABLATE=1 (AIRS_DBG=65536)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ts && export TMPDIR=/tmp && \
for v in ${VARIANTS:-r1abl leanabl}; do for w in ${WLS:-cfg2}; do \
  AIRS_LIB=exp/$v/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=gpurun_out/ts/${v}_$w.bin timeout -k 10 120 python scripts/kbench.py $w > gpurun_out/ts/${v}_$w.log 2>&1 || exit 1; \
done; done
