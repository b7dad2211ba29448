# shader clock during the encode (debug timeline with s_memtime) at two sizes
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ts && export TMPDIR=/tmp && \
for f in ${FRAMES:-1024 4096}; do \
  AIRS_LIB=exp/r1abl/libairscmp.so AIRS_DBG=65536 AIRS_KB_FRAMES=$f AIRS_DBGTS_PATH=gpurun_out/ts/clk_$f.bin timeout -k 10 120 python scripts/kbench.py cfg4 > gpurun_out/ts/clk_$f.log 2>&1 || exit 1; \
done
