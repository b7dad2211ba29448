# pipelined-kernel timelines: exp/$V build with -DAIRS_PIPE_TS=1
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pts && export TMPDIR=/tmp && \
for w in ${WLS:-cfg2 cfg4}; do for r in ${ROTS:-1 4}; do \
  AIRS_LIB=exp/${V:-TS}/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=gpurun_out/pts/${w}_r$r.bin AIRS_KB_ROT=$r timeout -k 10 120 python scripts/kbench.py $w > gpurun_out/pts/${w}_r$r.json 2>> gpurun_out/pts/err.log || exit 1; \
done; done; ls -la gpurun_out/pts
