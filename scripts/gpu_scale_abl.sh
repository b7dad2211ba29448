# frames scaling under ablation modes (exp/r1abl built with -DAIRS_ABLATE=1)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/scale_abl.txt && \
for m in ${MODES:-0 32768 1024 512}; do for f in ${FRAMES:-1024 4096}; do \
  echo -n "mode $m frames $f: " >> gpurun_out/scale_abl.txt; \
  AIRS_LIB=exp/r1abl/libairscmp.so AIRS_DBG=$m AIRS_KB_FRAMES=$f timeout -k 10 120 python scripts/kbench.py cfg4 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(f'{d[\"median_ms\"]*1000:8.2f} us  {d[\"GBps\"]:7.1f} GB/s')" >> gpurun_out/scale_abl.txt || exit 1; \
done; done; cat gpurun_out/scale_abl.txt
