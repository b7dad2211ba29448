cd "$GRAFT_REPO_ROOT" && MODES="0 2 32 512 514 1024 2048 4096 16384 32768" ROTS="4" bash scripts/gpu_ablate.sh r03_abl1 && \
for v in auto0 auto1 auto2; do AIRS_KB_ROT=4 AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 120 python scripts/kbench.py cfg3 >> gpurun_out/r03_abl1/auto.jsonl 2>>gpurun_out/r03_abl1/auto.err || exit 1; done; cat gpurun_out/r03_abl1/auto.jsonl
