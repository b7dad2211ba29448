# fused auto-Rice ablations (cold) and timelines: exp/autoa1 (no histogram atomics), exp/autoa2 (no frame wait), exp/autots (stamps)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ts && export TMPDIR=/tmp && : > gpurun_out/aabl.jsonl || exit 1
for v in autoa1 autoa2 autots; do for r in 1 4; do
  echo "{\"variant\": \"$v\"}" >> gpurun_out/aabl.jsonl
  AIRS_KB_ROT=$r AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 120 python scripts/kbench.py cfg3 >> gpurun_out/aabl.jsonl 2>> gpurun_out/aabl.err || exit 1
done; done
AIRS_KB_ROT=4 AIRS_LIB=exp/autots/libairscmp.so AIRS_DBG=65536 AIRS_DBGTS_PATH=gpurun_out/ts/auto_cfg3.bin timeout -k 10 120 python scripts/kbench.py cfg3 > gpurun_out/ts/auto_cfg3.log 2>&1 || exit 1
cat gpurun_out/aabl.jsonl
