# ablation modes of exp/abl (warm, rot 1): compute-bound breakdown without HBM reads (512)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && : > gpurun_out/abl2.jsonl || exit 1
for w in cfg2 cfg4; do for m in ${MODES:-0 512 514 544 1536 33280 4608 2560 516}; do
  AIRS_LIB=exp/abl/libairscmp.so AIRS_DBG=$m AIRS_KB_ROT=1 timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/abl2.jsonl 2>> gpurun_out/abl2.err || exit 1
done; done
python3 -c "
import json
for l in open('gpurun_out/abl2.jsonl'):
    d=json.loads(l); print(d['workload'], 'dbg', d['dbg'], round(d['median_ms']*1e3,2), 'us')
"
