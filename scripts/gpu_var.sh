# kernel timings (kbench, HIP events) of exp variants: VARIANTS, WLS, ROTS
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/var.jsonl && \
for v in ${VARIANTS}; do for w in ${WLS:-cfg2 cfg4}; do for r in ${ROTS:-1 4}; do \
  AIRS_LIB=exp/$v/libairscmp.so AIRS_KB_ROT=$r timeout -k 10 120 python scripts/kbench.py $w > gpurun_out/kb.json 2>> gpurun_out/var.err || exit 1; \
  python3 -c "import json; d=json.load(open('gpurun_out/kb.json')); d['variant']='$v'; print(json.dumps(d))" >> gpurun_out/var.jsonl; \
done; done; done; python3 -c "
import json
for l in open('gpurun_out/var.jsonl'):
    d=json.loads(l); print(d['variant'], d['workload'], 'rot', d['rot'], 'us %.1f' % (d['median_ms']*1e3), d['GBps'], d['bitexact'])"
