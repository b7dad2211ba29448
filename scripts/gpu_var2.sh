# kernel variants (exp/<v>), cold (rot 4) and warm (rot 1), cfg2 and cfg4
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/var2.jsonl || exit 1
for v in ${VARIANTS}; do for w in ${WLS:-cfg2 cfg4}; do for r in 4 1; do
  echo "{\"variant\": \"$v\"}" >> gpurun_out/var2.jsonl
  if [ "$v" = base ]; then L=airs-compression_amd/lib/libairscmp.so; else L=exp/$v/libairscmp.so; fi
  AIRS_LIB=$L AIRS_KB_ROT=$r timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/var2.jsonl 2>> gpurun_out/var2.err || exit 1
done; done; done
python3 - <<'PY'
import json
v=None
for l in open('gpurun_out/var2.jsonl'):
    d=json.loads(l)
    if 'variant' in d: v=d['variant']; continue
    print(f"{v:8s} {d['workload']} rot{d['rot']} {d['median_ms']*1e3:7.2f} us  bitexact={d['bitexact']}")
PY
