# A/B of exp/base vs exp/<variant> (cold rotated inputs and warm), twice interleaved
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/slb.jsonl || exit 1
for rep in 1 2; do for w in ${WLS:-cfg2 cfg4}; do for r in 4 1; do for v in ${VARIANTS:-base slb}; do
  echo "{\"variant\": \"$v\", \"rot\": $r}" >> gpurun_out/slb.jsonl
  AIRS_KB_ROT=$r AIRS_LIB=exp/$v/libairscmp.so timeout -k 10 120 python scripts/kbench.py $w >> gpurun_out/slb.jsonl 2>> gpurun_out/slb.err || exit 1
done; done; done; done
python3 - <<'PY'
import json
v=None
for l in open("gpurun_out/slb.jsonl"):
    d=json.loads(l)
    if "variant" in d: v=(d["variant"], d["rot"]); continue
    print(f"{v[0]:6s} rot={v[1]} {d['workload']} {d['median_ms']*1000:7.1f} us bitexact={d['bitexact']}")
PY
