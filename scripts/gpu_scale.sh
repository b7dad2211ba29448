# frames scaling probe (ramp-up / tail cost per launch): VARIANTS, FRAMES
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp && : > gpurun_out/scale.jsonl && \
for v in ${VARIANTS:-r1}; do for f in ${FRAMES:-256 512 1024 2048 4096}; do \
  echo "{\"variant\": \"$v\"}" >> gpurun_out/scale.jsonl; \
  AIRS_LIB=exp/$v/libairscmp.so AIRS_KB_FRAMES=$f timeout -k 10 120 python scripts/kbench.py cfg4 >> gpurun_out/scale.jsonl 2>> gpurun_out/scale.err || exit 1; \
done; done; python3 - <<'PY'
import json
v=None
for l in open("gpurun_out/scale.jsonl"):
    d=json.loads(l)
    if "variant" in d: v=d["variant"]; continue
    print(f'{v:6s} frames {d["frames"]:5d}  {d["median_ms"]*1000:8.2f} us  {d["GBps"]:7.1f} GB/s  per-frame {d["median_ms"]*1e6/d["frames"]:.1f} ns')
PY
