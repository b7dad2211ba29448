"""Summarise gpurun_out/exp.jsonl (written by scripts/gpu_exp.sh): variant workload median/min us."""
import json, sys
v = None
for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/exp.jsonl"):
    d = json.loads(l)
    if "variant" in d:
        v = d["variant"]; continue
    print(f'{v:8s} {d["workload"]:6s} dbg={d["dbg"]:>6s} median {d["median_ms"]*1000:7.2f} us  min {d["min_ms"]*1000:7.2f} us  exact={d.get("bitexact")}')
