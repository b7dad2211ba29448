"""print gpurun_out/exp.jsonl as a table: variant workload us GB/s bitexact"""
import json
v = None
for line in open("gpurun_out/exp.jsonl"):
    d = json.loads(line)
    if "variant" in d:
        v = d["variant"]
        continue
    print(f"{v:8s} {d['workload']} {d['median_ms'] * 1000:7.1f} us {d['GBps']:8.1f} GB/s  bitexact={d['bitexact']}")
