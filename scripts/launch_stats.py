"""Per-launch durations of one kernel from a rocprofv3 kernel-trace CSV:
count, min / p50 / p90 / max, launches above 1.10x and 1.20x the minimum,
and the sequence in launch order; --skip N leaves out the first N launches
(bench.py's untimed warmups) and --count C keeps C launches after them.
usage: launch_stats.py KERNEL_TRACE.csv KERNEL_SUBSTRING [--skip N] [--count C] [--json OUT]"""
import csv
import json
import sys

import numpy as np


def stats(path, ksub, skip=0, count=None):
    rows = [r for r in csv.DictReader(open(path)) if ksub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[skip:skip + count] if count else rows[skip:]
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in rows])
    if not len(d):
        raise SystemExit(f"{path}: no launches of {ksub}")
    mn = d.min()
    return dict(kernel=rows[0]["Kernel_Name"][:120], launches=len(d), min_us=round(mn, 2),
                p50_us=round(float(np.median(d)), 2), p90_us=round(float(np.percentile(d, 90)), 2),
                max_us=round(float(d.max()), 2), mean_us=round(float(d.mean()), 2),
                over_1p10_min=int((d > 1.10 * mn).sum()), over_1p20_min=int((d > 1.20 * mn).sum()),
                max_over_min=round(float(d.max() / mn), 3), sequence_us=[round(float(v), 1) for v in d])


if __name__ == "__main__":
    opt = {k: int(sys.argv[sys.argv.index(k) + 1]) for k in ("--skip", "--count") if k in sys.argv}
    s = stats(sys.argv[1], sys.argv[2], opt.get("--skip", 0), opt.get("--count"))
    s["skipped"] = opt.get("--skip", 0)
    print(json.dumps({k: v for k, v in s.items() if k != "sequence_us"}))
    print(" ".join(f"{v:.1f}" for v in s["sequence_us"]))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(s, f, indent=1)
