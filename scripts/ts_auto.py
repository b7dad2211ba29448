"""Per-phase medians of the AUTO Rice kernel's per-segment timeline (cfg3;
ablation build, AIRS_DBG 65536, scripts/gpu.sh ts step): slots 0 start,
5 candidates published, 6 the frame's candidates seen (k known), 1 aggregate
(phase 1 and the scan done), 3 / 2 tail wait start / end, 4 done.
usage: ts_auto.py FILE RING"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
R = int(sys.argv[2])
a_all = raw.reshape(R, -1, 8).astype(np.int64)
names = [("start->published", 0, 5), ("frame barrier", 5, 6), ("k->aggregate", 6, 1), ("packing", 1, 3),
         ("tail wait", 3, 2), ("store+exit", 2, 4), ("resident", 0, 4)]
rows = []
for r in range(R):
    a = a_all[r]
    a = a[a[:, 0] > 0]
    if not len(a):
        continue
    base = a[:, 0].min()
    span = (a[:, 4].max() - base) / 100.0
    d = {n: np.median((a[:, j] - a[:, i]) / 100.0) for n, i, j in names}
    d90 = {n: np.percentile((a[:, j] - a[:, i]) / 100.0, 90) for n, i, j in names}
    rows.append((span, d, d90, (a[:, 0].max() - base) / 100.0))
spans = np.array([x[0] for x in rows])
print(f"launches {len(rows)}  span min/median/max {spans.min():.1f}/{np.median(spans):.1f}/{spans.max():.1f} us")
print("median over launches of the per-segment median (p90) us:")
for n, _, _ in names:
    print(f"  {n:18s} {np.median([x[1][n] for x in rows]):6.2f} ({np.median([x[2][n] for x in rows]):6.2f})")
print(f"  last start          {np.median([x[3] for x in rows]):6.2f}")
