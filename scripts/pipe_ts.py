"""Per-phase durations of the pipelined encode kernel from a timeline dump
(-DAIRS_PIPE_TS=1 build, AIRS_DBG=65536, AIRS_DBGTS_PATH=FILE): slots
0 iteration start, 1 packed, 2 next phase 1 done, 3 look-back done,
4 stored, 5 cleared, 7 workgroup | xcc << 32.  Times in us.
usage: pipe_ts.py FILE"""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.int64)
ok = a[:, 0] > 0
a = a[ok]
base = a[:, 0].min()
t = np.where(a[:, :6] > 0, (a[:, :6] - base) / 100.0, np.nan)
R = lambda x: f"{np.nanmedian(x):6.2f}/{np.nanpercentile(x, 90):6.2f}/{np.nanmax(x):6.2f}"  # noqa: E731
print(f"segments {len(a)}  span {np.nanmax(t):.1f} us  (median/p90/max us)")
names = ["pack", "phase1(next)", "look-back", "store", "clear"]
for i, nm in enumerate(names):
    print(f"  {nm:14s} {R(t[:, i + 1] - t[:, i])}")
wg = a[:, 7] & 0xFFFFFFFF
order = np.lexsort((t[:, 0], wg))
tw, ww = t[order], wg[order]
same = ww[1:] == ww[:-1]
gap = tw[1:, 0] - tw[:-1, 4]
print(f"  iteration (start->next start) {R((tw[1:, 0] - tw[:-1, 0])[same])}")
print(f"  first start {np.nanmin(t[:, 0]):.2f}  last start {np.nanmax(t[:, 0]):.2f}  last end {np.nanmax(t[:, 4]):.2f}")
for g in sorted(set(ww))[:3]:
    s = tw[ww == g]
    print(f"  wg {g}: starts", np.round(s[:, 0], 1).tolist())
pl = a[:, 6] & 0xFFFFFFFF
tp = a[:, 6] >> 32
print(f"  look-back re-polls: mean {pl.mean():.2f} (>0 in {np.mean(pl > 0) * 100:.1f}%)  tail re-polls: mean {tp.mean():.2f} (>0 in {np.mean(tp > 0) * 100:.1f}%)")
lb = t[:, 3] - t[:, 2]
for k in (0, 1, 2):
    m = pl == k
    if m.any():
        print(f"   polls={k}: {m.sum()} segs, LB {R(lb[m])}")
