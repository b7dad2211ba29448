"""Analyse a per-segment debug timeline (AIRS_DBG bit 65536 dump of an
ablation build): slots 0 start, 1 aggregate published, 2 look-back done,
3 look-back start, 4 segment done (wave 0), 5 look-back rounds | retries
<< 32, 6 tail re-polls, 7 hw id.  Times in us (realtime clock, 100 MHz).
usage: ts_analyze.py FILE SEGS_PER_FRAME"""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.int64)
spf = int(sys.argv[2])
nf = len(a) // spf
ok = a[:, 0] > 0
base = a[ok, 0].min()
t = np.where(a[:, :5] > 0, (a[:, :5] - base) / 100.0, np.nan)
st, ag, lbd, lbs, end = (t[:, i] for i in range(5))
R = lambda x: f"{np.nanmedian(x):6.2f}/{np.nanpercentile(x, 90):6.2f}"  # noqa: E731
print(f"segments {len(a)} frames {nf} kernel span {np.nanmax(end):.1f} us  (median/p90 us)")
print(f" start->agg {R(ag - st)}  start->LBstart {R(lbs - st)}  LB wait {R(lbd - lbs)}  "
      f"LBdone->end {R(end - lbd)}  residency {R(end - st)}")
T = lambda x: x.reshape(nf, spf)  # noqa: E731
ag2, lbs2, lbd2, st2 = T(ag), T(lbs), T(lbd), T(st)
print(f" pred agg later than succ LB start: {np.nanmean(ag2[:, :-1] > lbs2[:, 1:]) * 100:.1f}%   "
      f"pred LB done later than succ LB start: {np.nanmean(lbd2[:, :-1] > lbs2[:, 1:]) * 100:.1f}%")
# occupancy over time
grid = np.arange(0, np.nanmax(end), 1.0)
act = [int(((st <= g) & (end > g)).sum()) for g in grid]
wait = [int(((lbs <= g) & (lbd > g)).sum()) for g in grid]
step = max(1, len(grid) // 25)
print(" resident per us:", act[::step])
print(" in LB wait per us:", wait[::step])
nf_ = a[:, 5] & 0xFFFFFFFF
rt = a[:, 5] >> 32
m = lbs >= 0
print(f" LB rounds: mean {nf_[m].mean():.2f} max {nf_[m].max()}  retries: mean {rt[m].mean():.2f}  "
      f"tail re-polls: mean {a[m, 6].mean():.2f} (>0 in {np.mean(a[m, 6] > 0) * 100:.1f}%)")
for r in (1, 2, 3):
    sel = m & (nf_ == r)
    if sel.any():
        print(f"  rounds={r}: {sel.sum()} segs, LB wait {R(lbd[sel] - lbs[sel])}")
sel = m & (nf_ == 1) & (a[:, 6] == 0)
if sel.any():
    print(f"  1 round, no tail re-poll: {sel.sum()} segs, LB wait {R(lbd[sel] - lbs[sel])}")
