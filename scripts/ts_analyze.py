"""Analyse a per-segment debug timeline (AIRS_DBG bit 65536 dump): slots
0 start, 1 aggregate published, 2 look-back done (3-6: optional extra stamps
of experimental kernels: look-back start, tail obtained, stored, own tail
published), 7 hw id.
usage: ts_analyze.py FILE SEGS_PER_FRAME"""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8)
spf = int(sys.argv[2])
nf = len(a) // spf
t = a[:, :7].astype(np.int64)
base = t[:, 0][t[:, 0] > 0].min()
t = np.where(t > 0, t - base, -1)
st, ag, lbd, lbs, tl, sd, tp = (t[:, i] for i in range(7))
R = lambda x: f"{np.median(x) / 100:.2f}/{np.percentile(x, 90) / 100:.2f}"  # noqa: E731
m = lbs >= 0
print(f"segments {len(a)} frames {nf} span {st.max() / 100:.1f} us; (median/p90, us after start)")
print(f" agg {R(ag - st)}  own tail pub {R(tp[tp >= 0] - st[tp >= 0])}  LB start {R(lbs[m] - st[m])}  "
      f"LB done {R(lbd[m] - st[m])}  tail got {R(tl[m] - st[m])}  stored {R(sd - st)}")
print(f" LB duration {R(lbd[m] - lbs[m])}  tail wait {R(tl[m] - lbd[m])}")
T = lambda x: x.reshape(nf, spf)  # noqa: E731
ag2, lbs2, lbd2, tp2, st2 = T(ag), T(lbs), T(lbd), T(tp), T(st)
print(f" pred agg after succ LB start: {np.mean(ag2[:, :-1] > lbs2[:, 1:]) * 100:.1f}%   "
      f"pred tail after succ LB done: {np.mean(tp2[:, :-1] > lbd2[:, 1:]) * 100:.1f}%   "
      f"pred started after succ: {np.mean(st2[:, :-1] > st2[:, 1:]) * 100:.1f}%")
d = lbd2[:, 1:] - lbd2[:, :-1]
print(f" succ LB done - pred LB done: {R(d)}")
# shader clock: slots 5/6 = s_memtime at start / look-back done (encode_kernel)
c0, c1 = a[:, 5].astype(np.int64), a[:, 6].astype(np.int64)
ok = (c0 > 0) & (c1 > c0) & (t[:, 2] > t[:, 0])
if ok.any():
    f = (c1 - c0)[ok] / ((t[:, 2] - t[:, 0])[ok] / 100.0)  # cycles per us
    print(f" shader clock (s_memtime / realtime): median {np.median(f) / 1e3:.3f} GHz  p10 {np.percentile(f, 10) / 1e3:.3f}  p90 {np.percentile(f, 90) / 1e3:.3f}")
