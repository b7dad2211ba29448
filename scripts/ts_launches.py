"""Per-launch analysis of a ring of debug timelines (ablation build,
AIRS_DBG bit 65536 with AIRS_DBGTS_RING=R): R launches x segs x 8 stamps
(slots as scripts/ts_analyze.py: 0 start, 1 aggregate, 2 look-back done,
3 look-back start, 4 done, 5 rounds | spins << 32, 6 tail re-polls, 7 hw id).
Prints one line per launch (span, look-back waits, spins, dispatch skew) and
then contrasts fast and slow launches.
usage: ts_launches.py FILE RING SEGS_PER_FRAME [NSEGS]"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
R, spf = int(sys.argv[2]), int(sys.argv[3])
per = len(raw) // R
a_all = raw.reshape(R, per // 8, 8).astype(np.int64)
nseg = int(sys.argv[4]) if len(sys.argv) > 4 else None


def one(a):
    ok = a[:, 0] > 0
    a = a[ok] if nseg is None else a[:nseg]
    base = a[:, 0].min()
    t = np.where(a[:, :5] > 0, (a[:, :5] - base) / 100.0, np.nan)
    st, ag, lbd, lbs, end = (t[:, i] for i in range(5))
    xcc = a[:, 7] & 0xF
    hw = a[:, 7] >> 32
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    rounds = a[:, 5] & 0xFFFFFFFF
    spins = a[:, 5] >> 32
    light = not (a[:, 3] > 0).any()
    mhz = np.nan
    if light:  # slots 1 and 2: the shader clock at start and end
        dt = (a[:, 4] - a[:, 0]) / 100.0
        okc = (a[:, 2] > a[:, 1]) & (dt > 0)
        mhz = float(np.median((a[okc, 2] - a[okc, 1]) / dt[okc]))
        ag = lbs = lbd = np.full(len(a), np.nan)
    d = dict(span=np.nanmax(end), n=len(a), st=st, ag=ag, lbs=lbs, lbd=lbd, end=end, xcc=xcc, cu=cu, se=se,
             rounds=rounds, spins=spins, tail=a[:, 6], light=light, mhz=mhz)
    return d


L = [one(a_all[r]) for r in range(R) if (a_all[r][:, 0] > 0).any()]
spans = np.array([x["span"] for x in L])
print(f"launches {len(L)}  span min/median/max {spans.min():.1f}/{np.median(spans):.1f}/{spans.max():.1f} us")
light = L[0]["light"]
if light:
    print("  #  span  MHz  resid(med/p90)  spins>0  rounds>1  start p50/p90/max  xcd-end min-max")
    for i, x in enumerate(L):
        st, end = x["st"], x["end"]
        xe = [np.nanmax(end[x["xcc"] == c]) for c in range(8) if (x["xcc"] == c).any()]
        print(f"{i:3d} {x['span']:5.1f} {x['mhz']:5.0f}  {np.nanmedian(end - st):5.2f}/{np.nanpercentile(end - st, 90):5.2f}"
              f"   {np.mean(x['spins'] > 0) * 100:5.1f}%  {np.mean(x['rounds'] > 1) * 100:5.1f}%   "
              f"{np.nanmedian(st):5.1f}/{np.nanpercentile(st, 90):5.1f}/{np.nanmax(st):5.1f}   {min(xe):5.1f}-{max(xe):5.1f}")
hdr = ("  #  span  agg-st(med/p90)  LBwait(med/p90/max)  spins>0  rounds>1  tailrp>0  "
       "start p50/p90/max  xcd-end-spread  last-start")
print(hdr)
for i, x in enumerate([] if light else L):
    st, ag, lbs, lbd, end = x["st"], x["ag"], x["lbs"], x["lbd"], x["end"]
    lw = lbd - lbs
    xe = [np.nanmax(end[x["xcc"] == c]) for c in range(8) if (x["xcc"] == c).any()]
    print(f"{i:3d} {x['span']:5.1f}  {np.nanmedian(ag - st):5.2f}/{np.nanpercentile(ag - st, 90):5.2f}    "
          f"{np.nanmedian(lw):5.2f}/{np.nanpercentile(lw, 90):5.2f}/{np.nanmax(lw):6.2f}   "
          f"{np.mean(x['spins'] > 0) * 100:5.1f}%  {np.mean(x['rounds'] > 1) * 100:5.1f}%  "
          f"{np.mean(x['tail'] > 0) * 100:5.1f}%   {np.nanmedian(st):5.1f}/{np.nanpercentile(st, 90):5.1f}/"
          f"{np.nanmax(st):5.1f}   {min(xe):5.1f}-{max(xe):5.1f}   {np.nanmax(st):5.1f}")

# fast vs slow: split at 1.15 x the minimum span
thr = 1.15 * spans.min()
for name, sel in (("fast", spans <= thr), ("slow", spans > thr)):
    idx = np.nonzero(sel)[0]
    if not len(idx):
        continue
    print(f"\n== {name}: {len(idx)} launches (span <= / > {thr:.1f} us)")
    for i in idx[:3]:
        x = L[i]
        st, end, lbs, lbd = x["st"], x["end"], x["lbs"], x["lbd"]
        grid = np.arange(0, x["span"], 2.0)
        act = [int(((st <= g) & (end > g)).sum()) for g in grid]
        wait = [int(((lbs <= g) & (lbd > g)).sum()) for g in grid]
        print(f" launch {i} span {x['span']:.1f}: resident per 2us {act}")
        print(f"   in look-back wait per 2us {wait}")
        # per frame: time the frame's last segment ended
        nf = x["n"] // spf
        fe = [np.nanmax(end[f * spf:(f + 1) * spf]) for f in range(nf)]
        print(f"   frame end times {[round(v, 1) for v in fe]}")
        # per XCD end time
        print(f"   xcd end times {[round(float(np.nanmax(end[x['xcc'] == c])), 1) for c in range(8)]}")
        # spins by frame
        sp = [int(x['spins'][f * spf:(f + 1) * spf].sum()) for f in range(nf)]
        print(f"   spins per frame {sp}")
        # segments with the longest look-back wait
        lw = lbd - lbs
        top = np.argsort(-np.nan_to_num(lw))[:5]
        print("   longest LB waits (seg, frame, sif, wait, start, rounds, spins, xcc):",
              [(int(s), int(s // spf), int(s % spf), round(float(lw[s]), 2), round(float(st[s]), 1),
                int(x['rounds'][s]), int(x['spins'][s]), int(x['xcc'][s])) for s in top])
