#!/usr/bin/env python3
"""Summarise rocprofv3 SQLite output (rocpd_*): per-kernel dispatch
durations and, when present, PMC counters summed per dispatch.

usage: rocpd_summary.py DB [DB ...] [--kernel SUBSTR]
"""
import sqlite3
import statistics
import sys
from collections import defaultdict


def summarise(db, ksub=None):
    con = sqlite3.connect(db)
    names = dict(con.execute("select id, kernel_name from rocpd_info_kernel_symbol"))
    rows = con.execute("select id, kernel_id, start, end, event_id, grid_size_x, workgroup_size_x "
                       "from rocpd_kernel_dispatch").fetchall()
    per = defaultdict(list)
    ev2k = {}
    for rid, kid, s, e, ev, gx, wx in rows:
        nm = names.get(kid, str(kid))
        if ksub and ksub not in nm:
            continue
        per[nm].append((e - s) / 1e3)
        ev2k[ev] = nm
    out = []
    for nm, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        out.append(dict(kernel=nm, calls=len(d), total_us=round(sum(d), 2), avg_us=round(statistics.mean(d), 3),
                        median_us=round(statistics.median(d), 3), min_us=round(min(d), 3)))
    pmc_names = dict(con.execute("select id, name from rocpd_info_pmc"))
    pmc = defaultdict(lambda: defaultdict(float))
    for ev, pid, val in con.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
        if ev in ev2k:
            pmc[ev][pmc_names.get(pid, str(pid))] += val
    counters = defaultdict(list)
    for ev, cs in pmc.items():
        for cn, v in cs.items():
            counters[(ev2k[ev], cn)].append(v)
    return out, {k: statistics.median(v) for k, v in counters.items()}


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    ks = None
    if "--kernel" in sys.argv:
        ks = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != ks]
    for db in args:
        kern, cnt = summarise(db, ks)
        print(f"== {db}")
        for k in kern:
            print(f"  {k['kernel'][:90]:90s} calls={k['calls']:5d} avg={k['avg_us']:9.3f}us "
                  f"median={k['median_us']:9.3f}us min={k['min_us']:9.3f}us total={k['total_us']:10.1f}us")
        for (kn, cn), v in sorted(cnt.items()):
            print(f"  [{kn[:50]}] {cn} = {v:.6g} (median per dispatch)")
