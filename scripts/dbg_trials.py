"""Debug: run random-sequence trials on the GPU library and the oracle, print per-frame diffs.
usage: python scripts/dbg_trials.py 82 141"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import scenarios
from conftest import load_pkg, ORC_PATH
pkg = load_pkg()
api = pkg.cmpapi
gpu = pkg.load()
orc = pkg.CmpLib(ORC_PATH)
for t in map(int, sys.argv[1:]):
    params, kind, n = scenarios.random_case(api.CmpParams, t, allow_iwt=True)
    a = scenarios.run_sequence(gpu, params, kind, n, seed=t)
    b = scenarios.run_sequence(orc, params, kind, n, seed=t)
    print("trial", t, kind, n)
    for i, (x, y) in enumerate(zip(a, b)):
        if x == y:
            print("  frame", i, "same")
            continue
        if i == 0:
            print("  init", x, y); continue
        print("  frame", i, "r", x[0], y[0], "id", x[2], y[2], "seq", x[3], y[3])
        if x[1] is not None and y[1] is not None:
            d = [j for j in range(min(len(x[1]), len(y[1]))) if x[1][j] != y[1][j]]
            print("    ndiff", len(d), "first", d[:8], "len", len(x[1]), len(y[1]))
            if d:
                j = d[0]; print("    gpu", x[1][j-4:j+8].hex(), "orc", y[1][j-4:j+8].hex())
        if x[5] != y[5]:
            print("    work buf differs")
