"""Where a walk batch differs from the call loop (developer diagnostic):
python3 scripts/walk_diag.py TRIAL [TRIAL ...] -> one JSON line per trial."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import conftest  # noqa: E402
import test_gpu_walk as t  # noqa: E402


def first_diff(a, b):
    if a is None or b is None:
        return None
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i
    return min(len(a), len(b)) if len(a) != len(b) else None


def compare(want, got):
    out = []
    for ci, ((fw, sw), (fg, sg)) in enumerate(zip(want, got)):
        for fi, ((rw, bw), (rg, bg)) in enumerate(zip(fw, fg)):
            if rw != rg or bw != bg:
                out.append({"call": ci, "frame": fi, "size_want": rw, "size_got": rg, "byte": first_diff(bw, bg)})
        for c, (a, b) in enumerate(zip(sw, sg)):
            if a != b:
                out.append({"call": ci, "ctx": c, "id": [a[0], b[0]], "seq": [a[1], b[1]], "msize": [a[2], b[2]],
                            "wbyte": first_diff(a[3], b[3])})
    return out[:12]


def main():
    pkg = conftest.load_pkg()
    prod = pkg.load()
    orc = pkg.CmpLib(conftest.ORC_PATH)
    eng = prod.engine()
    for tr in map(int, sys.argv[1:]):
        params, kind, n, nctx, calls, cap = t.make_case(tr)
        want = t.run_host(orc, params, kind, n, nctx, calls, cap)
        got = t.run_gpu(prod, eng, params, kind, n, nctx, calls, cap)
        step = t.run_gpu(prod, eng, params, kind, n, nctx, calls, cap, flags=t.api.GPU_STEPWISE)
        print(json.dumps({"trial": tr, "walk": compare(want, got), "stepwise": compare(want, step)}), flush=True)


if __name__ == "__main__":
    main()
