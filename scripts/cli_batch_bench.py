#!/usr/bin/env python3
"""CLI file throughput for parameter sets with a work buffer: N files of n
u16 samples (big-endian, a smooth synthetic signal) compressed by one
`airspace -c ... --stdout` call, with the round-5 CLI (files batched on the
GPU, the work buffer on the device) and with the CLI before it (one host-API
call per file, exp/oldcli).  Wall clock of the whole process, median of 3.
Prints one JSON line.  usage: cli_batch_bench.py [N] [n]"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
SETS = {
    "model_chain": "primary_preprocessing=DIFF,primary_encoder_type=GOLOMB_ZERO,primary_encoder_param=16,"
                   "secondary_iterations=3,secondary_preprocessing=MODEL,secondary_encoder_type=GOLOMB_ZERO,"
                   "secondary_encoder_param=8,model_rate=11",
    "iwt": "primary_preprocessing=IWT,primary_encoder_type=GOLOMB_ZERO,primary_encoder_param=16",
}
rng = np.random.default_rng(1)
d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
t = np.arange(n)
paths = []
for i in range(N):
    x = (30000 + 8000 * np.sin(t / 300.0 + i * 0.01) + rng.integers(-30, 30, n)).astype(np.uint16)
    p = os.path.join(d, f"f{i:04d}.dat")
    with open(p, "wb") as f:
        f.write(x.astype(">u2").tobytes())
    paths.append(p)
out = {"files": N, "samples_per_file": n}
for name, par in SETS.items():
    outs = {}
    for tool in ("new", "old"):
        exe = os.path.join(ROOT, "airs-compression_amd/bin/airspace" if tool == "new" else "exp/oldcli/bin/airspace")
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = subprocess.run([exe, "-c", "--params", par, "--stdout", "-q"] + paths, capture_output=True)
            ts.append(time.perf_counter() - t0)
            assert r.returncode == 0, r.stderr[-2000:]
        outs[tool] = r.stdout
        out[f"{name}_{tool}_s"] = round(sorted(ts)[1], 3)
    # identifiers (bytes 8..13 of each frame) come from the clock: compare the rest
    a, b = bytearray(outs["new"]), bytearray(outs["old"])
    same = len(a) == len(b)
    pos = 0
    while same and pos < len(a):
        size = int.from_bytes(a[pos + 2:pos + 5], "big")
        same = a[pos:pos + 8] == b[pos:pos + 8] and a[pos + 14:pos + size] == b[pos + 14:pos + size]
        pos += size
    out[f"{name}_same_frames"] = same
print(json.dumps(out))
