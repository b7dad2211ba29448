#!/usr/bin/env python3
"""Per-sample issue / wait figures of the encode kernels from the two
rocprofv3 --pmc passes of scripts/gpu_pmc.sh.

usage: pmc_summary.py DIR        (DIR holds pmc_<workload>_{1,2}/p_results.db)

SQ_* wave counters count quad-cycles (MI355X_MICROARCH.md, s_memtime row);
WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES (disjoint).
"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import rocpd_summary  # noqa: E402

SAMPLES = {"cfg2": 64 << 20, "cfg2s": 64 << 20, "cfg3": 64 << 20, "cfg4": 64 << 20,
           "cfg5": 256 << 20, "cfg5fb": 256 << 20, "cfg5s8": 32 << 20, "cfg5fbs8": 32 << 20}


def main():
    d = sys.argv[1]
    out = {}
    for p1 in sorted(glob.glob(os.path.join(d, "pmc_*_1"))):
        wl = os.path.basename(p1)[4:-2]
        cnt = {}
        kern = {}
        for p in (p1, p1[:-1] + "2"):
            for db in glob.glob(os.path.join(p, "**", "*.db"), recursive=True):
                ks, c = rocpd_summary.summarise(db, "kernel")
                for k in ks:
                    kern.setdefault(k["kernel"], k)
                for (kn, cn), v in c.items():
                    cnt.setdefault(kn, {})[cn] = v
        res = {}
        for kn, c in cnt.items():
            # launches per step of this kernel: cfg5 runs 15 MODEL + 1 primary
            r = dict(c)
            wc = c.get("SQ_WAVE_CYCLES")
            if wc:
                for key in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                    if key in c:
                        r[key + "/WAVE_CYCLES"] = round(c[key] / wc, 3)
            ga = c.get("GRBM_GUI_ACTIVE")
            if ga:
                # SIMD-cycles = GUI_ACTIVE / 8 XCDs x 1024 SIMDs; SQ_* wave counters in quad-cycles
                simd_cycles = ga / 8.0 * 1024.0
                if "SQ_ACTIVE_INST_VALU" in c:
                    r["valu_busy"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / simd_cycles, 3)
                if wc:
                    r["resident_waves_per_simd"] = round(wc * 4 / simd_cycles, 3)
            kd = kern.get(kn)
            if kd:
                r["avg_us"] = kd["avg_us"]
                r["median_us"] = kd["median_us"]
            out.setdefault(wl, {})[kn[:80]] = r
        # per-sample figures for the dominant encode kernel (most VALU; the
        # bench's input synthesis is not part of the path)
        enc = {k: v for k, v in out.get(wl, {}).items()
               if "encode_kernel" in k or "rice_kernel" in k or "walk_kernel" in k or "walk_ctx_kernel" in k}
        dom = max(enc.items(), key=lambda kv: kv[1].get("SQ_INSTS_VALU", 0), default=None)
        if dom:
            kn, r = dom
            n = SAMPLES.get(wl)
            if wl.startswith("cfg5") and "encode_kernel" in kn:
                n = n // 16  # per-step launches: one acquisition of the streams
            per = {k: round(r[k] * 64 / n, 3) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                                          "SQ_INSTS_SMEM") if k in r}
            out[wl]["_per_sample_dominant"] = dict(kernel=kn, samples_per_launch=n,
                                                   lane_instructions_per_sample=per,
                                                   lds_bank_conflict_per_lds_inst=round(
                                                       r.get("SQ_LDS_BANK_CONFLICT", 0) /
                                                       max(1, r.get("SQ_INSTS_LDS", 1)), 3))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
