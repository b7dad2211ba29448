"""Register and spill budgets of the hot kernels, read from the built
library's code-object metadata (tests/kernel_meta.py; no GPU).

ADVICE r3: the encode kernel's speed depends on how the compiler allocates
its registers (a 20 % swing came from one kernel-argument field, DESIGN.md
5.2); a toolchain or source change that adds spills, or more VGPRs than the
occupancy the kernel is designed for, must fail here rather than show up as
a slower bench.  Budgets are today's counts; the VGPR ceilings are the
occupancy steps (MI355X_MICROARCH.md: <= 96 VGPRs -> 5 waves per SIMD,
<= 128 -> 4)."""
import os

import pytest

import kernel_meta
from conftest import PKG_DIR

LIB = os.path.join(PKG_DIR, "lib", "libairscmp.so")

# symbol: (max VGPRs, max SGPR spills to VGPR lanes); VGPR spills must be 0
BUDGETS = {
    # cfg2 / cfg4: the Rice/ZERO frame kernel (enc_rice.hip), DIFF and NONE:
    # six workgroups per CU since round 6: <= 85 VGPRs (65 with the pair
    # table of round 6)
    # (round 6: the scalar look-back of XCD-local frames, rice_lookback_s,
    # holds a 16-granule window in 32 SGPRs: 19 spills to VGPR lanes, all in
    # wave 0's look-back, once per segment)
    "_ZN4airs11rice_kernelILi1ELb0ELb0EEEvNS_5KArgsE": (85, 24),
    "_ZN4airs11rice_kernelILi0ELb0ELb0EEEvNS_5KArgsE": (85, 24),
    "_ZN4airs11rice_kernelILi1ELb1ELb0EEEvNS_5KArgsE": (85, 0),
    # cfg3: the Rice kernel with the frame's k chosen in it (AUTO; round 6):
    # the 64 mapped samples stay in registers across the candidate barrier;
    # five workgroups per CU: <= 96 VGPRs (62 since the barrier's granules
    # are polled one per lane at a time)
    "_ZN4airs11rice_kernelILi1ELb0ELb1EEEvNS_5KArgsE": (96, 0),
    "_ZN4airs11rice_kernelILi0ELb0ELb1EEEvNS_5KArgsE": (96, 0),
    # encode_kernel<2, DIFF, ZERO, Rice, no model, FULL>: frames the Rice
    # kernel does not take (k > 7, holes in device-planned launch lists); no
    # longer a bench path, so the kernel-argument padding that kept it at 13
    # spills went (round 5: the Rice kernels went from 8 spills to 0)
    "_ZN4airs13encode_kernelILi2ELi1ELi1ELb1ELi0ELb1ELb0ELb0EEEvNS_5KArgsE": (128, 40),
    # cfg3: encode_kernel's fused per-frame Rice selection
    "_ZN4airs13encode_kernelILi2ELi1ELi1ELb1ELi0ELb1ELb1ELb0EEEvNS_5KArgsE": (128, 0),
    # cfg2s: payload-only stream
    "_ZN4airs13encode_kernelILi2ELi1ELi1ELb1ELi0ELb1ELb0ELb1EEEvNS_5KArgsE": (128, 0),
    # cfg5 / cfg5fb: the context walk (1024-thread workgroups: <= 128 VGPRs)
    "_ZN4airs15walk_ctx_kernelILi4ELi1ELi1ELb1ELi2ELb1ELi4EEEvNS_5WArgsE": (128, 74),
    # the segment walk, 16 samples per lane and 8 (cfg5s8: grids of fewer than 1024 4096-sample workgroups)
    "_ZN4airs11walk_kernelILi4ELi1ELi1ELb1ELi2ELb1ELi16EEEvNS_5WArgsE": (112, 28),
    "_ZN4airs11walk_kernelILi4ELi1ELi1ELb1ELi2ELb1ELi8EEEvNS_5WArgsE": (80, 26),
}


@pytest.fixture(scope="module")
def meta():
    if not os.path.exists(LIB):
        pytest.skip("libairscmp.so not built")
    return kernel_meta.kernels(LIB)


@pytest.mark.parametrize("sym", sorted(BUDGETS))
def test_hot_kernel_register_budget(meta, sym):
    assert sym in meta, f"{sym} not in the library"
    k = meta[sym]
    vmax, smax = BUDGETS[sym]
    assert k[".vgpr_spill_count"] == 0, (sym, k[".vgpr_spill_count"])
    assert k.get(".private_segment_fixed_size", 0) == 0, sym  # no scratch
    assert k[".vgpr_count"] <= vmax, (sym, k[".vgpr_count"], vmax)
    assert k[".sgpr_spill_count"] <= smax, (sym, k[".sgpr_spill_count"], smax)


def test_every_kernel_is_gfx950_and_listed(meta):
    names = set(meta)
    for stem in ("rice_kernel", "encode_kernel", "walk_ctx_kernel", "walk_kernel", "ck_chain_kernel",
                 "select_rice_hist_kernel", "fb_step_kernel", "dec_parse_kernel"):
        assert any(stem in n for n in names), stem
