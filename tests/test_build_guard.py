"""Build-level guards for the HIP kernels (CPU-only; needs hipcc, which this image has).

* Hazard H1/H2: the device IR must contain no FMA contraction (llvm.fmuladd,
  `contract`) and no fast-math flags (afn/arcp/nnan/ninf/nsz/reassoc) -- the bit-exact
  parity of every float on the path depends on it.
* The traversal kernels must not spill or put walk state in LDS/scratch (a pointer-select
  over struct fields once did exactly that and cost 14%).
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import PKG_DIR

SRC = os.path.join(PKG_DIR, "csrc", "rt_kernels.hip")
WALK = os.path.join(PKG_DIR, "csrc", "rt_walk.h")
GRID_SRC = os.path.join(PKG_DIR, "csrc", "rt_grid_build.hip")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
         "--cuda-device-only"]
pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


@pytest.mark.parametrize("src", [SRC, GRID_SRC], ids=["tracer", "grid_build"])
def test_device_ir_has_no_contraction_or_fast_math(tmp_path, src):
    """Covers the fp64 tri/box SAT of the grid build too (aabb_tri_internal.h is exact only
    without contraction)."""
    ll = tmp_path / "rt.ll"
    subprocess.run([HIPCC] + FLAGS + ["-emit-llvm", "-S", "-o", str(ll), src], check=True,
                   capture_output=True)
    ir = ll.read_text()
    assert "fmuladd" not in ir
    # explicit FMAs are allowed only in rtd::rcp_nr (the Newton step of the exhaustively
    # checked reciprocal) and box_exit_bound (a walk bound compared against crossing times, never a
    # pixel's arithmetic; tests/test_lane_runs.py); any other llvm.fma would be a contraction in
    # disguise
    assert not re.search(r"\bllvm\.fma\.f64\b", ir)
    for f in (SRC, WALK, GRID_SRC, os.path.join(PKG_DIR, "csrc", "rt_device.h")):
        text = open(f).read().splitlines()
        lines = [l for l in text if re.search(r"\bfmaf?\b|__builtin_fma", l)]
        assert all("__builtin_fmaf(" in l for l in lines), lines
        assert len(lines) == (0 if f in (SRC, GRID_SRC) else 2), (f, lines)
        if f == WALK:
            i = next(j for j, l in enumerate(text) if "float box_exit_bound(" in l)
            assert all(l in text[i:i + 5] for l in lines), lines
    for flag in (" contract ", " afn ", " arcp ", " nnan ", " ninf ", " nsz ", " reassoc ", " fast "):
        assert flag not in ir, flag
    assert "denormal-fp-math-f32" not in ir or '"denormal-fp-math-f32"="ieee' in ir


def test_render_kernels_do_not_spill(tmp_path):
    out = subprocess.run([HIPCC] + FLAGS + ["-c", "-o", str(tmp_path / "rt.o"), SRC,
                          "-Rpass-analysis=kernel-resource-usage"], check=True, capture_output=True,
                         text=True).stderr
    names = re.findall(r"Function Name: (\S+)", out)
    sgprs = [int(x) for x in re.findall(r"SGPRs: (\d+)", out)]
    scratch = [int(x) for x in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", out)]
    vgprs = [int(x) for x in re.findall(r"VGPRs: (\d+)", out)]
    occ = [int(x) for x in re.findall(r"Occupancy \[waves/SIMD\]: (\d+)", out)]
    assert len(names) == len(scratch) == len(vgprs) == len(occ)
    table = dict(zip(names, zip(scratch, vgprs, occ)))
    render = {n: v for n, v in table.items() if "k_render_" in n}
    assert render, table
    for n, (sc, vg, oc) in render.items():
        assert sc == 0, f"{n} spills {sc} B/lane"
    # the AUTO kernel (kVarAuto = 80398: lanes + wave gate + distance skip + origin terms + Newton
    # reciprocal + packed counts + uniform cells + empty runs + XCD rows), its fallbacks for scenes
    # outside the reciprocal / packing ranges, and its arms keep 8 waves/SIMD
    # Also every kernel bench.py dispatches: the one-wave-workgroup AUTO kernels (k_render_lanes_w64,
    # the N = 1 bench step; k_render_batch_w64, the batched step at 1, 2 and >= 8 ranks, with the wide
    # section fused in front: kVarWideHeavy 524288, kVarWideFused 1048576, kVarWideG4 2097152), the
    # 256-lane batch kernels (a rank of 3-7) and the wide-section kernels
    for key in ("k_render_lanesILi0ELi80398E", "k_render_lanesILi0ELi78350E", "k_render_lanesILi0ELi76298E",
                "k_render_lanesILi0ELi74250E", "k_render_lanesILi0ELi604686E", "k_render_lanesILi0ELi0E",
                "k_render_compact", "k_render_lanes_w64ILi0ELi80398E", "k_render_batch_w64ILi0ELi80398E",
                "k_render_batch_w64ILi0ELi1653262E",
                "k_render_batch_w64ILi0ELi3750414E", "k_render_batchILi0ELi80398E", 
                "k_render_whILj16E", "k_render_whILj4E"):
        arm = [v for n, v in render.items() if key in n]
        assert arm and all(a[2] == 8 for a in arm), (key, arm)
    # the 256-lane batch kernels with the wide section fused in (a rank of 3-7): their 84-91 SGPRs
    # already allow 7 waves/SIMD (800 / (96 + 16)), so up to 72 VGPRs cost nothing more
    for key in ("k_render_batchILi0ELi1653262E", "k_render_batchILi0ELi3750414E"):
        arm = [v for n, v in render.items() if key in n]
        assert arm and all(a[2] >= 7 and a[1] <= 72 for a in arm), (key, arm)
    # the bench's own kernels are pinned by name (a renamed kernel must update this guard)
    dispatched = ("k_render_lanes_w64", "k_render_batch_w64", "k_render_batch")
    assert all(any(d + "I" in n for n in render) for d in dispatched), sorted(render)
    # ... and at 8 waves per SIMD by the HARDWARE's admission rule, floor(800 / (ceil(sgpr / 16) * 16 +
    # 16)) (MI355X_MICROARCH.md, residency: 82-96 SGPRs admit 7 although the compiler's estimate says
    # 8): the one-rank kernels and the fused kernels of N >= 2 (k_render_batch_w64_o8)
    hw = {n: min(table[n][2], 800 // (-(-sg // 16) * 16 + 16)) for n, sg in zip(names, sgprs)}
    for key in ("k_render_lanes_w64ILi0ELi80398E", "k_render_batch_w64ILi0ELi80398E",
                "k_render_batch_w64_o8ILi0ELi1653262E", "k_render_batch_w64_o8ILi0ELi3750414E"):
        arm = [hw[n] for n in names if key in n]
        assert arm and all(a == 8 for a in arm), (key, arm)
