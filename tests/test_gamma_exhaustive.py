"""Hazard H6: glibc powf(x, .5f) (reference gamma) vs sqrtf (HIP kernel), exhaustively.

oracle/gamma_exhaustive.c walks every float in [0, 1.0078]; the packed BGRA8 byte must never
differ.  The float colour differs by 1 ulp on ~678k inputs, inside the north_star's 1e-5
relative tolerance for float shading.
"""
import os
import subprocess

from conftest import ROOT


def test_sqrt_gamma_packs_like_powf(tmp_path):
    exe = str(tmp_path / "gamma_exhaustive")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off",
                    os.path.join(ROOT, "oracle", "gamma_exhaustive.c"), "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=600).stdout.split()
    float_diffs, byte_diffs = int(out[1]), int(out[3])
    assert byte_diffs == 0
    assert float_diffs < 1_000_000       # 1-ulp differences only (see oracle/gamma_exhaustive.c)
