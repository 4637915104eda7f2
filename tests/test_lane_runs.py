"""AUTO's per-lane box runs (grid_intersect, RT_LANE_RUNS) on the CPU: the jump
to just below a box's exit (per-axis add chains up to a proven lower bound of the exit crossing)
replayed in the kernel's f32 arithmetic against the reference's cell-by-cell walk.  Every tested
cell, its crossing t and the last cell must agree exactly -- for every sample of the 1080p x 4
bench frames of all 10 scenes and for random rays with still, axis-aligned, tiny and near-axis
direction components.  tests/lane_run_check.cpp is the checker."""
import json
import os
import subprocess

import pytest

from conftest import ROOT

_EXE = {}


def _checker(tmp_path_factory):
    if "exe" not in _EXE:
        exe = str(tmp_path_factory.mktemp("lanerun") / "lane_run_check")
        subprocess.run(["g++", "-O2", "-std=c++11", "-pthread", "-ffp-contract=off", "-I", os.path.join(ROOT, "oracle"),
                        os.path.join(ROOT, "tests", "lane_run_check.cpp"), "-o", exe], check=True)
        _EXE["exe"] = exe
    return _EXE["exe"]


def _run(exe, *args):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out["mismatches"] == 0 and out["rays"] > 0 and out["tested_cells"] > 0, out
    return out


@pytest.mark.parametrize("sid", range(10))
def test_lane_runs_bench_frame(tmp_path_factory, sid):
    out = _run(_checker(tmp_path_factory), os.path.join(ROOT, "data", "scenes", f"scene{sid}.rtscene"), 1920, 1080, 4)
    # the bound is tight: after the add chains the box's exit is (almost always) the next step
    assert out["bare_steps_per_run"] < 1.01, out


@pytest.mark.parametrize("sid", [1, 5, 8])
def test_lane_runs_random_rays(tmp_path_factory, sid):
    _run(_checker(tmp_path_factory), os.path.join(ROOT, "data", "scenes", f"scene{sid}.rtscene"), "random", 1000000,
         sid + 11)


@pytest.mark.parametrize("sid", [1, 5, 8])
def test_lane_runs_any_lower_bound(tmp_path_factory, sid):
    """Time-synchronised runs take each lane's crossings below the WAVE's lowest bound: any T <= the
    lane's own bound must give the same walk (T drawn between the next crossing and the bound)."""
    exe = _checker(tmp_path_factory)
    _run(exe, os.path.join(ROOT, "data", "scenes", f"scene{sid}.rtscene"), 960, 540, 4, "shrink")
    _run(exe, os.path.join(ROOT, "data", "scenes", f"scene{sid}.rtscene"), "random", 500000, sid + 3, "shrink")
