"""AUTO's box-run words (csrc/rt_box_words.h) on the CPU: for all 10 scenes and
all 24 copies (ray octant x major axis), every non-empty cell's word is its CSR range and every
empty cell's box -- the cells a walk may cross without a lookup -- holds no non-empty cell.  The
kernel's exactness rests on this: a box that covered a non-empty cell would skip its tests.
tests/box_words_check.cpp is the checker (grid from the oracle's Grid::Grid restatement)."""
import os
import subprocess

import pytest

from conftest import ROOT

_EXE = {}


def _checker(tmp_path_factory):
    if "exe" not in _EXE:
        exe = str(tmp_path_factory.mktemp("boxcheck") / "box_words_check")
        subprocess.run(["g++", "-O2", "-std=c++11", "-pthread", "-ffp-contract=off", "-I", os.path.join(ROOT, "oracle"),
                        os.path.join(ROOT, "tests", "box_words_check.cpp"), "-o", exe], check=True)
        _EXE["exe"] = exe
    return _EXE["exe"]


@pytest.mark.parametrize("sid", range(10))
def test_box_words_cover_only_empty_cells(tmp_path_factory, sid):
    exe = _checker(tmp_path_factory)
    r = subprocess.run([exe, os.path.join(ROOT, "data", "scenes", f"scene{sid}.rtscene")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    f = r.stdout.split()
    assert int(f[1]) > 0 and int(f[3]) > 0          # cells and empty cells checked
