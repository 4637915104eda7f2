"""Oracle restatement of the alternate intersectors (oracle/cpu_tracer.cpp: IntersectBruteForce,
RayMarch, DistancePointTri -- renderer.cpp:24-41, 138-197, triangle.h:163-198) against the
reference's own outputs (tests/golden/alt, oracle/gen_golden_alt.py via oracle/_ref/refdriver).
CPU only; sized to finish in well under a minute."""
import numpy as np
import pytest

from conftest import ALT_REC_DTYPE, ISECT, read_gz


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_alt_crops_cover_both_modes_and_all_scenes(golden_alt):
    modes = {(c["mode"], c["scene"]) for c in golden_alt["crops"]}
    assert all(("brute", s) in modes and ("march", s) in modes for s in range(10))


@pytest.mark.parametrize("i", range(26))
def test_oracle_alt_crop(oracle, golden_alt, i):
    c = golden_alt["crops"][i]
    exp = read_gz(f"alt/{c['name']}.rec.gz", ALT_REC_DTYPE)
    got = oracle.records(c["scene"], c["W"], c["H"], c["spp"], c["x0"], c["y0"], c["w"], c["h"],
                         tri_test=ISECT[c["mode"]] << 8)
    np.testing.assert_array_equal(got["hit"], exp["hit"])
    np.testing.assert_array_equal(got["tri"], exp["tri"])
    for k in ("t", "u", "v", "r", "g", "b"):
        np.testing.assert_array_equal(bits(got[k]), bits(exp[k]), err_msg=k)
    if c["mode"] == "march":
        np.testing.assert_array_equal(got["steps"], exp["steps"])


# frames small enough for the CPU suite (the GPU tests check every frame in alt.json)
CPU_FRAMES = {"brute_scene1_96x54x4", "brute_scene3_96x54x4", "brute_scene1_37x23x3", "brute_scene8_33x17x5",
              "march_scene1_48x27x1", "march_scene2_48x27x1", "march_scene3_48x27x1", "march_scene1_64x48x4",
              "march_scene3_31x19x2"}


@pytest.mark.parametrize("name", sorted(CPU_FRAMES))
def test_oracle_alt_frame(oracle, golden_alt, name):
    f = next(x for x in golden_alt["frames"] if x["name"] == name)
    img, hits, _ = oracle.render(f["scene"], f["W"], f["H"], f["spp"], tri_test=ISECT[f["mode"]] << 8,
                                 hits=True)
    np.testing.assert_array_equal(img.reshape(-1), read_gz(f"alt/{name}.bgra.gz", "<u4"))
    np.testing.assert_array_equal(hits, read_gz(f"alt/{name}.hits.gz", "<u4"))
